// Microbenchmark (diagnostics, not product code): per-CU feed rate from an
// L2-resident buffer (a 1 MiB "weight" tensor every CU re-reads, as the encoder
// GEMMs re-read their weights) by
//   mode 0: global_load_dwordx4 into registers, 1 KiB contiguous per wave-instruction
//   mode 1: global_load_lds_dwordx4 (LDS-DMA) into a 32 KiB LDS ring, same pattern
//   mode 2: global_load_dwordx4 fragment-shaped: 16 rows x 64 B per instruction
//           from a [rows][K] bf16 layout with 1 KiB rows (an MFMA B fragment)
//   mode 3: LDS-DMA, 16 rows x 64 B per instruction (the encoder GEMMs' BK = 32 tiles)
//   mode 4: LDS-DMA, 8 rows x 128 B per instruction (BK = 64: whole cache lines)
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/l2feed tools/exp/l2feed.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

constexpr int BUF = 1 << 20;  // bytes

template <int MODE>
__global__ void __launch_bounds__(256) feed(const uint4* __restrict__ buf, int iters, uint4* out) {
  __shared__ uint4 ring[2048];  // 32 KiB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nchunk = BUF / 1024;  // 1 KiB chunks
  int c = (blockIdx.x * 4 + wave) * 37 % nchunk;
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (MODE == 0) {
    for (int it = 0; it < iters; it += 8) {
      uint4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = buf[((c + q) % nchunk) * 64 + lane];
#pragma unroll
      for (int q = 0; q < 8; ++q) { acc.x ^= v[q].x; acc.y ^= v[q].y; acc.z ^= v[q].z; acc.w ^= v[q].w; }
      c = (c + 8) % nchunk;
    }
  } else if (MODE == 1) {
    for (int it = 0; it < iters; it += 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        __builtin_amdgcn_global_load_lds(GPTR(buf + ((c + q) % nchunk) * 64 + lane),
                                         LPTR(ring + (wave * 8 + q) * 64), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      c = (c + 8) % nchunk;
    }
    __syncthreads();
    acc = ring[threadIdx.x];
  } else if (MODE == 3 || MODE == 4) {
    // [1024 rows][1 KiB]: piece f = RPI rows x (1024 / RPI) bytes
    constexpr int RPI = MODE == 3 ? 16 : 8, LPR = 64 / RPI;
    const int row = lane / LPR, kq = lane % LPR;
    for (int it = 0; it < iters; it += 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int f = (c + q) % nchunk;
        const int r0 = (f / (1024 / (LPR * 16))) * RPI % 1024, k0 = (f % (1024 / (LPR * 16))) * LPR * 16;
        __builtin_amdgcn_global_load_lds(
            GPTR(reinterpret_cast<const char*>(buf) + (size_t)(r0 + row) * 1024 + k0 + kq * 16),
            LPTR(ring + (wave * 8 + q) * 64), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      c = (c + 8) % nchunk;
    }
    __syncthreads();
    acc = ring[threadIdx.x];
  } else {
    // [1024 rows][512 bf16] = 1 MiB: fragment = rows r0..r0+15, K bytes k0..k0+63
    const int row = lane & 15, kq = lane >> 4;
    for (int it = 0; it < iters; it += 8) {
      uint4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int f = (c + q) % nchunk;           // fragment id: 64 row tiles x 16 k-steps
        const int r0 = (f >> 4) * 16, k0 = (f & 15) * 64;  // bytes
        v[q] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(buf) + (size_t)(r0 + row) * 1024 + k0 + kq * 16);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) { acc.x ^= v[q].x; acc.y ^= v[q].y; acc.z ^= v[q].z; acc.w ^= v[q].w; }
      c = (c + 8) % nchunk;
    }
  }
  if (acc.x == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  uint4* buf;
  uint4* out;
  hipMalloc(&buf, BUF);
  hipMalloc(&out, (size_t)4096 * 256 * 16);
  hipMemset(buf, 1, BUF);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int wgs_per_cu = 1; wgs_per_cu <= 4; wgs_per_cu *= 2) {
    const int grid = 256 * wgs_per_cu;
    for (int mode = 0; mode < 5; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(feed<0>, dim3(grid), dim3(256), 0, 0, buf, iters, out);
        else if (mode == 1) hipLaunchKernelGGL(feed<1>, dim3(grid), dim3(256), 0, 0, buf, iters, out);
        else if (mode == 3) hipLaunchKernelGGL(feed<3>, dim3(grid), dim3(256), 0, 0, buf, iters, out);
        else if (mode == 4) hipLaunchKernelGGL(feed<4>, dim3(grid), dim3(256), 0, 0, buf, iters, out);
        else hipLaunchKernelGGL(feed<2>, dim3(grid), dim3(256), 0, 0, buf, iters, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = (double)grid * 4 * iters * 1024;
        if (rep == 2)
          printf("wg/cu %d mode %d (%s): %.1f us, %.2f TB/s chip, %.1f GB/s per CU\n", wgs_per_cu, mode,
                 mode == 0 ? "reg 1KiB" : mode == 1 ? "lds-dma 1KiB" : mode == 2 ? "reg fragment 16x64B" : mode == 3 ? "lds-dma 16x64B" : "lds-dma 8x128B", ms * 1e3,
                 bytes / ms / 1e9, bytes / ms / 1e6 / 256);
      }
    }
  }
  return 0;
}
