// Experiment harness (not product code): dwconv5 variants timed with hipEvents.
// MODE 0 = full kernel, 1 = no compute (load+commit+store zeros), 2 = no store,
// 3 = loads only.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  __hip_bfloat16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)*reinterpret_cast<uint16_t*>(&x) | ((uint32_t)*reinterpret_cast<uint16_t*>(&y) << 16);
}

template <int MODE, int ROIS, int DEPTH>
__global__ void __launch_bounds__(320) dw(const uint16_t* __restrict__ in, const float* __restrict__ w,
                                         uint16_t* __restrict__ out, int N, int C) {
  constexpr int H = 10, W = 10, HW = 100, PPP = 8, MAXP = 3;
  extern __shared__ __align__(16) unsigned char smem[];
  f2* tiles = reinterpret_cast<f2*>(smem);
  const int nchunk = C / 64;
  const int chunk = blockIdx.x % nchunk, grp = blockIdx.x / nchunk;
  const int n0 = grp * ROIS, n1 = min(N, n0 + ROIS);
  const int c0 = chunk * 64;
  const int tid = threadIdx.x, nthr = 320;
  const int total = HW * PPP;
  uint4 stg[DEPTH][MAXP];
  auto issue = [&](int n, uint4 (&sg)[MAXP]) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + nthr * k;
      const int p = q / PPP, e = (q % PPP) * 8;
      const uint16_t* base = in + (int64_t)n * HW * C + c0;
      sg[k] = q < total ? *reinterpret_cast<const uint4*>(base + (p * C + e)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&](f2* tile, const uint4 (&sg)[MAXP]) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + nthr * k;
      if (q >= total) continue;
      const int p = q / PPP, e = (q % PPP) * 8;
      f2* d = tile + p * 32 + e / 2;
      const uint4 v = sg[k];
      d[0] = f2{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u)};
      d[1] = f2{__uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
      d[2] = f2{__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xffff0000u)};
      d[3] = f2{__uint_as_float(v.w << 16), __uint_as_float(v.w & 0xffff0000u)};
    }
  };
  const int cp = tid % 32, y = tid / 32;
  f2* wl = tiles + (DEPTH + 1) * HW * 32;
  for (int q = tid; q < 25 * 32; q += nthr) {
    const int k = q / 32, pp = q % 32;
    wl[q] = *reinterpret_cast<const f2*>(w + (int64_t)k * C + c0 + 2 * pp);
  }
  // prologue: tiles n0 .. n0+DEPTH-1 in flight, n0 committed
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (n0 + d < n1) issue(n0 + d, stg[d]);
  if (n0 < n1) commit(tiles, stg[0]);
  __syncthreads();
  for (int n = n0; n < n1; ++n) {
    const int slot = (n - n0) % (DEPTH + 1);
    const f2* cur = tiles + slot * HW * 32;
    f2* nxt = tiles + ((n - n0 + 1) % (DEPTH + 1)) * HW * 32;
    // rotate the register stages: stg[0] holds n+1 after this
#pragma unroll
    for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
      for (int k = 0; k < MAXP; ++k) stg[d][k] = stg[d + 1][k];
    if (n + DEPTH < n1) issue(n + DEPTH, stg[DEPTH - 1]);
    if (MODE != 3) {
      f2 acc[10];
#pragma unroll
      for (int x = 0; x < 10; ++x) acc[x] = f2{0.f, 0.f};
      if (MODE != 1) {
#pragma unroll
        for (int ky = 0; ky < 5; ++ky) {
          const int yy = y + ky - 2;
          if (yy < 0 || yy >= H) continue;
          f2 rr[14], wv[5];
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(ky * 5 + kx) * 32 + cp];
#pragma unroll
          for (int x = 0; x < 14; ++x) {
            const int xx = x - 2;
            rr[x] = (xx >= 0 && xx < 10) ? cur[(yy * W + xx) * 32 + cp] : f2{0.f, 0.f};
          }
#pragma unroll
          for (int x = 0; x < 10; ++x)
#pragma unroll
            for (int kx = 0; kx < 5; ++kx) acc[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], acc[x]);
        }
      }
      uint32_t* dst = reinterpret_cast<uint32_t*>(out + (int64_t)n * HW * C + c0);
      const int orow = y * W * (C / 2) + cp;
      if (MODE != 2) {
#pragma unroll
        for (int x = 0; x < 10; ++x) dst[orow + x * (C / 2)] = pack2(acc[x].x, acc[x].y);
      } else if (acc[0].x == 12345.f) {
        dst[orow] = 0;
      }
    }
    if (n + 1 < n1 && MODE != 3) commit(nxt, stg[0]);
    __syncthreads();
  }
}

template <int MODE, int ROIS, int DEPTH>
static float run_t(const void* in, const float* w, void* out, int N, int C, int reps) {
  const int nchunk = C / 64;
  const int ngrp = (N + ROIS - 1) / ROIS;
  size_t lds = 8 * 32 * ((DEPTH + 1) * 100 + 25);
  hipFuncSetAttribute(reinterpret_cast<const void*>(dw<MODE, ROIS, DEPTH>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((dw<MODE, ROIS, DEPTH>), dim3(ngrp * nchunk), dim3(320), lds, 0, (const uint16_t*)in, w,
                     (uint16_t*)out, N, C);
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((dw<MODE, ROIS, DEPTH>), dim3(ngrp * nchunk), dim3(320), lds, 0, (const uint16_t*)in, w,
                       (uint16_t*)out, N, C);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

extern "C" float dw_run(int mode, int rois, int depth, const void* in, const float* w, void* out, int N, int C,
                        int reps) {
#define V(M, R, D) if (mode == M && rois == R && depth == D) return run_t<M, R, D>(in, w, out, N, C, reps);
  V(0, 16, 1) V(1, 16, 1) V(2, 16, 1) V(3, 16, 1)
  V(0, 4, 1) V(0, 64, 1) V(0, 16, 2) V(0, 32, 2) V(0, 64, 3)
  V(1, 16, 2) V(3, 16, 2)
  return -1.f;
}
