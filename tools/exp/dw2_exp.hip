// Experiment harness: dwconv5 with 2-row register blocking, 128-channel chunks
// (wave = one output row pair x 64 channel pairs), LDS tile f32 or bf16.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  __hip_bfloat16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)*reinterpret_cast<uint16_t*>(&x) | ((uint32_t)*reinterpret_cast<uint16_t*>(&y) << 16);
}
__device__ __forceinline__ f2 unpack2(uint32_t v) {
  return f2{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
}

template <bool BF16TILE, int ROIS>
__global__ void __launch_bounds__(320) dw2(const uint16_t* __restrict__ in, const float* __restrict__ w,
                                          uint16_t* __restrict__ out, int N, int C) {
  constexpr int H = 10, W = 10, HW = 100, CH = 128, NP = 64, PPP = CH / 8;  // 16-B pieces per pixel
  constexpr int MAXP = (HW * PPP + 319) / 320;
  constexpr int ESZ = BF16TILE ? 4 : 8;  // bytes per pair in LDS
  extern __shared__ __align__(16) unsigned char smem[];
  const int nchunk = C / CH;
  const int chunk = blockIdx.x % nchunk, grp = blockIdx.x / nchunk;
  const int n0 = grp * ROIS, n1 = min(N, n0 + ROIS);
  const int c0 = chunk * CH;
  const int tid = threadIdx.x;
  const int cp = tid & 63, rp = tid >> 6;  // wave = row pair
  const int total = HW * PPP;
  uint4 stg[MAXP];
  auto issue = [&](int n) {
    const uint16_t* base = in + (int64_t)n * HW * C + c0;
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + 320 * k;
      const int p = q / PPP, e = (q % PPP) * 8;
      stg[k] = q < total ? *reinterpret_cast<const uint4*>(base + (p * C + e)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&](unsigned char* tile) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + 320 * k;
      if (q >= total) continue;
      const int p = q / PPP, e = (q % PPP) * 8;
      const uint4 v = stg[k];
      if (BF16TILE) {
        *reinterpret_cast<uint4*>(tile + (p * NP + e / 2) * 4) = v;
      } else {
        f2* d = reinterpret_cast<f2*>(tile) + p * NP + e / 2;
        d[0] = unpack2(v.x); d[1] = unpack2(v.y); d[2] = unpack2(v.z); d[3] = unpack2(v.w);
      }
    }
  };
  f2* wl = reinterpret_cast<f2*>(smem + 2 * HW * NP * ESZ);  // [25][64 pairs]
  for (int q = tid; q < 25 * NP; q += 320)
    wl[q] = *reinterpret_cast<const f2*>(w + (int64_t)(q / NP) * C + c0 + 2 * (q % NP));
  if (n0 < n1) { issue(n0); commit(smem); }
  __syncthreads();
  const int y0 = 2 * rp;
  for (int n = n0; n < n1; ++n) {
    const unsigned char* cur = smem + ((n - n0) & 1) * (HW * NP * ESZ);
    unsigned char* nxt = smem + ((n - n0 + 1) & 1) * (HW * NP * ESZ);
    if (n + 1 < n1) issue(n + 1);
    f2 a0[10], a1[10];
#pragma unroll
    for (int x = 0; x < 10; ++x) { a0[x] = f2{0.f, 0.f}; a1[x] = f2{0.f, 0.f}; }
#pragma unroll
    for (int r = 0; r < 6; ++r) {  // input rows y0-2 .. y0+3
      const int yy = y0 - 2 + r;
      if (yy < 0 || yy >= H) continue;  // wave-uniform
      f2 rr[14];
#pragma unroll
      for (int x = 0; x < 14; ++x) {
        const int xx = x - 2;
        if (xx >= 0 && xx < W) {
          if (BF16TILE) rr[x] = unpack2(*reinterpret_cast<const uint32_t*>(cur + ((yy * W + xx) * NP + cp) * 4));
          else rr[x] = *reinterpret_cast<const f2*>(cur + ((yy * W + xx) * NP + cp) * 8);
        } else {
          rr[x] = f2{0.f, 0.f};
        }
      }
      if (r <= 4) {  // output row y0 uses ky = r
        f2 wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(r * 5 + kx) * NP + cp];
#pragma unroll
        for (int x = 0; x < 10; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) a0[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], a0[x]);
      }
      if (r >= 1) {  // output row y0+1 uses ky = r-1
        f2 wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[((r - 1) * 5 + kx) * NP + cp];
#pragma unroll
        for (int x = 0; x < 10; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) a1[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], a1[x]);
      }
    }
    uint32_t* dst = reinterpret_cast<uint32_t*>(out + (int64_t)n * HW * C + c0);
#pragma unroll
    for (int x = 0; x < 10; ++x) {
      dst[(y0 * W + x) * (C / 2) + cp] = pack2(a0[x].x, a0[x].y);
      dst[((y0 + 1) * W + x) * (C / 2) + cp] = pack2(a1[x].x, a1[x].y);
    }
    if (n + 1 < n1) commit(nxt);
    __syncthreads();
  }
}

template <bool B, int R>
static float run_t(const void* in, const float* w, void* out, int N, int C, int reps) {
  const int nchunk = C / 128, ngrp = (N + R - 1) / R;
  size_t lds = 2 * 100 * 64 * (B ? 4 : 8) + 25 * 64 * 8;
  hipFuncSetAttribute(reinterpret_cast<const void*>(dw2<B, R>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((dw2<B, R>), dim3(ngrp * nchunk), dim3(320), lds, 0, (const uint16_t*)in, w, (uint16_t*)out,
                     N, C);
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((dw2<B, R>), dim3(ngrp * nchunk), dim3(320), lds, 0, (const uint16_t*)in, w,
                       (uint16_t*)out, N, C);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

extern "C" float dw2_run(int bf, int rois, const void* in, const float* w, void* out, int N, int C, int reps) {
  if (bf && rois == 16) return run_t<true, 16>(in, w, out, N, C, reps);
  if (bf && rois == 32) return run_t<true, 32>(in, w, out, N, C, reps);
  if (bf && rois == 64) return run_t<true, 64>(in, w, out, N, C, reps);
  if (!bf && rois == 16) return run_t<false, 16>(in, w, out, N, C, reps);
  if (!bf && rois == 32) return run_t<false, 32>(in, w, out, N, C, reps);
  if (!bf && rois == 64) return run_t<false, 64>(in, w, out, N, C, reps);
  return -1.f;
}
