// Encoder helper kernels for gfx950: the parts of the RMB eval graph
// (reference model/utils/modules/card.py:48-148) that are not GEMMs.
//
//  * depthwise 5x5 conv, stride 1, pad 2, NHWC (card.DSC depth.1 / point.1,
//    card.py:28-29,38-39), all four branches at once (1024 channels).  MIOpen
//    has no fast bf16 NHWC depthwise path on gfx950 (it falls back to a naive
//    kernel at ~0.14 TB/s); this one stages one ROI x 64-channel tile in LDS and
//    register-blocks a whole output row per thread.  HBM-bound: it reads and
//    writes the [N*S*S, C] activation once.
//  * act + per-ROI channel mean in one pass (SiLU / Hardswish after the BN-
//    folded GEMM, card.py:53-56; the SE squeeze, card.py:75; the GAP of
//    encoderAndHead.py:29), optionally in place, optionally without writing.
//  * per-ROI channel scale in place (SE excitation, card.py:78).
#include "trk_common.h"

#include <type_traits>

namespace {

// 2 consecutive channels per access
template <typename T> struct Pair;
template <> struct Pair<float> {
  using S = float2;
  static __device__ __forceinline__ void unpack(S s, float& a, float& b) { a = s.x; b = s.y; }
  static __device__ __forceinline__ S pack(float a, float b) { return make_float2(a, b); }
};
template <> struct Pair<uint16_t> {
  using S = uint32_t;
  static __device__ __forceinline__ void unpack(S s, float& a, float& b) {
    a = __uint_as_float(s << 16);
    b = __uint_as_float(s & 0xffff0000u);
  }
  static __device__ __forceinline__ S pack(float a, float b) {
    return (uint32_t)trk::f32_to_bf16(a) | ((uint32_t)trk::f32_to_bf16(b) << 16);
  }
};

constexpr int kDwCh = 64;   // channels per workgroup
constexpr int kMaxW = 32;   // max spatial width handled in registers

// grid: (N * ceil(C/64)); block: 32 x H threads (channel pair x output row);
// kW = compile-time row width (>= W) so the register row is exactly sized
template <typename T, int kW>
__global__ void __launch_bounds__(512) dwconv5_nhwc_kernel(const T* __restrict__ in, const float* __restrict__ w,
                                    T* __restrict__ out, int N, int H, int W, int C, int nchunk) {
  using PS = typename Pair<T>::S;
  extern __shared__ __align__(16) unsigned char smem[];
  PS* tile = reinterpret_cast<PS*>(smem);  // [H][W][32] pairs
  const int n = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk;
  const int c0 = chunk * kDwCh;
  const int nch = min(kDwCh, C - c0);
  const int npair = nch / 2;
  const int tid = threadIdx.x;
  const PS* src = reinterpret_cast<const PS*>(in + ((int64_t)n * H * W) * C + c0);
  // stage [H*W][32 pairs] with 16-B pieces, BATCH loads in flight per thread
  constexpr int EPP = 16 / (int)sizeof(T);             // elements per 16-B piece
  constexpr int PPP = kDwCh / EPP;                      // pieces per pixel
  constexpr int BATCH = 4;
  const int total = H * W * PPP;
  const bool vec_ok = (C % EPP) == 0;
  for (int q0 = tid; q0 < total; q0 += blockDim.x * BATCH) {
    uint4 tmp[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int q = q0 + (int)blockDim.x * k;
      const int p = q / PPP, e = (q % PPP) * EPP;
      tmp[k] = (q < total && vec_ok && e < nch)
                   ? *reinterpret_cast<const uint4*>(in + ((int64_t)n * H * W + p) * C + c0 + e)
                   : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int q = q0 + (int)blockDim.x * k;
      if (q >= total) continue;
      const int p = q / PPP, e = (q % PPP) * EPP;
      if (vec_ok && e < nch) {
        *reinterpret_cast<uint4*>(reinterpret_cast<char*>(tile + p * 32) + (q % PPP) * 16) = tmp[k];
      } else {
        for (int kk = 0; kk < EPP; kk += 2)
          if (e + kk < nch) tile[p * 32 + (e + kk) / 2] = src[(int64_t)p * (C / 2) + (e + kk) / 2];
      }
    }
  }
  __syncthreads();
  const int cp = tid % 32, y = tid / 32;
  if (cp >= npair || y >= H) return;
  const int c = c0 + 2 * cp;
  float wa[25], wb[25];  // weights stored tap-major [25][C]: one 8-B load per tap
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    const float2 ww = *reinterpret_cast<const float2*>(w + (int64_t)k * C + c);
    wa[k] = ww.x;
    wb[k] = ww.y;
  }
  float acc_a[kW], acc_b[kW];
#pragma unroll
  for (int x = 0; x < kW; ++x) { acc_a[x] = 0.f; acc_b[x] = 0.f; }
#pragma unroll
  for (int ky = 0; ky < 5; ++ky) {
    const int yy = y + ky - 2;
    if (yy < 0 || yy >= H) continue;
    float ra[kW + 4], rb[kW + 4];
#pragma unroll
    for (int x = 0; x < kW + 4; ++x) {
      const int xx = x - 2;
      if (xx >= 0 && xx < W) Pair<T>::unpack(tile[(yy * W + xx) * 32 + cp], ra[x], rb[x]);
      else { ra[x] = 0.f; rb[x] = 0.f; }
    }
#pragma unroll
    for (int x = 0; x < kW; ++x) {
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        acc_a[x] = fmaf(wa[ky * 5 + kx], ra[x + kx], acc_a[x]);
        acc_b[x] = fmaf(wb[ky * 5 + kx], rb[x + kx], acc_b[x]);
      }
    }
  }
  PS* dst = reinterpret_cast<PS*>(out + ((int64_t)n * H * W + (int64_t)y * W) * C + c0);
#pragma unroll
  for (int x = 0; x < kW; ++x)
    if (x < W) dst[(int64_t)x * (C / 2) + cp] = Pair<T>::pack(acc_a[x], acc_b[x]);
}

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == 1) return v / (1.0f + expf(-v));                        // SiLU
  if (act == 2) return v * fminf(fmaxf(v + 3.0f, 0.0f), 6.0f) / 6.0f;  // Hardswish
  return v;
}

// x [N, P, C] (P = pixels per ROI); y = act(x) written to out (may alias x,
// may be null); mean[N, C] f32 = mean over P of y.  One workgroup per
// (ROI, 256-channel slab), threads over channel pairs x pixel groups.
template <typename T>
__global__ void __launch_bounds__(256)
act_mean_kernel(const T* __restrict__ x, T* out, float* __restrict__ mean, int N, int P, int C,
                int act, int nslab) {
  using PS = typename Pair<T>::S;
  __shared__ float red[2][256];
  const int n = blockIdx.x / nslab, slab = blockIdx.x % nslab;
  const int cp = threadIdx.x % 128, pg = threadIdx.x / 128;  // 2 pixel groups
  const int c = slab * 256 + 2 * cp;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    const PS* src = reinterpret_cast<const PS*>(x + (int64_t)n * P * C + c);
    PS* dst = out ? reinterpret_cast<PS*>(out + (int64_t)n * P * C + c) : nullptr;
    for (int p = pg; p < P; p += 2) {
      float a, b;
      Pair<T>::unpack(src[(int64_t)p * (C / 2)], a, b);
      a = act_apply(a, act);
      b = act_apply(b, act);
      if (dst) dst[(int64_t)p * (C / 2)] = Pair<T>::pack(a, b);
      sa += a;
      sb += b;
    }
  }
  red[0][threadIdx.x] = sa;
  red[1][threadIdx.x] = sb;
  __syncthreads();
  if (pg == 0 && c < C) {
    mean[(int64_t)n * C + c] = (red[0][cp] + red[0][cp + 128]) / (float)P;
    mean[(int64_t)n * C + c + 1] = (red[1][cp] + red[1][cp + 128]) / (float)P;
  }
}

// x[n, p, c] *= s[n, c] (in place)
template <typename T>
__global__ void __launch_bounds__(256)
scale_rows_kernel(T* __restrict__ x, const float* __restrict__ s, int64_t total_pairs, int P, int C) {
  using PS = typename Pair<T>::S;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total_pairs) return;
  const int64_t e = q * 2;
  const int c = (int)(e % C);
  const int64_t n = e / ((int64_t)P * C);
  PS* px = reinterpret_cast<PS*>(x) + q;
  float a, b;
  Pair<T>::unpack(*px, a, b);
  *px = Pair<T>::pack(a * s[n * C + c], b * s[n * C + c + 1]);
}

}  // namespace

extern "C" int trk_dwconv5_nhwc(const void* in, const float* weight, void* out, int64_t N, int64_t H,
                                int64_t W, int64_t C, int dtype, void* stream) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "dwconv5: dtype must be f32 or bf16");
  TRK_REQUIRE(N >= 0 && H >= 1 && W >= 1 && C >= 2 && C % 2 == 0, "dwconv5: bad shape");
  TRK_REQUIRE(W <= kMaxW && 32 * H <= 512, "dwconv5: spatial size %lldx%lld above 16 rows x 32 cols",
              (long long)H, (long long)W);
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(in && weight && out && in != out, "dwconv5: null or aliased pointer");
  const int nchunk = (int)((C + kDwCh - 1) / kDwCh);
  const size_t esz = dtype == TRK_F32 ? 8 : 4;  // bytes per channel pair
  const size_t lds = esz * 32 * (size_t)(H * W);
  TRK_REQUIRE(lds <= 160 * 1024, "dwconv5: %lldx%lld tile does not fit LDS", (long long)H, (long long)W);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(N * nchunk)), block((unsigned)(32 * H));
  auto go = [&](auto kw) {
    constexpr int KW = decltype(kw)::value;
    if (lds > 64 * 1024) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dwconv5_nhwc_kernel<float, KW>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dwconv5_nhwc_kernel<uint16_t, KW>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
    if (dtype == TRK_F32)
      hipLaunchKernelGGL((dwconv5_nhwc_kernel<float, KW>), grid, block, lds, st, (const float*)in, weight,
                         (float*)out, (int)N, (int)H, (int)W, (int)C, nchunk);
    else
      hipLaunchKernelGGL((dwconv5_nhwc_kernel<uint16_t, KW>), grid, block, lds, st, (const uint16_t*)in,
                         weight, (uint16_t*)out, (int)N, (int)H, (int)W, (int)C, nchunk);
  };
  if (W <= 7) go(std::integral_constant<int, 7>{});
  else if (W <= 10) go(std::integral_constant<int, 10>{});
  else if (W <= 16) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, kMaxW>{});
  return trk::check_launch("dwconv5_nhwc_kernel");
}

extern "C" int trk_act_mean(const void* x, void* out, float* mean, int64_t N, int64_t P, int64_t C,
                            int act, int dtype, void* stream) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "act_mean: dtype must be f32 or bf16");
  TRK_REQUIRE(N >= 0 && P >= 1 && C >= 2 && C % 2 == 0, "act_mean: bad shape");
  TRK_REQUIRE(act >= 0 && act <= 2, "act_mean: act must be 0 (none), 1 (SiLU) or 2 (Hardswish)");
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(x && mean, "act_mean: null pointer");
  const int nslab = (int)((C + 255) / 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == TRK_F32)
    hipLaunchKernelGGL(act_mean_kernel<float>, dim3((unsigned)(N * nslab)), dim3(256), 0, st,
                       (const float*)x, (float*)out, mean, (int)N, (int)P, (int)C, act, nslab);
  else
    hipLaunchKernelGGL(act_mean_kernel<uint16_t>, dim3((unsigned)(N * nslab)), dim3(256), 0, st,
                       (const uint16_t*)x, (uint16_t*)out, mean, (int)N, (int)P, (int)C, act, nslab);
  return trk::check_launch("act_mean_kernel");
}

extern "C" int trk_scale_rows(void* x, const float* s, int64_t N, int64_t P, int64_t C, int dtype,
                              void* stream) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "scale_rows: dtype must be f32 or bf16");
  TRK_REQUIRE(N >= 0 && P >= 1 && C >= 2 && C % 2 == 0, "scale_rows: bad shape");
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(x && s, "scale_rows: null pointer");
  const int64_t pairs = N * P * C / 2;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned g = (unsigned)((pairs + 255) / 256);
  if (dtype == TRK_F32)
    hipLaunchKernelGGL(scale_rows_kernel<float>, dim3(g), dim3(256), 0, st, (float*)x, s, pairs, (int)P, (int)C);
  else
    hipLaunchKernelGGL(scale_rows_kernel<uint16_t>, dim3(g), dim3(256), 0, st, (uint16_t*)x, s, pairs, (int)P,
                       (int)C);
  return trk::check_launch("scale_rows_kernel");
}
