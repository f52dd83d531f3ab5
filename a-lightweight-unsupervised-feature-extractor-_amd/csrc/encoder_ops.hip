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
    return trk::pack2_bf16(a, b);
  }
};

constexpr int kDwCh = 64;   // channels per workgroup
constexpr int kMaxW = 32;   // max spatial width handled in registers
constexpr int kDwRois = 16; // ROIs per workgroup (weights stay in registers across them)

typedef float dw_f2 __attribute__((ext_vector_type(2)));

// 16-B global piece -> f32 channel pairs in LDS
template <typename T> struct Piece;
template <> struct Piece<float> {  // 4 channels
  static __device__ __forceinline__ void put(dw_f2* d, uint4 v) {
    d[0] = dw_f2{__uint_as_float(v.x), __uint_as_float(v.y)};
    d[1] = dw_f2{__uint_as_float(v.z), __uint_as_float(v.w)};
  }
};
template <> struct Piece<uint16_t> {  // 8 channels
  static __device__ __forceinline__ void put(dw_f2* d, uint4 v) {
    d[0] = dw_f2{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u)};
    d[1] = dw_f2{__uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
    d[2] = dw_f2{__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xffff0000u)};
    d[3] = dw_f2{__uint_as_float(v.w << 16), __uint_as_float(v.w & 0xffff0000u)};
  }
};

// grid: (ceil(N / kDwRois) * ceil(C/64)); block: 32 x H threads (channel pair
// x output row).  The workgroup's 25 x 64 weights are loaded once into
// registers and reused for kDwRois ROIs.  ROI tiles are double-buffered in LDS
// as f32 channel pairs [H*W][32] (converted once at staging, so the 5 x (W+4)
// tap reads per output row need no unpacking): the next ROI's global loads are
// issued before the current ROI is computed and committed to the other buffer
// after.  Taps run on channel pairs (v_pk_fma_f32).  kW = compile-time width.
template <typename T, int kW>
__global__ void __launch_bounds__(512) dwconv5_nhwc_kernel(const T* __restrict__ in, const float* __restrict__ w,
                                    T* __restrict__ out, int N, int H, int W, int C, int nchunk) {
  using PS = typename Pair<T>::S;
  extern __shared__ __align__(16) unsigned char smem[];
  const int HW = H * W;
  dw_f2* tiles = reinterpret_cast<dw_f2*>(smem);  // 2 x [H*W][32] f32 pairs
  const int chunk = blockIdx.x % nchunk, grp = blockIdx.x / nchunk;
  const int n0 = grp * kDwRois, n1 = min(N, n0 + kDwRois);
  const int c0 = chunk * kDwCh;
  const int nch = min(kDwCh, C - c0);
  const int npair = nch / 2;
  const int tid = threadIdx.x, nthr = blockDim.x;
  constexpr int EPP = 16 / (int)sizeof(T);  // elements per 16-B piece
  constexpr int PPP = kDwCh / EPP;          // pieces per pixel
  constexpr int MAXP = (kW * PPP + 31) / 32;  // pieces per thread per tile (W <= kW, 32*H threads)
  const int total = HW * PPP;
  const bool vec_ok = (C % EPP) == 0;

  uint4 stg[MAXP];
  auto issue = [&](int n) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + nthr * k;
      const int p = q / PPP, e = (q % PPP) * EPP;
      const T* base = in + (int64_t)n * HW * C + c0;  // uniform; the per-lane offset is 32-bit
      stg[k] = (q < total && vec_ok && e < nch) ? *reinterpret_cast<const uint4*>(base + (p * C + e))
                                                : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&](int n, dw_f2* tile) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + nthr * k;
      if (q >= total) continue;
      const int p = q / PPP, e = (q % PPP) * EPP;
      if (vec_ok && e < nch) {
        Piece<T>::put(tile + p * 32 + e / 2, stg[k]);
      } else {  // ragged channel tail (C not a multiple of 64 / of the piece width)
        const PS* src = reinterpret_cast<const PS*>(in + ((int64_t)n * HW) * C + c0);
        for (int kk = 0; kk < EPP; kk += 2)
          if (e + kk < nch) {
            float a, b;
            Pair<T>::unpack(src[(int64_t)p * (C / 2) + (e + kk) / 2], a, b);
            tile[p * 32 + (e + kk) / 2] = dw_f2{a, b};
          }
      }
    }
  };

  const int cp = tid % 32, y = tid / 32;
  const bool worker = cp < npair && y < H;
  // the workgroup's weights [25][32 pairs] in LDS (tap-major [25][C] in HBM),
  // loaded once and read 5 pairs per input row
  dw_f2* wl = tiles + 2 * HW * 32;
  for (int q = tid; q < 25 * 32; q += nthr) {
    const int k = q / 32, pp = q % 32;
    wl[q] = pp < npair ? *reinterpret_cast<const dw_f2*>(w + (int64_t)k * C + c0 + 2 * pp) : dw_f2{0.f, 0.f};
  }

  if (n0 < n1) {
    issue(n0);
    commit(n0, tiles);
  }
  __syncthreads();
  for (int n = n0; n < n1; ++n) {
    const dw_f2* cur = tiles + ((n - n0) & 1) * HW * 32;
    dw_f2* nxt = tiles + ((n - n0 + 1) & 1) * HW * 32;
    if (n + 1 < n1) issue(n + 1);
    if (worker) {
      dw_f2 acc[kW];
#pragma unroll
      for (int x = 0; x < kW; ++x) acc[x] = dw_f2{0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        const int yy = y + ky - 2;
        if (yy < 0 || yy >= H) continue;
        dw_f2 rr[kW + 4], wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(ky * 5 + kx) * 32 + cp];
#pragma unroll
        for (int x = 0; x < kW + 4; ++x) {
          const int xx = x - 2;  // static edge test when W == kW (the 7x7 / 10x10 instantiations)
          const bool in_row = xx >= 0 && (W == kW ? xx < kW : xx < W);
          rr[x] = in_row ? cur[(yy * W + xx) * 32 + cp] : dw_f2{0.f, 0.f};
        }
#pragma unroll
        for (int x = 0; x < kW; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) acc[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], acc[x]);
      }
      PS* dst = reinterpret_cast<PS*>(out + (int64_t)n * HW * C + c0);  // uniform base
      const int orow = y * W * (C / 2) + cp;                           // 32-bit per-lane offset
#pragma unroll
      for (int x = 0; x < kW; ++x)
        if (W == kW || x < W) dst[orow + x * (C / 2)] = Pair<T>::pack(acc[x].x, acc[x].y);
    }
    if (n + 1 < n1) commit(n + 1, nxt);
    __syncthreads();
  }
}

// Fast path for the encoder's shapes (S x S ROIs with S in {7, 10}, C a
// multiple of 128): 128-channel chunks, one wave per output ROW PAIR (lanes =
// 64 channel pairs, so LDS reads and global stores are 512 B / 256 B
// contiguous), each thread accumulating two output rows from six input rows
// (4.2 tap reads per output instead of 7).  f32 channel-pair tiles, double-
// buffered, kDwRoisFast ROIs per workgroup; weights [25][64 pairs] in LDS.
// Same per-output FMA order as the generic kernel (ky, then kx): identical.
constexpr int kDwRoisFast = 64;

template <typename T, int kS>
__global__ void __launch_bounds__(64 * ((kS + 1) / 2))
dwconv5_rows2_kernel(const T* __restrict__ in, const float* __restrict__ w, T* __restrict__ out, int N, int C) {
  using PS = typename Pair<T>::S;
  constexpr int H = kS, W = kS, HW = kS * kS, CH = 128, NP = 64;
  constexpr int NTHR = 64 * ((kS + 1) / 2);
  constexpr int EPP = 16 / (int)sizeof(T), PPP = CH / EPP;  // 16-B pieces per pixel
  constexpr int MAXP = (HW * PPP + NTHR - 1) / NTHR;
  extern __shared__ __align__(16) unsigned char smem[];
  dw_f2* tiles = reinterpret_cast<dw_f2*>(smem);  // 2 x [HW][64 pairs]
  dw_f2* wl = tiles + 2 * HW * NP;                // [25][64 pairs]
  const int nchunk = C / CH;
  const int chunk = blockIdx.x % nchunk, grp = blockIdx.x / nchunk;
  const int n0 = grp * kDwRoisFast, n1 = min(N, n0 + kDwRoisFast);
  const int c0 = chunk * CH;
  const int tid = threadIdx.x;
  const int cp = tid & 63, y0 = 2 * (tid >> 6);
  constexpr int total = HW * PPP;
  uint4 stg[MAXP];
  auto issue = [&](int n) {
    const T* base = in + (int64_t)n * HW * C + c0;  // uniform; per-lane offset is 32-bit
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + NTHR * k;
      const int p = q / PPP, e = (q % PPP) * EPP;
      stg[k] = q < total ? *reinterpret_cast<const uint4*>(base + (p * C + e)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&](dw_f2* tile) {
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
      const int q = tid + NTHR * k;
      if (q >= total) continue;
      const int p = q / PPP, e = (q % PPP) * EPP;
      Piece<T>::put(tile + p * NP + e / 2, stg[k]);
    }
  };
  for (int q = tid; q < 25 * NP; q += NTHR)
    wl[q] = *reinterpret_cast<const dw_f2*>(w + (int64_t)(q / NP) * C + c0 + 2 * (q % NP));
  if (n0 < n1) {
    issue(n0);
    commit(tiles);
  }
  __syncthreads();
  for (int n = n0; n < n1; ++n) {
    const dw_f2* cur = tiles + ((n - n0) & 1) * HW * NP;
    dw_f2* nxt = tiles + ((n - n0 + 1) & 1) * HW * NP;
    if (n + 1 < n1) issue(n + 1);
    dw_f2 a0[kS], a1[kS];
#pragma unroll
    for (int x = 0; x < kS; ++x) { a0[x] = dw_f2{0.f, 0.f}; a1[x] = dw_f2{0.f, 0.f}; }
#pragma unroll
    for (int r = 0; r < 6; ++r) {  // input rows y0-2 .. y0+3 (wave-uniform bounds)
      const int yy = y0 - 2 + r;
      if (yy < 0 || yy >= H) continue;
      dw_f2 rr[kS + 4];
#pragma unroll
      for (int x = 0; x < kS + 4; ++x) {
        const int xx = x - 2;
        rr[x] = (xx >= 0 && xx < W) ? cur[(yy * W + xx) * NP + cp] : dw_f2{0.f, 0.f};
      }
      if (r <= 4) {  // output row y0: ky = r
        dw_f2 wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(r * 5 + kx) * NP + cp];
#pragma unroll
        for (int x = 0; x < kS; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) a0[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], a0[x]);
      }
      if (r >= 1) {  // output row y0 + 1: ky = r - 1
        dw_f2 wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[((r - 1) * 5 + kx) * NP + cp];
#pragma unroll
        for (int x = 0; x < kS; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) a1[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx], a1[x]);
      }
    }
    PS* dst = reinterpret_cast<PS*>(out + (int64_t)n * HW * C + c0);
#pragma unroll
    for (int x = 0; x < kS; ++x) {
      dst[(y0 * W + x) * (C / 2) + cp] = Pair<T>::pack(a0[x].x, a0[x].y);
      if (y0 + 1 < H) dst[((y0 + 1) * W + x) * (C / 2) + cp] = Pair<T>::pack(a1[x].x, a1[x].y);
    }
    if (n + 1 < n1) commit(nxt);
    __syncthreads();
  }
}

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == 1) return v / (1.0f + expf(-v));                        // SiLU
  if (act == 2) return v * fminf(fmaxf(v + 3.0f, 0.0f), 6.0f) / 6.0f;  // Hardswish
  return v;
}

// 16-B vector of T: 8 bf16 or 4 f32 channels
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int kN = 4;
  static __device__ __forceinline__ void unpack(uint4 v, float (&f)[4]) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float (&f)[4]) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <> struct Vec16<uint16_t> {
  static constexpr int kN = 8;
  static __device__ __forceinline__ void unpack(uint4 v, float (&f)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { f[2 * k] = __uint_as_float(w[k] << 16); f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u); }
  }
  static __device__ __forceinline__ uint4 pack(const float (&f)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = trk::pack2_bf16(f[2 * k], f[2 * k + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// x [N, P, C] (P = pixels per ROI); y = act(x) written to out (may alias x,
// may be null); mean[N, C] f32 = mean over P of y.  One workgroup per ROI:
// each thread owns one 16-B channel vector and a pixel stride, with kUnroll
// independent 16-B loads in flight; pixel groups are reduced through LDS.
// Requires C % (16 / sizeof(T)) == 0 and C / vec <= 256.
constexpr int kAmUnroll = 5;

template <typename T>
__global__ void __launch_bounds__(256)
act_mean_kernel(const T* __restrict__ x, T* out, float* __restrict__ mean, int N, int P, int C, int ld,
                int act) {
  using V = Vec16<T>;
  constexpr int E = V::kN;
  __shared__ float red[256 * 8];
  const int n = blockIdx.x;
  const int nv = C / E;                 // vectors per pixel
  const int groups = 256 / nv;          // pixel groups
  const int v = threadIdx.x % nv, g = threadIdx.x / nv;
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  if (g < groups) {
    const T* src = x + (int64_t)n * P * ld + v * E;
    T* dst = out ? out + (int64_t)n * P * ld + v * E : nullptr;
    for (int p0 = g; p0 < P; p0 += groups * kAmUnroll) {
      uint4 raw[kAmUnroll];
#pragma unroll
      for (int u = 0; u < kAmUnroll; ++u) {
        const int p = p0 + u * groups;
        raw[u] = p < P ? *reinterpret_cast<const uint4*>(src + (int64_t)p * ld) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kAmUnroll; ++u) {
        const int p = p0 + u * groups;
        if (p >= P) break;
        float f[E];
        V::unpack(raw[u], f);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          f[e] = act_apply(f[e], act);
          acc[e] += f[e];
        }
        if (dst) *reinterpret_cast<uint4*>(dst + (int64_t)p * ld) = V::pack(f);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) red[e * 256 + threadIdx.x] = acc[e];
  __syncthreads();
  if (g == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float sum = 0.f;
      for (int q = 0; q < groups; ++q) sum += red[e * 256 + q * nv + v];
      mean[(int64_t)n * C + v * E + e] = sum / (float)P;
    }
  }
}

// x[n, p, c] = act(x[n, p, c]) * s[n, c] (in place; act 0 = identity);
// one 16-B vector per thread (C % (16 / sizeof(T)) == 0), else channel pairs
template <typename T>
__global__ void __launch_bounds__(256)
scale_rows_kernel(T* __restrict__ x, const float* __restrict__ s, int64_t total_vec, int P, int C, int ld,
                  int act) {
  using V = Vec16<T>;
  constexpr int E = V::kN;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total_vec) return;
  const int64_t e0 = q * E;
  const int c = (int)(e0 % C);
  const int64_t row = e0 / C;             // pixel row over all ROIs
  const int64_t n = row / P;
  uint4* px = reinterpret_cast<uint4*>(x + row * ld + c);
  float f[E];
  V::unpack(*px, f);
  const float4* sp = reinterpret_cast<const float4*>(s + n * C + c);  // 16-B aligned: c % E == 0
  float sv[E];
#pragma unroll
  for (int k = 0; k < E / 4; ++k) {
    const float4 t = sp[k];
    sv[4 * k] = t.x; sv[4 * k + 1] = t.y; sv[4 * k + 2] = t.z; sv[4 * k + 3] = t.w;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) f[e] = act_apply(f[e], act) * sv[e];
  *px = V::pack(f);
}

template <typename T>
__global__ void __launch_bounds__(256)
scale_rows_pairs_kernel(T* __restrict__ x, const float* __restrict__ s, int64_t total_pairs, int P, int C,
                        int act) {
  using PS = typename Pair<T>::S;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total_pairs) return;
  const int64_t e = q * 2;
  const int c = (int)(e % C);
  const int64_t n = e / ((int64_t)P * C);
  PS* px = reinterpret_cast<PS*>(x) + q;
  float a, b;
  Pair<T>::unpack(*px, a, b);
  a = act_apply(a, act);
  b = act_apply(b, act);
  *px = Pair<T>::pack(a * s[n * C + c], b * s[n * C + c + 1]);
}

}  // namespace

int g_dw_fast = 1;  // trk_set_tuning("dw_fast"): 0 forces the generic depthwise kernel

extern "C" int trk_dwconv5_nhwc(const void* in, const float* weight, void* out, int64_t N, int64_t H,
                                int64_t W, int64_t C, int dtype, void* stream) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "dwconv5: dtype must be f32 or bf16");
  TRK_REQUIRE(N >= 0 && H >= 1 && W >= 1 && C >= 2 && C % 2 == 0, "dwconv5: bad shape");
  TRK_REQUIRE(W <= kMaxW && 32 * H <= 512, "dwconv5: spatial size %lldx%lld above 16 rows x 32 cols",
              (long long)H, (long long)W);
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(in && weight && out && in != out, "dwconv5: null or aliased pointer");
  const int nchunk = (int)((C + kDwCh - 1) / kDwCh);
  const size_t lds = 8 * 32 * (2 * (size_t)(H * W) + 25);  // 2 tiles of f32 channel pairs + weights
  TRK_REQUIRE(lds <= 160 * 1024, "dwconv5: %lldx%lld tile does not fit LDS", (long long)H, (long long)W);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (H == W && (H == 10 || H == 7) && C % 128 == 0 && g_dw_fast) {
    const int64_t ng = (N + kDwRoisFast - 1) / kDwRoisFast;
    const size_t lf = 8 * 64 * (2 * (size_t)(H * W) + 25);
    auto fast = [&](auto ks) {
      constexpr int KS = decltype(ks)::value;
      constexpr int NT = 64 * ((KS + 1) / 2);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dwconv5_rows2_kernel<float, KS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dwconv5_rows2_kernel<uint16_t, KS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (dtype == TRK_F32)
        hipLaunchKernelGGL((dwconv5_rows2_kernel<float, KS>), dim3((unsigned)(ng * (C / 128))), dim3(NT), lf, st,
                           (const float*)in, weight, (float*)out, (int)N, (int)C);
      else
        hipLaunchKernelGGL((dwconv5_rows2_kernel<uint16_t, KS>), dim3((unsigned)(ng * (C / 128))), dim3(NT), lf,
                           st, (const uint16_t*)in, weight, (uint16_t*)out, (int)N, (int)C);
    };
    if (H == 10) fast(std::integral_constant<int, 10>{});
    else fast(std::integral_constant<int, 7>{});
    return trk::check_launch("dwconv5_rows2_kernel");
  }
  const int64_t ngrp = (N + kDwRois - 1) / kDwRois;
  dim3 grid((unsigned)(ngrp * nchunk)), block((unsigned)(32 * H));
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

extern "C" int trk_act_mean(const void* x, void* out, float* mean, int64_t N, int64_t P, int64_t C, int64_t ld,
                            int act, int dtype, void* stream) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "act_mean: dtype must be f32 or bf16");
  const int E = dtype == TRK_F32 ? 4 : 8;
  TRK_REQUIRE(N >= 0 && P >= 1 && C >= E && C % E == 0 && C / E <= 256,
              "act_mean: C must be a multiple of %d and at most %d", E, 256 * E);
  TRK_REQUIRE(ld >= C && ld % E == 0, "act_mean: row stride ld must be >= C and a multiple of %d", E);
  TRK_REQUIRE(act >= 0 && act <= 2, "act_mean: act must be 0 (none), 1 (SiLU) or 2 (Hardswish)");
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(x && mean, "act_mean: null pointer");
  TRK_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && (!out || reinterpret_cast<uintptr_t>(out) % 16 == 0),
              "act_mean: x/out must be 16-B aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == TRK_F32)
    hipLaunchKernelGGL(act_mean_kernel<float>, dim3((unsigned)N), dim3(256), 0, st, (const float*)x, (float*)out,
                       mean, (int)N, (int)P, (int)C, (int)ld, act);
  else
    hipLaunchKernelGGL(act_mean_kernel<uint16_t>, dim3((unsigned)N), dim3(256), 0, st, (const uint16_t*)x,
                       (uint16_t*)out, mean, (int)N, (int)P, (int)C, (int)ld, act);
  return trk::check_launch("act_mean_kernel");
}

static int scale_rows_impl(void* x, const float* s, int64_t N, int64_t P, int64_t C, int64_t ld, int act,
                           int dtype, void* stream, const char* what) {
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_BF16, "%s: dtype must be f32 or bf16", what);
  TRK_REQUIRE(N >= 0 && P >= 1 && C >= 2 && C % 2 == 0, "%s: bad shape", what);
  TRK_REQUIRE(act >= 0 && act <= 2, "%s: act must be 0 (none), 1 (SiLU) or 2 (Hardswish)", what);
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(x && s, "%s: null pointer", what);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int E = dtype == TRK_F32 ? 4 : 8;
  TRK_REQUIRE(ld == C || (C % E == 0 && ld % E == 0 && ld > C), "%s: row stride ld must equal C or be a "
              "multiple of %d", what, E);
  if (C % E == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0) {
    const int64_t nv = N * P * C / E;
    const unsigned g = (unsigned)((nv + 255) / 256);
    if (dtype == TRK_F32)
      hipLaunchKernelGGL(scale_rows_kernel<float>, dim3(g), dim3(256), 0, st, (float*)x, s, nv, (int)P, (int)C,
                         (int)ld, act);
    else
      hipLaunchKernelGGL(scale_rows_kernel<uint16_t>, dim3(g), dim3(256), 0, st, (uint16_t*)x, s, nv, (int)P,
                         (int)C, (int)ld, act);
  } else {
    TRK_REQUIRE(ld == C, "%s: a row stride needs C %% %d == 0 and 16-B alignment", what, E);
    const int64_t pairs = N * P * C / 2;
    const unsigned g = (unsigned)((pairs + 255) / 256);
    if (dtype == TRK_F32)
      hipLaunchKernelGGL(scale_rows_pairs_kernel<float>, dim3(g), dim3(256), 0, st, (float*)x, s, pairs, (int)P,
                         (int)C, act);
    else
      hipLaunchKernelGGL(scale_rows_pairs_kernel<uint16_t>, dim3(g), dim3(256), 0, st, (uint16_t*)x, s, pairs,
                         (int)P, (int)C, act);
  }
  return trk::check_launch("scale_rows_kernel");
}

extern "C" int trk_scale_rows(void* x, const float* s, int64_t N, int64_t P, int64_t C, int dtype,
                              void* stream) {
  return scale_rows_impl(x, s, N, P, C, C, 0, dtype, stream, "scale_rows");
}

extern "C" int trk_act_scale_rows(void* x, const float* s, int64_t N, int64_t P, int64_t C, int64_t ld, int act,
                                  int dtype, void* stream) {
  return scale_rows_impl(x, s, N, P, C, ld, act, dtype, stream, "act_scale_rows");
}
