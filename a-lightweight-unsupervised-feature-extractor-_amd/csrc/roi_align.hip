// ROI Align forward for gfx950 (MI355X).
//
// Replaces torchvision.ops.roi_align as called at reference tracking.py:214-221
// (MainInfer.roi_align_from_input_boxes), infer.py:163-170 and
// trainingCard.py:70-77.  Semantics: torchvision 0.20.1 CPU kernel
// (roi_align_forward_kernel_impl + pre_calc_for_bilinear_interpolate), restated
// in SURVEY.md Appendix A.1 and oracle/trk_oracle.c:ora_roi_align.  Built with
// -ffp-contract=off so every product and sum rounds where the CPU kernel rounds:
// f32 output is bit-exact against the oracle.
//
// Design:
//  * The [B,C,H,W] map is transposed once per call to NHWC (3.28 MB per frame
//    at 512x40x40) so each bilinear tap is a contiguous channel vector: a lane
//    owns VEC consecutive channels, one wave-instruction gathers 64*VEC*4 bytes.
//  * Bilinear interpolation is separable: the y sample table (PH*gh entries)
//    and x table (PW*gw entries) are built once per workgroup in LDS; the
//    per-sample weights w1..w4 = {hy,ly} x {hx,lx} are the same float products
//    torchvision's pre_calc forms.
//  * Output NHWC (encoder GEMM layout, f32 or bf16) is written directly, one
//    contiguous 64*VEC-channel vector per bin; output NCHW (torchvision's
//    contract) is staged as a [channels][PH*PW] tile in LDS and written as one
//    contiguous chunk per workgroup.
//  * blockIdx -> (roi, channel chunk) is remapped XCD-aware so that the ROIs of
//    one frame (batch index) run on one XCD and its NHWC map stays in that L2.
#include "trk_common.h"

// cache policy of the row sweep's output stores (buffer aux bits; 2 = nt, non-temporal: the
// 210 MB of ROI features stream past L2 instead of evicting the frame's map rows)
#ifndef ROI_OUT_POLICY
#define ROI_OUT_POLICY 0
#endif

#include <type_traits>

namespace {

struct AxisTab {  // one sample coordinate along y or x (pre_calc restated)
  int lo, hi;
  float l, h;     // ly (or lx) and hy = 1 - ly
  int valid;      // !(c < -1 || c > extent)
};

__device__ __forceinline__ AxisTab axis_sample(float c, int extent) {
  AxisTab t;
  if ((double)c < -1.0 || c > (float)extent) {
    t.lo = 0; t.hi = 0; t.l = 0.f; t.h = 0.f; t.valid = 0;
    return t;
  }
  if (c <= 0.f) c = 0.f;
  int lo = (int)c, hi;
  if (lo >= extent - 1) {
    hi = lo = extent - 1;
    c = (float)lo;
  } else {
    hi = lo + 1;
  }
  t.lo = lo; t.hi = hi;
  t.l = c - (float)lo;
  t.h = (float)(1. - (double)t.l);
  t.valid = 1;
  return t;
}

template <int VEC> struct VecT;
template <> struct VecT<1> { using T = float; };
template <> struct VecT<2> { using T = float2; };
template <> struct VecT<4> { using T = float4; };

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float (&v)[VEC]) {
  typename VecT<VEC>::T x = *reinterpret_cast<const typename VecT<VEC>::T*>(p);
  const float* s = reinterpret_cast<const float*>(&x);
#pragma unroll
  for (int k = 0; k < VEC; ++k) v[k] = s[k];
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD under round-robin dispatch; give
// each XCD group a contiguous range of logical block ids.
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t nx = 8;
  if (nwg < nx) return bid;
  int64_t q = nwg / nx, r = nwg % nx, x = bid % nx;
  int64_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

// (frame, channel tile, pixel tile) of a transpose block: the 1-D grid is XCD-remapped
// like roi_sweep_kernel's, so with B = 8 frames each frame's NHWC copy is written by (and
// stays in the L2 of) the XCD whose roi_sweep blocks read it next
struct TBlk { int64_t b; int cy, px; };
__device__ __forceinline__ TBlk tblk(int gx, int gy) {
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t per = (int64_t)gx * gy;
  TBlk t;
  t.b = lb / per;
  const int rem = (int)(lb - t.b * per);
  t.cy = rem / gx;
  t.px = rem - t.cy * gx;
  return t;
}

__global__ void __launch_bounds__(256)
nchw_to_nhwc_kernel(const float* __restrict__ in, float* __restrict__ out,
                    int64_t C, int64_t HW, int gx, int gy) {
  // tile: 64 channels x 64 pixels through LDS
  __shared__ float tile[64][65];
  const TBlk tb = tblk(gx, gy);
  const int64_t b = tb.b;
  const int64_t c0 = (int64_t)tb.cy * 64, p0 = (int64_t)tb.px * 64;
  const float* src = in + b * C * HW;
  float* dst = out + b * C * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 4 rows per pass
  for (int r = ty; r < 64; r += 4) {
    int64_t c = c0 + r, p = p0 + tx;
    tile[r][tx] = (c < C && p < HW) ? src[c * HW + p] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    int64_t p = p0 + r, c = c0 + tx;
    if (c < C && p < HW) dst[p * C + c] = tile[tx][r];
  }
}

// The same transpose with 16-B accesses on both sides (HW % 4 == 0, C % 4 == 0):
// 8 lanes read 32 consecutive pixels of one channel, 8 lanes write 32
// consecutive channels of one pixel (128 B each); the 4 x 4 element turn goes
// through the LDS tile.  HBM-bound: 2 x 4 B per element.  Thread -> (q, r0) puts
// the 32 lanes of a half-wave on q = 8 h + 0..7, r0 = 4 g + 0..3, so their 4-B
// tile accesses (bank = row + column mod 32 with the 65-float row) fall on 32
// distinct banks in both phases (16 lanes x 16 q: 2-way conflicts)
__global__ void __launch_bounds__(256)
nchw_to_nhwc4_kernel(const float* __restrict__ in, float* __restrict__ out, int C, int HW, int gx, int gy) {
  __shared__ float tile[64][65];
  const TBlk tb = tblk(gx, gy);
  const int64_t b = tb.b;
  const int c0 = tb.cy * 64, p0 = tb.px * 64;
  const float* src = in + b * (int64_t)C * HW;
  float* dst = out + b * (int64_t)C * HW;
  const int t = threadIdx.x;
  const int q = (((t >> 5) & 1) << 3) | (t & 7), r0 = ((t >> 6) << 2) | ((t >> 3) & 3);
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + r0 + 16 * k, p = p0 + 4 * q;
    v[k] = (c < C && p < HW) ? *reinterpret_cast<const float4*>(src + (int64_t)c * HW + p)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float* t = &tile[r0 + 16 * k][4 * q];
    t[0] = v[k].x; t[1] = v[k].y; t[2] = v[k].z; t[3] = v[k].w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int pl = r0 + 16 * k, p = p0 + pl, c = c0 + 4 * q;
    if (p < HW && c < C)
      *reinterpret_cast<float4*>(dst + (int64_t)p * C + c) =
          make_float4(tile[4 * q][pl], tile[4 * q + 1][pl], tile[4 * q + 2][pl], tile[4 * q + 3][pl]);
  }
}

// Per-wave sample tables in registers: entry q of the y (x) table lives in
// lane q % 64, slot q / 64 (<= 2 slots: PH*gh, PW*gw <= 128).  Lookups in the
// bin loop are readlanes with a wave-uniform index, so the per-sample weights
// and tap offsets are scalar values and the loop issues LDS/VMEM traffic only
// for the taps themselves.
struct RegTab {
  int lo[2], hi[2], valid[2];
  float l[2], h[2];
};

__device__ __forceinline__ void tab_put(RegTab& t, int slot, const AxisTab& a) {
  t.lo[slot] = a.lo; t.hi[slot] = a.hi; t.valid[slot] = a.valid; t.l[slot] = a.l; t.h[slot] = a.h;
}

__device__ __forceinline__ AxisTab tab_get(const RegTab& t, int q) {
  const int ln = q & 63, sl = q >> 6;
  AxisTab a;
  if (sl == 0) {
    a.lo = __builtin_amdgcn_readlane(t.lo[0], ln);
    a.hi = __builtin_amdgcn_readlane(t.hi[0], ln);
    a.valid = __builtin_amdgcn_readlane(t.valid[0], ln);
    a.l = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.l[0]), ln));
    a.h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.h[0]), ln));
  } else {
    a.lo = __builtin_amdgcn_readlane(t.lo[1], ln);
    a.hi = __builtin_amdgcn_readlane(t.hi[1], ln);
    a.valid = __builtin_amdgcn_readlane(t.valid[1], ln);
    a.l = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.l[1]), ln));
    a.h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.h[1]), ln));
  }
  return a;
}

__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = min(x, __shfl_xor(x, o));
  return x;
}
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o));
  return x;
}

// tap source: the NHWC map in global memory (pixel (y,x) at (y*W+x)*C), or
// the ROI's source window staged in LDS (cell (y-y0, x-x0) at ((y-y0)*wx +
// (x-x0))*CPW).  `zero` is pixel (0,0), what torchvision reads for an empty
// sample (weights 0 at position 0 -- kept so NaN/inf propagate identically).
struct TapSrc {
  const float* base;
  const float* zero;
  int rstride, cstride, y0, x0;
};

template <int VEC, bool OUT_BF16>
__device__ __forceinline__ void store_nhwc(void* out, int64_t o, const float (&v)[VEC]) {
  if (OUT_BF16) {
    uint16_t* po = reinterpret_cast<uint16_t*>(out) + o;
    if constexpr (VEC == 4) {
      *reinterpret_cast<uint2*>(po) = make_uint2(trk::pack2_bf16(v[0], v[1]), trk::pack2_bf16(v[2], v[3]));
    } else if constexpr (VEC == 2) {
      *reinterpret_cast<uint32_t*>(po) = trk::pack2_bf16(v[0], v[1]);
    } else {
      po[0] = trk::f32_to_bf16(v[0]);
    }
  } else {
    float* po = reinterpret_cast<float*>(out) + o;
    if constexpr (VEC == 4) {
      *reinterpret_cast<float4*>(po) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (VEC == 2) {
      *reinterpret_cast<float2*>(po) = make_float2(v[0], v[1]);
    } else {
      po[0] = v[0];
    }
  }
}

template <int VEC, bool OUT_BF16, bool OUT_NHWC>
__device__ __forceinline__ void store_bin(void* out, float* otile, int lds_stride, int n, int bin,
                                          int nbins, int C, int c, int lane, const float (&v)[VEC]) {
  if (OUT_NHWC) {
    store_nhwc<VEC, OUT_BF16>(out, ((int64_t)n * nbins + bin) * C + c, v);
  } else if (lds_stride > 0) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) otile[(lane * VEC + k) * lds_stride + bin] = v[k];
  } else {  // NCHW without staging (large PH*PW): strided scalar stores
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int64_t o = ((int64_t)n * C + c + k) * nbins + bin;
      if (OUT_BF16) reinterpret_cast<uint16_t*>(out)[o] = trk::f32_to_bf16(v[k]);
      else reinterpret_cast<float*>(out)[o] = v[k];
    }
  }
}

// all bins of one (ROI, channel chunk) for one wave; exact torchvision order:
// per sample t = w1*f1; t += w2*f2; t += w3*f3; t += w4*f4; v += t; v /= count
template <int VEC, bool OUT_BF16, bool OUT_NHWC, int SR>
__device__ __forceinline__ void bins_loop(const TapSrc& src, const RegTab& yt, const RegTab& xt,
                                          int PH, int PW, int gh_rt, int gw_rt, float count, bool active,
                                          void* out, float* otile, int lds_stride, int n, int C,
                                          int c, int lane, int wave) {
  // SR > 0: compile-time sampling ratio -> the sample loops unroll and all
  // 4*SR*SR taps of a bin are in flight before the first use
  const int gh = SR > 0 ? SR : gh_rt, gw = SR > 0 ? SR : gw_rt;
  const int nbins = PH * PW;
  constexpr int UR = SR > 0 ? SR : 1;
  for (int bin = wave; bin < nbins; bin += 4) {
    const int ph = bin / PW, pw = bin % PW;
    float v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = 0.f;
#pragma unroll UR
    for (int iy = 0; iy < gh; ++iy) {
      const AxisTab ty = tab_get(yt, ph * gh + iy);
#pragma unroll UR
      for (int ix = 0; ix < gw; ++ix) {
        const AxisTab tx = tab_get(xt, pw * gw + ix);
        float w1, w2, w3, w4;
        const float *p1, *p2, *p3, *p4;
        if (ty.valid && tx.valid) {
          w1 = ty.h * tx.h; w2 = ty.h * tx.l; w3 = ty.l * tx.h; w4 = ty.l * tx.l;
          const float* r0 = src.base + (ty.lo - src.y0) * src.rstride;
          const float* r1 = src.base + (ty.hi - src.y0) * src.rstride;
          const int c0 = (tx.lo - src.x0) * src.cstride, c1 = (tx.hi - src.x0) * src.cstride;
          p1 = r0 + c0; p2 = r0 + c1; p3 = r1 + c0; p4 = r1 + c1;
        } else {
          w1 = w2 = w3 = w4 = 0.f;
          p1 = p2 = p3 = p4 = src.zero;
        }
        float f1[VEC], f2[VEC], f3[VEC], f4[VEC];
        load_vec<VEC>(p1, f1);
        load_vec<VEC>(p2, f2);
        load_vec<VEC>(p3, f3);
        load_vec<VEC>(p4, f4);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          float t = w1 * f1[k];
          t = t + w2 * f2[k];
          t = t + w3 * f3[k];
          t = t + w4 * f4[k];
          v[k] = v[k] + t;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = v[k] / count;
    if (active) store_bin<VEC, OUT_BF16, OUT_NHWC>(out, otile, lds_stride, n, bin, nbins, C, c, lane, v);
  }
}

template <int VEC, bool OUT_BF16, bool OUT_NHWC>
__global__ void __launch_bounds__(256)
roi_align_nhwc_kernel(const float* __restrict__ in,  // [B,H,W,C]
                      int B, int C, int H, int W,
                      const float* __restrict__ rois, int K, float spatial_scale,
                      int PH, int PW, int sampling_ratio, int aligned,
                      void* __restrict__ out, int nchunks, int lds_stride, int win_cells) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int CPW = 64 * VEC;  // channels per workgroup
  const int64_t nwg = (int64_t)K * nchunks;
  const int64_t lb = xcd_remap(blockIdx.x, nwg);
  const int n = (int)(lb / nchunks);
  const int chunk = (int)(lb % nchunks);
  // wave index and everything derived from the ROI are wave-uniform; say so
  // (readfirstlane) so the bin loop, the table lookups and the staged/direct
  // branch compile to scalar control flow instead of exec-masked branches
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const float* r = rois + (int64_t)n * 5;
  const int b = __builtin_amdgcn_readfirstlane((int)r[0]);
  const float off = aligned ? 0.5f : 0.0f;
  const float sw = r[1] * spatial_scale - off;
  const float sh = r[2] * spatial_scale - off;
  const float ew = r[3] * spatial_scale - off;
  const float eh = r[4] * spatial_scale - off;
  float rw = ew - sw, rh = eh - sh;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  const float bh = rh / (float)PH, bw = rw / (float)PW;
  const int gh = sampling_ratio, gw = sampling_ratio;  // > 0 (checked on the host)
  const float count = (float)max(gh * gw, 1);

  // ---- sample tables, per wave, in registers (pre_calc restated)
  const int ny = PH * gh, nx = PW * gw;
  RegTab yt, xt;
  int ylo = H, yhi = -1, xlo = W, xhi = -1;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int q = lane + 64 * sl;
    AxisTab a;
    a.lo = a.hi = a.valid = 0; a.l = a.h = 0.f;
    if (q < ny) {
      const int ph = q / gh, iy = q % gh;
      const float t0 = sh + (float)ph * bh;
      a = axis_sample(t0 + ((float)iy + .5f) * bh / (float)gh, H);
      if (a.valid) { ylo = min(ylo, a.lo); yhi = max(yhi, a.hi); }
    }
    tab_put(yt, sl, a);
    a.lo = a.hi = a.valid = 0; a.l = a.h = 0.f;
    if (q < nx) {
      const int pw = q / gw, ix = q % gw;
      const float s0 = sw + (float)pw * bw;
      a = axis_sample(s0 + ((float)ix + .5f) * bw / (float)gw, W);
      if (a.valid) { xlo = min(xlo, a.lo); xhi = max(xhi, a.hi); }
    }
    tab_put(xt, sl, a);
  }
  // source window of the valid samples (identical in every wave)
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min(ylo));
  const int y1 = __builtin_amdgcn_readfirstlane(wave_max(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min(xlo));
  const int x1 = __builtin_amdgcn_readfirstlane(wave_max(xhi));
  const int wy = max(y1 - y0 + 1, 0), wx = max(x1 - x0 + 1, 0);
  const bool staged = win_cells > 0 && wy * wx <= win_cells;

  // LDS: [NCHW output tile?][window: win_cells x CPW][pixel (0,0)]
  float* otile = reinterpret_cast<float*>(smem);
  float* win = otile + (OUT_NHWC || lds_stride == 0 ? 0 : (size_t)CPW * lds_stride);
  float* zcell = win + (size_t)win_cells * CPW;

  const int cbase = chunk * CPW;
  const int c = cbase + lane * VEC;
  const bool active = c < C;
  const float* img = in + (int64_t)b * H * W * C;
  TapSrc src;
  if (staged) {
    // whole 16-B pieces of each cell's CPW channels; the tail chunk (C not a
    // multiple of CPW) loads only channels < C
    constexpr int PPC = CPW / 4;  // float4 pieces per cell
    constexpr int BATCH = 8;      // pieces in flight per thread (no load->store chain)
    const int ncell = wy * wx;
    const int total = (ncell + 1) * PPC;
    for (int q0 = threadIdx.x; q0 < total; q0 += 256 * BATCH) {
      float4 tmp[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int q = min(q0 + 256 * k, total - 1);  // clamp: no data-dependent break
        const int cell = q / PPC, pc = (q % PPC) * 4;
        const int yy = cell < ncell ? y0 + cell / wx : 0, xx = cell < ncell ? x0 + cell % wx : 0;
        const float* sp = img + ((int64_t)yy * W + xx) * C + cbase + pc;
        if ((C & 3) == 0 && cbase + pc + 4 <= C) {
          tmp[k] = *reinterpret_cast<const float4*>(sp);
        } else {
          tmp[k].x = cbase + pc + 0 < C ? sp[0] : 0.f;
          tmp[k].y = cbase + pc + 1 < C ? sp[1] : 0.f;
          tmp[k].z = cbase + pc + 2 < C ? sp[2] : 0.f;
          tmp[k].w = cbase + pc + 3 < C ? sp[3] : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int q = q0 + 256 * k;
        if (q >= total) continue;
        const int cell = q / PPC, pc = (q % PPC) * 4;
        float* dst = cell < ncell ? win + (size_t)cell * CPW + pc : zcell + pc;
        *reinterpret_cast<float4*>(dst) = tmp[k];
      }
    }
    __syncthreads();
    src.base = win + lane * VEC;
    src.zero = zcell + lane * VEC;
    src.rstride = wx * CPW;
    src.cstride = CPW;
    src.y0 = y0;
    src.x0 = x0;
    if (sampling_ratio == 2)
      bins_loop<VEC, OUT_BF16, OUT_NHWC, 2>(src, yt, xt, PH, PW, gh, gw, count, active, out, otile,
                                            lds_stride, n, C, c, lane, wave);
    else
      bins_loop<VEC, OUT_BF16, OUT_NHWC, 0>(src, yt, xt, PH, PW, gh, gw, count, active, out, otile,
                                            lds_stride, n, C, c, lane, wave);
  } else {
    const int cc = active ? c : 0;
    src.base = img + cc;
    src.zero = img + cc;
    src.rstride = W * C;
    src.cstride = C;
    src.y0 = 0;
    src.x0 = 0;
    if (sampling_ratio == 2)
      bins_loop<VEC, OUT_BF16, OUT_NHWC, 2>(src, yt, xt, PH, PW, gh, gw, count, active, out, otile,
                                            lds_stride, n, C, c, lane, wave);
    else
      bins_loop<VEC, OUT_BF16, OUT_NHWC, 0>(src, yt, xt, PH, PW, gh, gw, count, active, out, otile,
                                            lds_stride, n, C, c, lane, wave);
  }
  if (!OUT_NHWC && lds_stride > 0) {
    __syncthreads();
    // out[n][chunk*CPW .. +nch][0..nbins) is one contiguous range
    const int nbins = PH * PW;
    const int nch = min(CPW, C - cbase);
    const int64_t base = ((int64_t)n * C + (int64_t)cbase) * nbins;
    const int total = nch * nbins;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const float val = otile[(e / nbins) * lds_stride + (e % nbins)];
      if (OUT_BF16) reinterpret_cast<uint16_t*>(out)[base + e] = trk::f32_to_bf16(val);
      else reinterpret_cast<float*>(out)[base + e] = val;
    }
  }
}

// ---------------------------------------------------------------------------
// Row-sweep kernel (NHWC output, sampling_ratio 2: the encoder / bench path).
//
// One wave = (ROI, bin row ph, 256*NH-channel chunk).  The x sample table is
// the same for every sample row and consecutive x samples mostly fall in the
// same pair of map columns, so the wave walks the bin row left to right and
// keeps, per sample row iy, the two current tap columns (rows ylo and yhi) in
// registers: a column is loaded only when a sample crosses into it (~6x fewer
// tap loads than 4 per sample for the reference's 1..10-cell ROIs; the
// per-sample-tap kernel above is L1/TA-bound).  The 2*PW samples are fully
// unrolled, so bin completion and store offsets are static.  Arithmetic is
// unchanged: t = w1*f1 + w2*f2 + w3*f3 + w4*f4 per sample in torchvision's
// order, samples added to the bin in (iy, ix) order (row iy = 1 held until
// row iy = 0 is in), times 1/4 (== / 4 exactly).  The math runs on float2
// pairs (v_pk_mul_f32 / v_pk_add_f32, separate mul and add: same rounding).
// Loads are buffer loads: the frame's map is one descriptor, the cell offset
// a scalar (soffset), the lane's channel offset the only per-lane part.
typedef float f2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff, f2_t (&v)[2]) {
  const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
  v[0] = f2_t{__uint_as_float(x[0]), __uint_as_float(x[1])};
  v[1] = f2_t{__uint_as_float(x[2]), __uint_as_float(x[3])};
}

// t = w1*f1 + w2*f2 + w3*f3 + w4*f4 (torchvision's order, no contraction); FMA: the
// same order with the three additions fused into their products (v_pk_fma_f32: 4
// instead of 7 packed ops per channel pair; each fused step rounds once instead of
// twice, so t moves by at most a few f32 ulp -- the bf16 fast path, see launch_sweep)
template <int NH, bool FMA>
__device__ __forceinline__ void sample4(f2_t (&t)[NH][2], float w1, float w2, float w3, float w4,
                                        const f2_t (&f1)[NH][2], const f2_t (&f2)[NH][2],
                                        const f2_t (&f3)[NH][2], const f2_t (&f4)[NH][2]) {
  const f2_t W1 = {w1, w1}, W2 = {w2, w2}, W3 = {w3, w3}, W4 = {w4, w4};
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      f2_t s = W1 * f1[h][p];
      if constexpr (FMA) {
        s = __builtin_elementwise_fma(W2, f2[h][p], s);
        s = __builtin_elementwise_fma(W3, f3[h][p], s);
        s = __builtin_elementwise_fma(W4, f4[h][p], s);
      } else {
        s = s + W2 * f2[h][p];
        s = s + W3 * f3[h][p];
        s = s + W4 * f4[h][p];
      }
      t[h][p] = s;
    }
}

// sample4 for one lane's 4 channels (NH = 1) as one asm block: the weights stay in the
// {w1, w2} / {w3, w4} pairs the LDS read returned and are broadcast by op_sel (the
// compiler copied w4 out of its pair before clobbering it, and kept nothing else in
// place), the two channel pairs' chains interleaved so every dependent packed op has
// one instruction between it and its producer (the gfx950 wait state the compiler
// otherwise pads with s_nop).  Same operations in the same order as sample4.
template <bool FMA>
__device__ __forceinline__ void sample4_asm(f2_t (&t)[1][2], f2_t w12, f2_t w34, const f2_t (&f1)[1][2],
                                            const f2_t (&f2)[1][2], const f2_t (&f3)[1][2],
                                            const f2_t (&f4)[1][2]) {
  if constexpr (FMA) {
    asm("v_pk_mul_f32 %0, %2, %4 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %1, %2, %5 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %6, %0 op_sel:[1,0,0]\n\t"
        "v_pk_fma_f32 %1, %2, %7, %1 op_sel:[1,0,0]\n\t"
        "v_pk_fma_f32 %0, %3, %8, %0 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %1, %3, %9, %1 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %0, %3, %10, %0 op_sel:[1,0,0]\n\t"
        "v_pk_fma_f32 %1, %3, %11, %1 op_sel:[1,0,0]\n\t"
        "s_nop 0"
        : "=&v"(t[0][0]), "=&v"(t[0][1])
        : "v"(w12), "v"(w34), "v"(f1[0][0]), "v"(f1[0][1]), "v"(f2[0][0]), "v"(f2[0][1]), "v"(f3[0][0]),
          "v"(f3[0][1]), "v"(f4[0][0]), "v"(f4[0][1]));
  } else {
    f2_t p0, p1;
    asm("v_pk_mul_f32 %0, %4, %6 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %1, %4, %7 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %2, %4, %8 op_sel:[1,0]\n\t"
        "v_pk_mul_f32 %3, %4, %9 op_sel:[1,0]\n\t"
        "v_pk_add_f32 %0, %0, %2\n\t"
        "v_pk_add_f32 %1, %1, %3\n\t"
        "v_pk_mul_f32 %2, %5, %10 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %3, %5, %11 op_sel_hi:[0,1]\n\t"
        "v_pk_add_f32 %0, %0, %2\n\t"
        "v_pk_add_f32 %1, %1, %3\n\t"
        "v_pk_mul_f32 %2, %5, %12 op_sel:[1,0]\n\t"
        "v_pk_mul_f32 %3, %5, %13 op_sel:[1,0]\n\t"
        "v_pk_add_f32 %0, %0, %2\n\t"
        "v_pk_add_f32 %1, %1, %3\n\t"
        "s_nop 0"
        : "=&v"(t[0][0]), "=&v"(t[0][1]), "=&v"(p0), "=&v"(p1)
        : "v"(w12), "v"(w34), "v"(f1[0][0]), "v"(f1[0][1]), "v"(f2[0][0]), "v"(f2[0][1]), "v"(f3[0][0]),
          "v"(f3[0][1]), "v"(f4[0][0]), "v"(f4[0][1]));
  }
}

// floor(n / d) for n < 2^31, 0 < d < 2^31, m = udiv_magic_m(d) = floor(2^32 / d) + 1:
// mulhi(n, m) is q or q + 1 (n * (m - 2^32 / d) < 2^31 * 1 < 2^32), one correction step.
// d == 1 has no 32-bit multiplier (2^32 + 1 truncates to 1), so it is a separate
// (wave-uniform, scalar) branch; its m is unused.
__host__ __device__ inline uint32_t udiv_magic_m(uint32_t d) {
  return d > 1 ? (uint32_t)((1ull << 32) / d + 1) : 0u;
}
__device__ __forceinline__ uint32_t udiv_magic(uint32_t n, uint32_t d, uint32_t m) {
  if (d == 1) return n;
  uint32_t q = __umulhi(n, m);
  if (q * d > n) --q;
  return q;
}

// Two-column register cache of one sample row: columns ca (a*) and cb (b*)
// at rows ylo (*0) and yhi (*1).
template <int NH>
struct ColCache2 {
  f2_t a0[NH][2], a1[NH][2], b0[NH][2], b1[NH][2];
  int ca, cb;
};

template <int NH>
__device__ __forceinline__ void cache_load(f2_t (&v0)[NH][2], f2_t (&v1)[NH][2], __amdgpu_buffer_rsrc_t rs,
                                           const int (&voff)[NH], int s0, int s1) {
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    bload4(rs, voff[h], s0, v0[h]);
    bload4(rs, voff[h], s1, v1[h]);
  }
}

template <int NH, bool OUT_BF16, int PW, bool g_sweep_wlds, bool FMA, bool g_sweep_asm>
__global__ void __launch_bounds__(256)
roi_sweep_kernel(const float* __restrict__ in,  // [B,H,W,C]
                 int C, int H, int W, const float* __restrict__ rois, float spatial_scale,
                 int PH, int aligned, void* __restrict__ out, int nchunks, int64_t nitems, uint32_t mch,
                 uint32_t mph) {
  constexpr int CPW = 256 * NH, NS = 2 * PW;
  static_assert(NS <= 64, "one x sample per lane");
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // per-wave sample weight table: [x sample][y sample] = {w1, w2, w3, w4}, read back
  // with a wave-uniform address (an LDS broadcast instead of four readlanes)
  __shared__ float4 wtab[4][NS][2];
  const int64_t item = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
  if (item >= nitems) return;  // wave-uniform (no barriers below)
  // item = (n * PH + ph) * nchunks + chunk < 2^31: scalar divisions by the host's
  // magic multipliers (udiv_magic) instead of the VALU division sequences
  const uint32_t it = (uint32_t)item;
  const uint32_t t_ = udiv_magic(it, (uint32_t)nchunks, mch);
  const int chunk = (int)(it - t_ * (uint32_t)nchunks);
  const uint32_t n_ = udiv_magic(t_, (uint32_t)PH, mph);
  const int ph = (int)(t_ - n_ * (uint32_t)PH);
  const int n = (int)n_;

  const float* r = rois + (int64_t)n * 5;
  const int b = __builtin_amdgcn_readfirstlane((int)r[0]);
  const float off = aligned ? 0.5f : 0.0f;
  const float sw = r[1] * spatial_scale - off;
  const float sh = r[2] * spatial_scale - off;
  const float ew = r[3] * spatial_scale - off;
  const float eh = r[4] * spatial_scale - off;
  float rw = ew - sw, rh = eh - sh;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  const float bh = rh / (float)PH, bw = rw / (float)PW;

  // the two y samples of this bin row (uniform)
  int so[2][2], yv[2];
  float yl[2], yh[2];
  const float t0 = sh + (float)ph * bh;
  const int rowb = W * C * 4, colb = C * 4;
#pragma unroll
  for (int iy = 0; iy < 2; ++iy) {
    const AxisTab a = axis_sample(t0 + ((float)iy + .5f) * bh / 2.0f, H);
    so[iy][0] = __builtin_amdgcn_readfirstlane(a.lo) * rowb;
    so[iy][1] = __builtin_amdgcn_readfirstlane(a.hi) * rowb;
    yv[iy] = __builtin_amdgcn_readfirstlane(a.valid);
    yl[iy] = a.l;
    yh[iy] = a.h;
  }
  // lane q = x sample q (pre_calc restated): packed lo | hi << 12 | valid << 24
  // and the sample's four weights for each y sample (the same float products)
  int xpk;
  float wq[2][4];
  {
    AxisTab a;
    a.lo = a.hi = a.valid = 0; a.l = a.h = 0.f;
    if (lane < NS) {
      const int pw = lane >> 1, ix = lane & 1;
      const float s0 = sw + (float)pw * bw;
      a = axis_sample(s0 + ((float)ix + .5f) * bw / 2.0f, W);
    }
    xpk = a.lo | (a.hi << 12) | (a.valid << 24);
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
      wq[iy][0] = yh[iy] * a.h; wq[iy][1] = yh[iy] * a.l;
      wq[iy][2] = yl[iy] * a.h; wq[iy][3] = yl[iy] * a.l;
      if (g_sweep_wlds && lane < NS) wtab[wave][lane][iy] = make_float4(wq[iy][0], wq[iy][1], wq[iy][2], wq[iy][3]);
    }
  }

  // the frame's map as one buffer (descriptor inputs readfirstlane'd so the
  // compiler can prove it uniform -- otherwise every buffer op is a waterfall)
  const uint64_t fa = reinterpret_cast<uint64_t>(in + (int64_t)b * H * W * C);
  const uint32_t fa_lo = __builtin_amdgcn_readfirstlane((uint32_t)fa);
  const uint32_t fa_hi = __builtin_amdgcn_readfirstlane((uint32_t)(fa >> 32));
  const int nbytes = __builtin_amdgcn_readfirstlane(H * W * C * 4);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)fa_hi << 32) | fa_lo), 0, nbytes, 0x00020000);
  int voff[NH];
  bool act[NH];
  const int cbase = chunk * CPW;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int c = cbase + h * 256 + lane * 4;
    act[h] = c < C;
    voff[h] = (act[h] ? c : 0) * 4;
  }
  f2_t zero[NH][2];  // pixel (0,0): what torchvision reads for an empty sample
#pragma unroll
  for (int h = 0; h < NH; ++h) bload4(rs, voff[h], 0, zero[h]);
  if (FMA) {
    // FMA: an empty sample is 0 * pixel(0,0) + 0: +0 for a finite pixel, NaN for a NaN / Inf
    // one, as torchvision's 0-weight sum of four pixel(0,0) reads (after its `0 + t`)
    const f2_t Z0 = {0.f, 0.f};
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int p = 0; p < 2; ++p) zero[h][p] = zero[h][p] * Z0 + Z0;
  }

  ColCache2<NH> kc[2];
  kc[0].ca = kc[0].cb = kc[1].ca = kc[1].cb = -1;
  // the wave's weight table as an opaque VGPR address: read with immediate offsets, not
  // rematerialised from its SGPR before every read
  uint32_t wtab_va = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)&wtab[wave][0][0]);
  if (g_sweep_asm) asm volatile("" : "+v"(wtab_va));
  const f2_t Z = {0.f, 0.f}, Q = {0.25f, 0.25f};
  f2_t acc[NH][2], hold[NH][2];
  // the wave's output row (PW bins x C channels) as one buffer: the bin's offset is a
  // scalar (soffset), the lane's channel offset the only per-lane part -- no 64-bit
  // address arithmetic per store
  constexpr int EB = OUT_BF16 ? 2 : 4;
  const uint64_t oa = reinterpret_cast<uint64_t>(out) + ((((uint64_t)n * PH + ph) * PW) * C) * EB;
  // (readfirstlane returns int: both halves go through uint32_t, or a set bit 31 of the
  // low half would sign-extend into the high one)
  const uint32_t oa_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)oa);
  const uint32_t oa_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(oa >> 32));
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)oa_hi << 32) | oa_lo), 0, __builtin_amdgcn_readfirstlane(PW * C * EB),
      0x00020000);
  int ovoff[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    ovoff[h] = (cbase + h * 256 + lane * 4) * EB;
    if (g_sweep_asm) asm volatile("" : "+v"(ovoff[h]));  // kept in a VGPR, not recomputed per store
  }

  auto sweep = [&](auto same_c) {
    constexpr bool SAME = decltype(same_c)::value;
  #pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int pk = __builtin_amdgcn_readlane(xpk, j);
      const int lo = pk & 0xfff, hi = (pk >> 12) & 0xfff, xv = pk >> 24;
      f2_t t[2][NH][2];
  #pragma unroll
      for (int iy = 0; iy < 2; ++iy) {
        if (yv[iy] && xv) {
          // SAME: both sample rows read the same two map rows -- one column cache serves
          // both, updated by the first
          ColCache2<NH>& k = kc[SAME ? 0 : iy];
          if (!(SAME && iy == 1) && lo != k.ca) {
            if (lo == k.cb) {
  #pragma unroll
              for (int h = 0; h < NH; ++h)
  #pragma unroll
                for (int p = 0; p < 2; ++p) { k.a0[h][p] = k.b0[h][p]; k.a1[h][p] = k.b1[h][p]; }
            } else {
              cache_load<NH>(k.a0, k.a1, rs, voff, so[iy][0] + lo * colb, so[iy][1] + lo * colb);
            }
            k.ca = lo;
          }
          if (!(SAME && iy == 1) && hi != k.cb) {
            if (hi == k.ca) {
  #pragma unroll
              for (int h = 0; h < NH; ++h)
  #pragma unroll
                for (int p = 0; p < 2; ++p) { k.b0[h][p] = k.a0[h][p]; k.b1[h][p] = k.a1[h][p]; }
            } else {
              cache_load<NH>(k.b0, k.b1, rs, voff, so[iy][0] + hi * colb, so[iy][1] + hi * colb);
            }
            k.cb = hi;
          }
          float w1, w2, w3, w4;
          if (g_sweep_wlds && NH == 1 && g_sweep_asm) {
            typedef float f4_t __attribute__((ext_vector_type(4)));
            const f4_t w = ((const __attribute__((address_space(3))) f4_t*)(uintptr_t)wtab_va)[j * 2 + iy];
            sample4_asm<FMA>(reinterpret_cast<f2_t (&)[1][2]>(t[iy]), f2_t{w.x, w.y}, f2_t{w.z, w.w},
                             reinterpret_cast<const f2_t (&)[1][2]>(k.a0), reinterpret_cast<const f2_t (&)[1][2]>(k.b0),
                             reinterpret_cast<const f2_t (&)[1][2]>(k.a1), reinterpret_cast<const f2_t (&)[1][2]>(k.b1));
            continue;
          }
          if (g_sweep_wlds) {
            const float4 w = wtab[wave][j][iy];
            w1 = w.x; w2 = w.y; w3 = w.z; w4 = w.w;
          } else {
            w1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wq[iy][0]), j));
            w2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wq[iy][1]), j));
            w3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wq[iy][2]), j));
            w4 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wq[iy][3]), j));
          }
          sample4<NH, FMA>(t[iy], w1, w2, w3, w4, k.a0, k.b0, k.a1, k.b1);
        } else {
          if (FMA) {
  #pragma unroll
            for (int h = 0; h < NH; ++h) { t[iy][h][0] = zero[h][0]; t[iy][h][1] = zero[h][1]; }
          } else {
            sample4<NH, FMA>(t[iy], 0.f, 0.f, 0.f, 0.f, zero, zero, zero, zero);
          }
        }
      }
      if ((j & 1) == 0) {
  #pragma unroll
        for (int h = 0; h < NH; ++h)
  #pragma unroll
          for (int p = 0; p < 2; ++p) {
            acc[h][p] = FMA ? t[0][h][p] : Z + t[0][h][p];  // (0 + t: torchvision's -0 -> +0)
            hold[h][p] = t[1][h][p];
          }
      } else {
  #pragma unroll
        for (int h = 0; h < NH; ++h) {
          float v[4];
  #pragma unroll
          for (int p = 0; p < 2; ++p) {
            f2_t s = acc[h][p] + t[0][h][p];
            s = s + hold[h][p];
            s = s + t[1][h][p];
            s = s * Q;  // == s / 4 exactly (power of two)
            v[2 * p] = s.x;
            v[2 * p + 1] = s.y;
          }
          if (act[h]) {
            const int so_ = __builtin_amdgcn_readfirstlane((j >> 1) * C * EB);
            if constexpr (OUT_BF16) {
              typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
              __builtin_amdgcn_raw_buffer_store_b64(u32x2{trk::pack2_bf16(v[0], v[1]), trk::pack2_bf16(v[2], v[3])},
                                                    ors, ovoff[h], so_, ROI_OUT_POLICY);
            } else {
              typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
              __builtin_amdgcn_raw_buffer_store_b128(u32x4_{__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                            __float_as_uint(v[2]), __float_as_uint(v[3])},
                                                     ors, ovoff[h], so_, ROI_OUT_POLICY);
            }
          }
        }
      }
    }
  };
  // the bin row's two sample rows usually fall between the same two map rows
  const bool same = yv[0] && yv[1] && so[0][0] == so[1][0] && so[0][1] == so[1][1];
  if (g_sweep_asm && same) sweep(std::true_type{});
  else sweep(std::false_type{});
}

// tuning knobs (trk_set_tuning): LDS window budget per workgroup, channels per lane
int g_roi_window_kb = 0;   // measured r01: direct L2 taps beat LDS window staging (229 vs 300+ us)
int g_roi_vec = 0;  // 0 = auto
int g_roi_sweep = 1;  // NHWC output: row-sweep kernel, 256 (1) or 512 (2) channels per wave
int g_roi_asm = 1;    // row sweep: the bilinear sample as one asm block (sample4_asm) and one column
                      // cache for a bin row whose two sample rows share their map rows (92 vs 100 us)
int g_roi_fma = 1;    // row sweep, bf16 output: fused multiply-adds in the bilinear sample (see sample4;
                      // 75 vs 92 us; 0 = the exact torchvision arithmetic, as f32 output always is)
int g_roi_wlds = 1;   // row sweep: sample weights from an LDS table (1: r02 A/B 97 vs 104 us) or readlanes (0)

template <int VEC, bool OUT_BF16, bool OUT_NHWC>
int launch_roi(const float* nhwc, int B, int C, int H, int W, const float* rois, int K,
               float scale, int PH, int PW, int sr, int aligned, void* out, hipStream_t st) {
  constexpr int CPW = 64 * VEC;
  const int nchunks = (C + CPW - 1) / CPW;
  int lds_stride = 0;
  size_t lds = 0;
  if (!OUT_NHWC) {
    const int stride = PH * PW + 1;  // +1: bank-conflict padding
    const size_t need = sizeof(float) * (size_t)CPW * stride;
    if (need <= 64 * 1024) {
      lds_stride = stride;
      lds = need;
    }
  }
  const size_t cell_bytes = sizeof(float) * CPW;
  const size_t budget = (size_t)g_roi_window_kb * 1024;
  int win_cells = lds + 2 * cell_bytes <= budget ? (int)((budget - lds) / cell_bytes) - 1 : 0;
  win_cells = std::min(win_cells, H * W);
  if (win_cells > 0) lds += cell_bytes * (size_t)(win_cells + 1);
  if (lds > 160 * 1024) {
    trk::set_error("roi_align: LDS request %zu too large", lds);
    return TRK_EUNSUPPORTED;
  }
  const int64_t nwg = (int64_t)K * nchunks;
  if (nwg > 0x7fffffff) {
    trk::set_error("roi_align: too many workgroups");
    return TRK_EUNSUPPORTED;
  }
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB dynamic LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(roi_align_nhwc_kernel<VEC, OUT_BF16, OUT_NHWC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL((roi_align_nhwc_kernel<VEC, OUT_BF16, OUT_NHWC>), dim3((unsigned)nwg), dim3(256),
                     lds, st, nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, nchunks,
                     lds_stride, win_cells);
  return trk::check_launch("roi_align_nhwc_kernel");
}

template <int NH, bool OUT_BF16, int PW>
int launch_sweep(const float* nhwc, int C, int H, int W, const float* rois, int K, float scale, int PH,
                 int aligned, void* out, hipStream_t st) {
  const int nchunks = (C + 256 * NH - 1) / (256 * NH);
  const int64_t nitems = (int64_t)K * PH * nchunks;
  const int64_t nwg = (nitems + 3) / 4;
  const uint32_t mch = udiv_magic_m((uint32_t)nchunks), mph = udiv_magic_m((uint32_t)PH);
  if (nitems >= ((int64_t)1 << 31)) {
    trk::set_error("roi_align: too many workgroups");
    return TRK_EUNSUPPORTED;
  }
  // roi_fma (bf16 output only; f32 output is always the exact arithmetic)
#define TRK_SWEEP(WL, F, A)                                                                                    \
  hipLaunchKernelGGL((roi_sweep_kernel<NH, OUT_BF16, PW, WL, F, A>), dim3((unsigned)nwg), dim3(256), 0, st, nhwc, \
                     C, H, W, rois, scale, PH, aligned, out, nchunks, nitems, mch, mph)
  if (OUT_BF16 && g_roi_fma) {
    if (g_roi_asm) TRK_SWEEP(true, OUT_BF16, true);
    else TRK_SWEEP(true, OUT_BF16, false);
  } else if (g_roi_wlds) {
    if (g_roi_asm) TRK_SWEEP(true, false, true);
    else TRK_SWEEP(true, false, false);
  } else {
    TRK_SWEEP(false, false, false);
  }
#undef TRK_SWEEP
  return trk::check_launch("roi_sweep_kernel");
}

template <bool OUT_BF16, int PW>
int dispatch_sweep(const float* nhwc, int C, int H, int W, const float* rois, int K, float scale, int PH,
                   int aligned, void* out, hipStream_t st) {
  if (g_roi_sweep == 2) return launch_sweep<2, OUT_BF16, PW>(nhwc, C, H, W, rois, K, scale, PH, aligned, out, st);
  return launch_sweep<1, OUT_BF16, PW>(nhwc, C, H, W, rois, K, scale, PH, aligned, out, st);
}

template <bool OUT_BF16, bool OUT_NHWC>
int dispatch_vec(int C, const float* nhwc, int B, int H, int W, const float* rois, int K, float scale,
                 int PH, int PW, int sr, int aligned, void* out, hipStream_t st) {
  int vec = g_roi_vec;
  if (vec == 0) vec = g_roi_window_kb > 0 ? 2 : 4;  // window: 8-B conflict-free LDS taps; direct: 16-B taps
  if (vec == 4 && C % 4 == 0)
    return launch_roi<4, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, st);
  if (vec >= 2 && C % 2 == 0)
    return launch_roi<2, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, st);
  return launch_roi<1, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, st);
}

}  // namespace

extern "C" int trk_set_tuning(const char* key, int value) {
  TRK_REQUIRE(key, "set_tuning: null key");
  if (!strcmp(key, "roi_window_kb")) { TRK_REQUIRE(value >= 0 && value <= 150, "roi_window_kb in [0,150]"); g_roi_window_kb = value; return TRK_OK; }
  if (!strcmp(key, "roi_sweep")) { TRK_REQUIRE(value >= 0 && value <= 2, "roi_sweep in {0,1,2}"); g_roi_sweep = value; return TRK_OK; }
  if (!strcmp(key, "se_waves")) { extern int g_se_waves; TRK_REQUIRE(value == 8 || value == 16, "se_waves in {8, 16}"); g_se_waves = value; return TRK_OK; }
  if (!strcmp(key, "head_waves")) { extern int g_head_waves; TRK_REQUIRE(value == 8 || value == 16, "head_waves in {8, 16}"); g_head_waves = value; return TRK_OK; }
  if (!strcmp(key, "roi_asm")) { TRK_REQUIRE(value == 0 || value == 1, "roi_asm in {0, 1}"); g_roi_asm = value; return TRK_OK; }
  if (!strcmp(key, "roi_fma")) { TRK_REQUIRE(value == 0 || value == 1, "roi_fma in {0, 1}"); g_roi_fma = value; return TRK_OK; }
  if (!strcmp(key, "roi_wlds")) { TRK_REQUIRE(value == 0 || value == 1, "roi_wlds in {0, 1}"); g_roi_wlds = value; return TRK_OK; }
  if (!strcmp(key, "cost_v2")) { extern int g_cost_v2; TRK_REQUIRE(value == 0 || value == 1, "cost_v2 in {0, 1}"); g_cost_v2 = value; return TRK_OK; }
  if (!strcmp(key, "rf_pf")) { extern int g_rf_pf; TRK_REQUIRE(value == 0 || value == 1, "rf_pf in {0, 1}"); g_rf_pf = value; return TRK_OK; }
  if (!strcmp(key, "cost_split")) { extern int g_cost_split; TRK_REQUIRE(value == 0 || value == 1, "cost_split in {0, 1}"); g_cost_split = value; return TRK_OK; }
  if (!strcmp(key, "enc_trans")) { extern int g_enc_trans; TRK_REQUIRE(value == 0 || value == 1, "enc_trans in {0, 1}"); g_enc_trans = value; return TRK_OK; }
  if (!strcmp(key, "rf3_chunks")) { extern int g_rf3_chunks; TRK_REQUIRE(value >= 1 && value <= 64, "rf3_chunks in 1..64"); g_rf3_chunks = value; return TRK_OK; }
  if (!strcmp(key, "rf3_groups")) { extern int g_rf3_groups; TRK_REQUIRE(value >= 0 && value <= 64, "rf3_groups in 0..64"); g_rf3_groups = value; return TRK_OK; }
  if (!strcmp(key, "dw_fast")) { extern int g_dw_fast; TRK_REQUIRE(value == 0 || value == 1, "dw_fast in {0,1}"); g_dw_fast = value; return TRK_OK; }
  if (!strcmp(key, "lsap_dev_lds_kb")) { extern int g_lsap_dev_lds_kb; TRK_REQUIRE(value >= 8 && value <= 156, "lsap_dev_lds_kb in [8, 156]"); g_lsap_dev_lds_kb = value; return TRK_OK; }
  if (!strcmp(key, "roi_vec")) { TRK_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, "roi_vec in {0,1,2,4}"); g_roi_vec = value; return TRK_OK; }
  trk::set_error("set_tuning: unknown key '%s'", key);
  return TRK_EINVAL;
}

extern "C" size_t trk_roi_align_workspace_bytes(int64_t B, int64_t C, int64_t H, int64_t W, int in_layout) {
  if (in_layout == TRK_NHWC) return 0;
  return (size_t)(B * C * H * W) * sizeof(float);
}

extern "C" int trk_nchw_to_nhwc(const float* in, int64_t B, int64_t C, int64_t H, int64_t W, float* out,
                                void* stream) {
  TRK_REQUIRE(B >= 1 && C >= 1 && H >= 1 && W >= 1 && B * C * H * W < (int64_t)1 << 31,
              "nchw_to_nhwc: bad shape [%lld,%lld,%lld,%lld]", (long long)B, (long long)C, (long long)H, (long long)W);
  TRK_REQUIRE(in && out, "nchw_to_nhwc: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t HW = H * W;
  const int gx = (int)((HW + 63) / 64), gy = (int)((C + 63) / 64);
  TRK_REQUIRE((int64_t)gx * gy * B < ((int64_t)1 << 31), "nchw_to_nhwc: too many blocks");
  const dim3 grid((unsigned)((int64_t)gx * gy * B));
  if (HW % 4 == 0 && C % 4 == 0 && trk::aligned16_ptr(in) && trk::aligned16_ptr(out)) {
    hipLaunchKernelGGL(nchw_to_nhwc4_kernel, grid, dim3(256), 0, st, in, out, (int)C, (int)HW, gx, gy);
    return trk::check_launch("nchw_to_nhwc4_kernel");
  }
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid, dim3(256), 0, st, in, out, C, HW, gx, gy);
  return trk::check_launch("nchw_to_nhwc_kernel");
}

extern "C" int trk_roi_align_fwd(const float* input, int64_t B, int64_t C, int64_t H, int64_t W,
                                 int in_layout, const float* rois, int64_t K, float spatial_scale,
                                 int PH, int PW, int sampling_ratio, int aligned, void* out,
                                 int out_dtype, int out_layout, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  TRK_REQUIRE(B >= 1 && C >= 1 && H >= 1 && W >= 1, "roi_align: bad input shape [%lld,%lld,%lld,%lld]",
              (long long)B, (long long)C, (long long)H, (long long)W);
  TRK_REQUIRE(K >= 0, "roi_align: negative K");
  TRK_REQUIRE(PH >= 1 && PW >= 1, "roi_align: output_size must be positive");
  TRK_REQUIRE(in_layout == TRK_NCHW || in_layout == TRK_NHWC, "roi_align: bad in_layout");
  TRK_REQUIRE(out_layout == TRK_NCHW || out_layout == TRK_NHWC, "roi_align: bad out_layout");
  TRK_REQUIRE(out_dtype == TRK_F32 || out_dtype == TRK_BF16, "roi_align: out dtype must be f32 or bf16");
  TRK_REQUIRE(B * H * W * C < (int64_t)1 << 31, "roi_align: input too large for 32-bit pixel offsets");
  if (K == 0) return TRK_OK;
  TRK_REQUIRE(input && rois && out, "roi_align: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const float* nhwc = input;
  if (in_layout == TRK_NCHW) {
    TRK_REQUIRE(workspace && workspace_bytes >= trk_roi_align_workspace_bytes(B, C, H, W, in_layout),
                "roi_align: NCHW input needs a workspace of %zu bytes",
                trk_roi_align_workspace_bytes(B, C, H, W, in_layout));
    if (int e = trk_nchw_to_nhwc(input, B, C, H, W, reinterpret_cast<float*>(workspace), stream)) return e;
    nhwc = reinterpret_cast<const float*>(workspace);
  }
  // gh/gw for adaptive sampling depend on each ROI; size the LDS tables for the
  // largest ROI on the host only when sampling_ratio <= 0 (not used by the
  // reference, which always passes 2).
  TRK_REQUIRE(sampling_ratio > 0,
              "roi_align: adaptive sampling (sampling_ratio <= 0) is not implemented; the reference uses 2");
  TRK_REQUIRE(PH * sampling_ratio <= 128 && PW * sampling_ratio <= 128,
              "roi_align: output_size x sampling_ratio must be <= 128 per axis");
  const int iB = (int)B, iC = (int)C, iH = (int)H, iW = (int)W, iK = (int)K;
  const bool bf = out_dtype == TRK_BF16, nhwc_out = out_layout == TRK_NHWC;
  if (nhwc_out && g_roi_sweep && iC % 4 == 0 && sampling_ratio == 2 && (PW == 10 || PW == 7) && iH < 4096 &&
      iW < 4096 && (int64_t)iH * iW * iC < ((int64_t)1 << 29)) {
    if (PW == 10)
      return bf ? dispatch_sweep<true, 10>(nhwc, iC, iH, iW, rois, iK, spatial_scale, PH, aligned, out, st)
                : dispatch_sweep<false, 10>(nhwc, iC, iH, iW, rois, iK, spatial_scale, PH, aligned, out, st);
    return bf ? dispatch_sweep<true, 7>(nhwc, iC, iH, iW, rois, iK, spatial_scale, PH, aligned, out, st)
              : dispatch_sweep<false, 7>(nhwc, iC, iH, iW, rois, iK, spatial_scale, PH, aligned, out, st);
  }
  if (bf && nhwc_out) return dispatch_vec<true, true>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, st);
  if (bf && !nhwc_out) return dispatch_vec<true, false>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, st);
  if (!bf && nhwc_out) return dispatch_vec<false, true>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, st);
  return dispatch_vec<false, false>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, st);
}
