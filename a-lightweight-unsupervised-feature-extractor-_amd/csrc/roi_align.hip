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

__global__ void __launch_bounds__(256)
nchw_to_nhwc_kernel(const float* __restrict__ in, float* __restrict__ out,
                    int64_t C, int64_t HW) {
  // tile: 64 channels x 64 pixels through LDS; blockIdx.z = batch
  __shared__ float tile[64][65];
  const int64_t b = blockIdx.z;
  const int64_t c0 = (int64_t)blockIdx.y * 64, p0 = (int64_t)blockIdx.x * 64;
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

template <int VEC, bool OUT_BF16, bool OUT_NHWC>
__global__ void __launch_bounds__(256)
roi_align_nhwc_kernel(const float* __restrict__ in,  // [B,H,W,C]
                      int B, int C, int H, int W,
                      const float* __restrict__ rois, int K, float spatial_scale,
                      int PH, int PW, int sampling_ratio, int aligned,
                      void* __restrict__ out, int nchunks, int lds_stride) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int CPW = 64 * VEC;  // channels per workgroup
  const int64_t nwg = (int64_t)K * nchunks;
  const int64_t lb = xcd_remap(blockIdx.x, nwg);
  const int n = (int)(lb / nchunks);
  const int chunk = (int)(lb % nchunks);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  const float* r = rois + (int64_t)n * 5;
  const int b = (int)r[0];
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
  const int gh = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rh / (float)PH);
  const int gw = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rw / (float)PW);
  const float count = (float)max(gh * gw, 1);

  // sample tables (LDS): y then x
  AxisTab* ytab = reinterpret_cast<AxisTab*>(smem);
  AxisTab* xtab = ytab + PH * gh;
  float* otile = reinterpret_cast<float*>(xtab + PW * gw);  // NCHW staging
  for (int q = threadIdx.x; q < PH * gh + PW * gw; q += blockDim.x) {
    if (q < PH * gh) {
      int ph = q / gh, iy = q % gh;
      float t0 = sh + (float)ph * bh;
      float yy = t0 + ((float)iy + .5f) * bh / (float)gh;
      ytab[q] = axis_sample(yy, H);
    } else {
      int q2 = q - PH * gh;
      int pw = q2 / gw, ix = q2 % gw;
      float s0 = sw + (float)pw * bw;
      float xx = s0 + ((float)ix + .5f) * bw / (float)gw;
      xtab[q2] = axis_sample(xx, W);
    }
  }
  __syncthreads();

  const int c = chunk * CPW + lane * VEC;
  const bool active = c < C;
  const float* img = in + (int64_t)b * H * W * C + (active ? c : 0);
  const int nbins = PH * PW;
  for (int bin = wave; bin < nbins; bin += 4) {
    const int ph = bin / PW, pw = bin % PW;
    float v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = 0.f;
    for (int iy = 0; iy < gh; ++iy) {
      const AxisTab ty = ytab[ph * gh + iy];
      for (int ix = 0; ix < gw; ++ix) {
        const AxisTab tx = xtab[pw * gw + ix];
        float w1, w2, w3, w4;
        int p1, p2, p3, p4;
        if (ty.valid && tx.valid) {
          w1 = ty.h * tx.h; w2 = ty.h * tx.l; w3 = ty.l * tx.h; w4 = ty.l * tx.l;
          p1 = ty.lo * W + tx.lo; p2 = ty.lo * W + tx.hi;
          p3 = ty.hi * W + tx.lo; p4 = ty.hi * W + tx.hi;
        } else {  // torchvision's empty PreCalc: weights 0 at position 0
          w1 = w2 = w3 = w4 = 0.f;
          p1 = p2 = p3 = p4 = 0;
        }
        float f1[VEC], f2[VEC], f3[VEC], f4[VEC];
        load_vec<VEC>(img + (int64_t)p1 * C, f1);
        load_vec<VEC>(img + (int64_t)p2 * C, f2);
        load_vec<VEC>(img + (int64_t)p3 * C, f3);
        load_vec<VEC>(img + (int64_t)p4 * C, f4);
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
    if (!active) continue;
    if (OUT_NHWC) {
      const int64_t o = ((int64_t)n * nbins + bin) * C + c;
      if (OUT_BF16) {
        uint16_t* po = reinterpret_cast<uint16_t*>(out) + o;
#pragma unroll
        for (int k = 0; k < VEC; ++k) po[k] = trk::f32_to_bf16(v[k]);
      } else {
        float* po = reinterpret_cast<float*>(out) + o;
        if constexpr (VEC == 4) {
          *reinterpret_cast<float4*>(po) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int k = 0; k < VEC; ++k) po[k] = v[k];
        }
      }
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
  if (!OUT_NHWC && lds_stride > 0) {
    __syncthreads();
    // out[n][chunk*CPW .. +nch][0..nbins) is one contiguous range
    const int nch = min(CPW, C - chunk * CPW);
    const int64_t base = ((int64_t)n * C + (int64_t)chunk * CPW) * nbins;
    const int total = nch * nbins;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const float val = otile[(e / nbins) * lds_stride + (e % nbins)];
      if (OUT_BF16) reinterpret_cast<uint16_t*>(out)[base + e] = trk::f32_to_bf16(val);
      else reinterpret_cast<float*>(out)[base + e] = val;
    }
  }
}

template <int VEC, bool OUT_BF16, bool OUT_NHWC>
int launch_roi(const float* nhwc, int B, int C, int H, int W, const float* rois, int K,
               float scale, int PH, int PW, int sr, int aligned, void* out, int gh, int gw,
               hipStream_t st) {
  constexpr int CPW = 64 * VEC;
  const int nchunks = (C + CPW - 1) / CPW;
  size_t tab = sizeof(AxisTab) * (size_t)(PH * gh + PW * gw);
  tab = (tab + 15) & ~size_t(15);
  int lds_stride = 0;
  size_t lds = tab;
  if (!OUT_NHWC) {
    const int stride = PH * PW + 1;  // +1: bank-conflict padding
    const size_t need = tab + sizeof(float) * (size_t)CPW * stride;
    if (need <= 96 * 1024) {
      lds_stride = stride;
      lds = need;
    }
  }
  if (lds > 160 * 1024) {
    trk::set_error("roi_align: sample tables too large (PH*gh + PW*gw = %d)", PH * gh + PW * gw);
    return TRK_EUNSUPPORTED;
  }
  const int64_t nwg = (int64_t)K * nchunks;
  if (nwg > 0x7fffffff) {
    trk::set_error("roi_align: too many workgroups");
    return TRK_EUNSUPPORTED;
  }
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB dynamic LDS for the NCHW staging tile
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(roi_align_nhwc_kernel<VEC, OUT_BF16, OUT_NHWC>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL((roi_align_nhwc_kernel<VEC, OUT_BF16, OUT_NHWC>), dim3((unsigned)nwg), dim3(256),
                     lds, st, nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, nchunks,
                     lds_stride);
  return trk::check_launch("roi_align_nhwc_kernel");
}

template <bool OUT_BF16, bool OUT_NHWC>
int dispatch_vec(int C, const float* nhwc, int B, int H, int W, const float* rois, int K, float scale,
                 int PH, int PW, int sr, int aligned, void* out, int gh, int gw, hipStream_t st) {
  // NHWC output: 4 channels per lane (16-B loads, 1 KiB per wave-instruction).
  // NCHW output: 2 channels per lane keeps the [128][PH*PW+1] staging tile small.
  if (OUT_NHWC && C % 4 == 0)
    return launch_roi<4, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, gh, gw, st);
  if (C % 2 == 0)
    return launch_roi<2, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, gh, gw, st);
  return launch_roi<1, OUT_BF16, OUT_NHWC>(nhwc, B, C, H, W, rois, K, scale, PH, PW, sr, aligned, out, gh, gw, st);
}

}  // namespace

extern "C" size_t trk_roi_align_workspace_bytes(int64_t B, int64_t C, int64_t H, int64_t W, int in_layout) {
  if (in_layout == TRK_NHWC) return 0;
  return (size_t)(B * C * H * W) * sizeof(float);
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
    const int64_t HW = H * W;
    dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)B);
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid, dim3(256), 0, st, input,
                       reinterpret_cast<float*>(workspace), C, HW);
    if (int e = trk::check_launch("nchw_to_nhwc_kernel")) return e;
    nhwc = reinterpret_cast<const float*>(workspace);
  }
  // gh/gw for adaptive sampling depend on each ROI; size the LDS tables for the
  // largest ROI on the host only when sampling_ratio <= 0 (not used by the
  // reference, which always passes 2).
  int gh = sampling_ratio, gw = sampling_ratio;
  TRK_REQUIRE(sampling_ratio > 0,
              "roi_align: adaptive sampling (sampling_ratio <= 0) is not implemented; the reference uses 2");
  const int iB = (int)B, iC = (int)C, iH = (int)H, iW = (int)W, iK = (int)K;
  const bool bf = out_dtype == TRK_BF16, nhwc_out = out_layout == TRK_NHWC;
  if (bf && nhwc_out) return dispatch_vec<true, true>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, gh, gw, st);
  if (bf && !nhwc_out) return dispatch_vec<true, false>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, gh, gw, st);
  if (!bf && nhwc_out) return dispatch_vec<false, true>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, gh, gw, st);
  return dispatch_vec<false, false>(iC, nhwc, iB, iH, iW, rois, iK, spatial_scale, PH, PW, sampling_ratio, aligned, out, gh, gw, st);
}
