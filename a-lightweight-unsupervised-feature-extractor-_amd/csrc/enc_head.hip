// Per-ROI tail of the encoder for gfx950: the work between / after the big
// GEMMs, one kernel each instead of ~25 small torch launches.
//
//   enc_se_kernel    squeeze means from the int64 ROI sums of trk_enc_dsc_gemm
//                    (m_r = mean SiLU(x_r), m_n = mean Hardswish(x_n)) and the SE
//                    excitation s = hardsigmoid(W2 relu(W1 m_r + b1) + b2)
//                    (reference model/utils/modules/card.py:59-78, SEBlock)
//   enc_head_kernel  Shake2 eval mix g = 0.5 m_cat + 0.5 (a (s m_r) + (1-a) m_n)
//                    (card.py:83-96, RMB.forward :128-148) and the projection head
//                    normalize(W4 silu(LN(W0 g)) + b4) (card.py:151-169)
//
// Workgroup = 16 ROIs, 8 waves.  The small f32 GEMMs run on
// v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation): the 16 ROI
// rows are the A operand (from LDS), each wave owns up to 4 column tiles of 16
// outputs whose weight rows it streams from L2.  Within each 16-wide K block,
// lane group g = lane >> 4 takes k = 4g + t at MFMA t (t = 0..3) for BOTH
// operands, so every lane reads 16 contiguous bytes of its A row and of its
// weight row (the sum's order is permuted, not its terms).
#include "trk_common.h"
#include "rb_linear.h"

trk::DiagBuf g_head_prof;  // trk_head_set_prof (diagnostics)
int g_head_waves = 16;  // trk_set_tuning("head_waves"): enc_head workgroup of 8 or 16 waves
int g_se_waves = 16;    // trk_set_tuning("se_waves"): enc_se workgroup of 8 or 16 waves (16: 26 vs 29 us)

namespace {

__device__ __forceinline__ unsigned long long hd_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// number of 128-row GEMM tiles covering ROI roi (its partial sums, trk_amd.h)
__device__ __forceinline__ int part_count(int64_t roi, int P) {
  return (int)((roi * P + P - 1) / 128 - roi * P / 128) + 1;
}

__device__ __forceinline__ float fix_mean(long long v, float P) {
  // (sums.double() * 2^-24).float() / P, as ops.enc_dsc_gemm + the encoder do
  return (float)((double)v * (1.0 / 16777216.0)) / P;
}

struct SeArgs {
  const float* means;  // trk_enc_se_means: m_r rows given (sums unused, m_r / m_n not written)
  const long long* sums;
  int64_t ld_sums;
  const float *w1, *b1, *w2, *b2;
  float *m_r, *m_n, *s;
  int R, C, H, Pi;
  float P;
};

template <int NW>
__global__ void __launch_bounds__(64 * NW) enc_se_kernel(const SeArgs a) {
  extern __shared__ __align__(16) float lds[];
  const int C = a.C, H = a.H, ldx = ld_rows(C), ldh = ld_rows(H);
  float* Xs = lds;                 // [16][ldx] m_r (swz_at rows)
  float* Hs = lds + RB * ldx;      // [16][ldh] relu(W1 m_r + b1)
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int nrow = (int)min<int64_t>(RB, a.R - r0);
  // 4 channels per item, all of a thread's loads in flight together
  const int C4 = C / 4;
#pragma unroll 4
  for (int q = threadIdx.x; q < RB * C4; q += blockDim.x) {
    const int rr = q / C4, c = (q % C4) * 4;
    float4 mr = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.means) {
      if (rr < nrow) mr = *reinterpret_cast<const float4*>(a.means + (r0 + rr) * C + c);
    } else if (rr < nrow) {
      // the ROI's 1..3 partial sums (one per 128-row tile of the DSC GEMM)
      const int64_t roi = r0 + rr;
      const int cnt = part_count(roi, a.Pi);
      longlong2 r01 = {0, 0}, r23 = {0, 0}, n01 = {0, 0}, n23 = {0, 0};
      for (int j = 0; j < cnt; ++j) {
        const long long* __restrict__ sp = a.sums + (roi * TRK_ENC_PARTS + j) * a.ld_sums + c;
        const longlong2 x0 = *reinterpret_cast<const longlong2*>(sp);
        const longlong2 x1 = *reinterpret_cast<const longlong2*>(sp + 2);
        const longlong2 y0 = *reinterpret_cast<const longlong2*>(sp + C);
        const longlong2 y1 = *reinterpret_cast<const longlong2*>(sp + C + 2);
        r01.x += x0.x; r01.y += x0.y; r23.x += x1.x; r23.y += x1.y;
        n01.x += y0.x; n01.y += y0.y; n23.x += y1.x; n23.y += y1.y;
      }
      mr = make_float4(fix_mean(r01.x, a.P), fix_mean(r01.y, a.P), fix_mean(r23.x, a.P), fix_mean(r23.y, a.P));
      *reinterpret_cast<float4*>(a.m_r + (r0 + rr) * C + c) = mr;
      *reinterpret_cast<float4*>(a.m_n + (r0 + rr) * C + c) =
          make_float4(fix_mean(n01.x, a.P), fix_mean(n01.y, a.P), fix_mean(n23.x, a.P), fix_mean(n23.y, a.P));
    }
    *reinterpret_cast<float4*>(Xs + swz_at(rr, c, ldx)) = mr;
  }
  __syncthreads();
  rb_linear<NW>(Xs, ldx, a.w1, a.b1, H, C, [&](int row, int col, float v) { Hs[swz_at(row, col, ldh)] = fmaxf(v, 0.f); });
  __syncthreads();
  // hardsigmoid (torch: min(max(x + 3, 0), 6) / 6), straight to global
  float* __restrict__ sout = a.s;
  rb_linear<NW>(Hs, ldh, a.w2, a.b2, C, H, [&](int row, int col, float v) {
    if (row < nrow) sout[(r0 + row) * C + col] = fminf(fmaxf(v + 3.0f, 0.f), 6.0f) / 6.0f;
  });
}

// LayerNorm over C (biased variance, eps inside the sqrt) + SiLU of rows w, w + NW, ...
// of Zs into Gs.  Lane-strided columns c = lane + 64 q (q < QL, QL * 64 >= C) held in
// registers; the affine parameters are loaded once per wave, all in flight together.
// Sums run in ascending q per lane, then the xor tree: the order of the plain loop.
template <int NW, int QL>
__device__ __forceinline__ void ln_silu_rows(const float* Zs, float* Gs, int ldx, int C, const float* ln_w,
                                             const float* ln_b, float eps) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float lw[QL], lb[QL];
#pragma unroll
  for (int q = 0; q < QL; ++q) {
    const int c = lane + 64 * q;
    lw[q] = c < C ? ln_w[c] : 0.f;
    lb[q] = c < C ? ln_b[c] : 0.f;
  }
  for (int rr = wave; rr < RB; rr += NW) {
    float zv[QL];
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < QL; ++q) {
      const int c = lane + 64 * q;
      zv[q] = c < C ? Zs[swz_at(rr, c, ldx)] : 0.f;
      if (c < C) sum += zv[q];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float mean = sum / (float)C;
    float sq = 0.f;
#pragma unroll
    for (int q = 0; q < QL; ++q) {
      const float d = zv[q] - mean;
      if (lane + 64 * q < C) sq += d * d;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    const float rstd = 1.0f / sqrtf(sq / (float)C + eps);
#pragma unroll
    for (int q = 0; q < QL; ++q) {
      const int c = lane + 64 * q;
      if (c < C) {
        const float y = (zv[q] - mean) * rstd * lw[q] + lb[q];
        Gs[swz_at(rr, c, ldx)] = y / (1.0f + expf(-y));
      }
    }
  }
}

struct HeadArgs {
  const long long* tsums;
  const float *s, *m_r, *m_n;
  const float *w0, *ln_w, *ln_b, *w4, *b4;
  float* out;
  int R, C, D, Pi;
  float P, eps;
  double alpha;
  unsigned long long* prof;  // per wave [prologue, W0, LN, W4, normalize] (diagnostics)
};

template <int NW>
__global__ void __launch_bounds__(64 * NW) enc_head_kernel(const HeadArgs a) {
  extern __shared__ __align__(16) float lds[];
  const int C = a.C, D = a.D, ldx = ld_rows(C), ldd = ld_rows(D);
  float* Gs = lds;                  // [16][ldx] g, then silu(LN(z)) (swz_at rows)
  float* Zs = lds + RB * ldx;       // [16][ldx] z = W0 g
  float* Ys = Zs + RB * ldx;        // [16][ldd] W4 . + b4
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int nrow = (int)min<int64_t>(RB, a.R - r0);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float al = (float)a.alpha, bl = (float)(1.0 - a.alpha);  // torch: a * (.), (1 - a) * (.)
  unsigned long long pt[6] = {0, 0, 0, 0, 0, 0};
  if (a.prof) pt[0] = hd_stamp();
  const int C4 = C / 4;
#pragma unroll 4
  for (int q = threadIdx.x; q < RB * C4; q += blockDim.x) {
    const int rr = q / C4, c = (q % C4) * 4;
    float gv[4] = {0.f, 0.f, 0.f, 0.f};
    if (rr < nrow) {
      const int64_t o = (r0 + rr) * C + c;
      const int cnt = part_count(r0 + rr, a.Pi);
      longlong2 t01 = {0, 0}, t23 = {0, 0};
      for (int j = 0; j < cnt; ++j) {
        const long long* __restrict__ tp = a.tsums + ((r0 + rr) * TRK_ENC_PARTS + j) * C + c;
        const longlong2 x0 = *reinterpret_cast<const longlong2*>(tp);
        const longlong2 x1 = *reinterpret_cast<const longlong2*>(tp + 2);
        t01.x += x0.x; t01.y += x0.y; t23.x += x1.x; t23.y += x1.y;
      }
      const float4 sv = *reinterpret_cast<const float4*>(a.s + o);
      const float4 rv = *reinterpret_cast<const float4*>(a.m_r + o);
      const float4 nv = *reinterpret_cast<const float4*>(a.m_n + o);
      const long long tv[4] = {t01.x, t01.y, t23.x, t23.y};
      const float s4[4] = {sv.x, sv.y, sv.z, sv.w}, r4[4] = {rv.x, rv.y, rv.z, rv.w};
      const float n4[4] = {nv.x, nv.y, nv.z, nv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mcat = fix_mean(tv[e], a.P);
        const float x2 = al * (s4[e] * r4[e]) + bl * n4[e];
        gv[e] = 0.5f * mcat + 0.5f * x2;
      }
    }
    *reinterpret_cast<float4*>(Gs + swz_at(rr, c, ldx)) = make_float4(gv[0], gv[1], gv[2], gv[3]);
  }
  __syncthreads();
  if (a.prof) pt[1] = hd_stamp();
  rb_linear<NW>(Gs, ldx, a.w0, nullptr, C, C, [&](int row, int col, float v) { Zs[swz_at(row, col, ldx)] = v; });
  __syncthreads();
  if (a.prof) pt[2] = hd_stamp();
  // LayerNorm over C (biased variance, eps inside the sqrt) + SiLU: wave w owns rows w, w + NW, ...
  if constexpr (NW == 16) {  // launched for C <= 512 only (register budget)
    ln_silu_rows<NW, 8>(Zs, Gs, ldx, C, a.ln_w, a.ln_b, a.eps);
  } else {
    if (C <= 512) ln_silu_rows<NW, 8>(Zs, Gs, ldx, C, a.ln_w, a.ln_b, a.eps);
    else ln_silu_rows<NW, MAXC / 64>(Zs, Gs, ldx, C, a.ln_w, a.ln_b, a.eps);
  }
  __syncthreads();
  if (a.prof) pt[3] = hd_stamp();
  rb_linear<NW>(Gs, ldx, a.w4, a.b4, D, C, [&](int row, int col, float v) { Ys[swz_at(row, col, ldd)] = v; });
  __syncthreads();
  if (a.prof) pt[4] = hd_stamp();
  // F.normalize(dim=1): y / max(||y||, 1e-12)
  for (int rr = wave; rr < RB; rr += NW) {
    float sq = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float yc = Ys[swz_at(rr, c, ldd)];
      sq += yc * yc;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    const float nrm = fmaxf(sqrtf(sq), 1e-12f);
    if (rr < nrow)
      for (int c = lane; c < D; c += 64) a.out[(r0 + rr) * D + c] = Ys[swz_at(rr, c, ldd)] / nrm;
  }
  if (a.prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pt[5] = hd_stamp();
    if (lane == 0) {
      unsigned long long* o = a.prof + ((int64_t)blockIdx.x * 16 + wave) * 5;
#pragma unroll
      for (int q = 0; q < 5; ++q) o[q] = pt[q + 1] - pt[q];
    }
  }
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

namespace {
int se_launch(const SeArgs& a, void* stream) {
  const size_t lds = (size_t)RB * (ld_rows(a.C) + ld_rows(a.H)) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_se_kernel<8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_se_kernel<16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const unsigned nwg = (unsigned)((a.R + RB - 1) / RB);
  if (g_se_waves == 16)
    hipLaunchKernelGGL(enc_se_kernel<16>, dim3(nwg), dim3(64 * 16), lds, reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(enc_se_kernel<8>, dim3(nwg), dim3(64 * 8), lds, reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("enc_se_kernel");
}
}  // namespace

extern "C" int trk_enc_se(const long long* sums, int64_t R, int64_t ld_sums, int64_t P, int64_t C,
                          const float* w1, const float* b1, int64_t H, const float* w2, const float* b2,
                          float* m_r, float* m_n, float* s, void* stream) {
  TRK_REQUIRE(R >= 0 && P > 0 && P <= 256 && C > 0 && C % 16 == 0 && C <= MAXC && H > 0 && H % 16 == 0 && H <= MAXC &&
                  ld_sums >= 2 * C && ld_sums % 2 == 0,
              "enc_se: need C, H multiples of 16 in [16, %d], ld_sums >= 2C and even", MAXC);
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(sums && w1 && b1 && w2 && b2 && m_r && m_n && s, "enc_se: null pointer");
  TRK_REQUIRE(al16(sums) && al16(w1) && al16(w2) && al16(m_r) && al16(m_n) && al16(s),
              "enc_se: operands must be 16-byte aligned");
  SeArgs a{nullptr, sums, ld_sums, w1, b1, w2, b2, m_r, m_n, s, (int)R, (int)C, (int)H, (int)P, (float)P};
  return se_launch(a, stream);
}

extern "C" int trk_enc_se_means(const float* m_r, int64_t R, int64_t C, const float* w1, const float* b1, int64_t H,
                                const float* w2, const float* b2, float* s, void* stream) {
  TRK_REQUIRE(R >= 0 && C > 0 && C % 16 == 0 && C <= MAXC && H > 0 && H % 16 == 0 && H <= MAXC,
              "enc_se_means: need C, H multiples of 16 in [16, %d]", MAXC);
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(m_r && w1 && b1 && w2 && b2 && s, "enc_se_means: null pointer");
  TRK_REQUIRE(al16(m_r) && al16(w1) && al16(w2) && al16(s), "enc_se_means: operands must be 16-byte aligned");
  SeArgs a{m_r, nullptr, 0, w1, b1, w2, b2, nullptr, nullptr, s, (int)R, (int)C, (int)H, 1, 1.f};
  return se_launch(a, stream);
}

extern "C" int trk_enc_head(const long long* tsums, int64_t R, int64_t P, int64_t C, const float* s,
                            const float* m_r, const float* m_n, double alpha, const float* w0, const float* ln_w,
                            const float* ln_b, float ln_eps, const float* w4, const float* b4, int64_t D,
                            float* out, void* stream) {
  TRK_REQUIRE(R >= 0 && P > 0 && P <= 256 && C > 0 && C % 16 == 0 && C <= MAXC && D > 0 && D % 16 == 0 &&
                  D <= MAXC,
              "enc_head: need P <= 256, C, D multiples of 16 in [16, %d]", MAXC);
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(tsums && s && m_r && m_n && w0 && ln_w && ln_b && w4 && b4 && out, "enc_head: null pointer");
  TRK_REQUIRE(al16(tsums) && al16(s) && al16(m_r) && al16(m_n) && al16(w0) && al16(w4),
              "enc_head: operands must be 16-byte aligned");
  HeadArgs a{tsums, s, m_r, m_n, w0, ln_w, ln_b, w4, b4, out, (int)R, (int)C, (int)D, (int)P, (float)P, ln_eps, alpha,
             g_head_prof.get()};
  const size_t lds = (size_t)RB * (2 * ld_rows((int)C) + ld_rows((int)D)) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_head_kernel<8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_head_kernel<16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (g_head_waves == 16 && C <= 512)
    hipLaunchKernelGGL(enc_head_kernel<16>, dim3((unsigned)((R + RB - 1) / RB)), dim3(64 * 16), lds,
                       reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(enc_head_kernel<8>, dim3((unsigned)((R + RB - 1) / RB)), dim3(64 * 8), lds,
                       reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("enc_head_kernel");
}

// diagnostics: enc_head per-wave s_memtime phases (u64 x 5 per wave, 8 waves per
// 16-ROI workgroup); NULL = off
extern "C" int trk_head_set_prof(unsigned long long* buf) {
  g_head_prof.set(buf);
  return TRK_OK;
}
