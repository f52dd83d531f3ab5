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

namespace {

typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int RB = 16;        // ROIs per workgroup
constexpr int NWAVE = 8;
constexpr int MAXC = 1024;    // channel bound (LDS sizing)

// acc[t] (t < nt) += X[16][K] . W[n0 + 16 t .. + 15][K]^T
__device__ __forceinline__ void rb_gemm4(const float* __restrict__ Xs, int ldx, const float* __restrict__ W,
                                         int64_t ldw, int n0, int nt, int K, f4_t (&acc)[4]) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const float* wp[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) wp[t] = W + (int64_t)(n0 + 16 * min(t, nt - 1) + r) * ldw + 4 * g;
  const float* xp = Xs + r * ldx + 4 * g;
#pragma unroll 2
  for (int kb = 0; kb < K; kb += 16) {
    const float4 a = *reinterpret_cast<const float4*>(xp + kb);
    float4 b[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = *reinterpret_cast<const float4*>(wp[t] + kb);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[t].x, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[t].y, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[t].z, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[t].w, acc[t], 0, 0, 0);
      }
    }
  }
}

// Y[16][N] = epi(X[16][K] . W[N][K]^T + bias) into LDS (ldy), tiles spread over
// the 8 waves in runs of <= 4.  epi(col, v) is applied per element.
template <class Epi>
__device__ __forceinline__ void rb_linear(const float* Xs, int ldx, const float* W, const float* bias, int N,
                                          int K, float* Ys, int ldy, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntile = N / 16;
  const int per = (ntile + NWAVE - 1) / NWAVE;
  const int t_begin = wave * per, t_end = min(ntile, t_begin + per);
  for (int t0 = t_begin; t0 < t_end; t0 += 4) {
    const int nt = min(4, t_end - t0);
    f4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f4_t{0.f, 0.f, 0.f, 0.f};
    rb_gemm4(Xs, ldx, W, K, t0 * 16, nt, K, acc);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt) {
        const int col = (t0 + t) * 16 + (lane & 15);
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * (lane >> 4) + i;
          Ys[row * ldy + col] = epi(col, acc[t][i] + bv);
        }
      }
    }
  }
}

__device__ __forceinline__ float fix_mean(long long v, float P) {
  // (sums.double() * 2^-24).float() / P, as ops.enc_dsc_gemm + the encoder do
  return (float)((double)v * (1.0 / 16777216.0)) / P;
}

struct SeArgs {
  const long long* sums;
  int64_t ld_sums;
  const float *w1, *b1, *w2, *b2;
  float *m_r, *m_n, *s;
  int R, C, H;
  float P;
};

__global__ void __launch_bounds__(512) enc_se_kernel(const SeArgs a) {
  extern __shared__ __align__(16) float lds[];
  const int C = a.C, H = a.H, ldx = C + 4, ldh = H + 4;
  float* Xs = lds;                 // [16][C + 4] m_r
  float* Hs = lds + RB * ldx;      // [16][H + 4] relu(W1 m_r + b1)
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int nrow = (int)min<int64_t>(RB, a.R - r0);
  for (int q = threadIdx.x; q < RB * C; q += blockDim.x) {
    const int rr = q / C, c = q % C;
    float mr = 0.f;
    if (rr < nrow) {
      const long long* sp = a.sums + (r0 + rr) * a.ld_sums;
      mr = fix_mean(sp[c], a.P);
      a.m_r[(r0 + rr) * C + c] = mr;
      a.m_n[(r0 + rr) * C + c] = fix_mean(sp[C + c], a.P);
    }
    Xs[rr * ldx + c] = mr;
  }
  __syncthreads();
  rb_linear(Xs, ldx, a.w1, a.b1, H, C, Hs, ldh, [](int, float v) { return fmaxf(v, 0.f); });
  __syncthreads();
  // hardsigmoid (torch: min(max(x + 3, 0), 6) / 6), straight to global
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntile = C / 16, per = (ntile + NWAVE - 1) / NWAVE;
  const int t_begin = wave * per, t_end = min(ntile, t_begin + per);
  for (int t0 = t_begin; t0 < t_end; t0 += 4) {
    const int nt = min(4, t_end - t0);
    f4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f4_t{0.f, 0.f, 0.f, 0.f};
    rb_gemm4(Hs, ldh, a.w2, H, t0 * 16, nt, H, acc);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt) {
        const int col = (t0 + t) * 16 + (lane & 15);
        const float bv = a.b2[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * (lane >> 4) + i;
          if (row < nrow) a.s[(r0 + row) * C + col] = fminf(fmaxf(acc[t][i] + bv + 3.0f, 0.f), 6.0f) / 6.0f;
        }
      }
    }
  }
}

struct HeadArgs {
  const long long* tsums;
  const float *s, *m_r, *m_n;
  const float *w0, *ln_w, *ln_b, *w4, *b4;
  float* out;
  int R, C, D;
  float P, eps;
  double alpha;
};

__global__ void __launch_bounds__(512) enc_head_kernel(const HeadArgs a) {
  extern __shared__ __align__(16) float lds[];
  const int C = a.C, D = a.D, ldx = C + 4, ldd = D + 4;
  float* Gs = lds;                  // [16][C + 4] g, then silu(LN(z))
  float* Zs = lds + RB * ldx;       // [16][C + 4] z = W0 g
  float* Ys = Zs + RB * ldx;        // [16][D + 4] W4 . + b4
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int nrow = (int)min<int64_t>(RB, a.R - r0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float al = (float)a.alpha, bl = (float)(1.0 - a.alpha);  // torch: a * (.), (1 - a) * (.)
  for (int q = threadIdx.x; q < RB * C; q += blockDim.x) {
    const int rr = q / C, c = q % C;
    float gv = 0.f;
    if (rr < nrow) {
      const int64_t o = (r0 + rr) * C + c;
      const float mcat = fix_mean(a.tsums[o], a.P);
      const float x2 = al * (a.s[o] * a.m_r[o]) + bl * a.m_n[o];
      gv = 0.5f * mcat + 0.5f * x2;
    }
    Gs[rr * ldx + c] = gv;
  }
  __syncthreads();
  rb_linear(Gs, ldx, a.w0, nullptr, C, C, Zs, ldx, [](int, float v) { return v; });
  __syncthreads();
  // LayerNorm over C (biased variance, eps inside the sqrt) + SiLU: wave w owns rows 2w, 2w + 1
  for (int rr = 2 * wave; rr < 2 * wave + 2; ++rr) {
    const float* z = Zs + rr * ldx;
    float sum = 0.f;
    for (int c = lane; c < C; c += 64) sum += z[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float mean = sum / (float)C;
    float sq = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = z[c] - mean;
      sq += d * d;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    const float rstd = 1.0f / sqrtf(sq / (float)C + a.eps);
    for (int c = lane; c < C; c += 64) {
      const float y = (z[c] - mean) * rstd * a.ln_w[c] + a.ln_b[c];
      Gs[rr * ldx + c] = y / (1.0f + expf(-y));
    }
  }
  __syncthreads();
  rb_linear(Gs, ldx, a.w4, a.b4, D, C, Ys, ldd, [](int, float v) { return v; });
  __syncthreads();
  // F.normalize(dim=1): y / max(||y||, 1e-12)
  for (int rr = 2 * wave; rr < 2 * wave + 2; ++rr) {
    const float* y = Ys + rr * ldd;
    float sq = 0.f;
    for (int c = lane; c < D; c += 64) sq += y[c] * y[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    const float nrm = fmaxf(sqrtf(sq), 1e-12f);
    if (rr < nrow)
      for (int c = lane; c < D; c += 64) a.out[(r0 + rr) * D + c] = y[c] / nrm;
  }
}

}  // namespace

extern "C" int trk_enc_se(const long long* sums, int64_t R, int64_t ld_sums, int64_t P, int64_t C,
                          const float* w1, const float* b1, int64_t H, const float* w2, const float* b2,
                          float* m_r, float* m_n, float* s, void* stream) {
  TRK_REQUIRE(R >= 0 && P > 0 && C > 0 && C % 16 == 0 && C <= MAXC && H > 0 && H % 16 == 0 && H <= MAXC &&
                  ld_sums >= 2 * C,
              "enc_se: need C, H multiples of 16 in [16, %d], ld_sums >= 2C", MAXC);
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(sums && w1 && b1 && w2 && b2 && m_r && m_n && s, "enc_se: null pointer");
  SeArgs a{sums, ld_sums, w1, b1, w2, b2, m_r, m_n, s, (int)R, (int)C, (int)H, (float)P};
  const size_t lds = (size_t)RB * ((C + 4) + (H + 4)) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_se_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(enc_se_kernel, dim3((unsigned)((R + RB - 1) / RB)), dim3(64 * NWAVE), lds,
                     reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("enc_se_kernel");
}

extern "C" int trk_enc_head(const long long* tsums, int64_t R, int64_t P, int64_t C, const float* s,
                            const float* m_r, const float* m_n, double alpha, const float* w0, const float* ln_w,
                            const float* ln_b, float ln_eps, const float* w4, const float* b4, int64_t D,
                            float* out, void* stream) {
  TRK_REQUIRE(R >= 0 && P > 0 && C > 0 && C % 16 == 0 && C <= MAXC && D > 0 && D % 16 == 0 && D <= MAXC,
              "enc_head: need C, D multiples of 16 in [16, %d]", MAXC);
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(tsums && s && m_r && m_n && w0 && ln_w && ln_b && w4 && b4 && out, "enc_head: null pointer");
  HeadArgs a{tsums, s, m_r, m_n, w0, ln_w, ln_b, w4, b4, out, (int)R, (int)C, (int)D, (float)P, ln_eps, alpha};
  const size_t lds = (size_t)RB * (2 * (C + 4) + (D + 4)) * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_head_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(enc_head_kernel, dim3((unsigned)((R + RB - 1) / RB)), dim3(64 * NWAVE), lds,
                     reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("enc_head_kernel");
}
