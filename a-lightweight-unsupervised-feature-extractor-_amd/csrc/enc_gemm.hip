// Fused bf16 GEMMs of the encoder's RMB (reference model/utils/modules/card.py:
// DSC :48-57, SEBlock :73-78, RMB.forward :128-148) for gfx950.
//
// C = A . B^T on MFMA 32x32x16 bf16 (f32 accumulate), A = activation rows
// [M, K] (row stride lda), B = weights [N, K] (the conv weight's natural
// [out, in] layout, K contiguous).  Workgroup tile 128 x 128 (kBM x kBN), BK = 32,
// 8 waves as 2 (M) x 4 (N), each wave 64 x 32 (two 32x32 accumulators; 256 x
// 256 tiles measured slower: the accumulators spill at 2 waves/SIMD); A and B tiles
// are register-staged into a double-buffered, row-padded LDS image (80-B rows:
// the 16-B fragment reads of the 32 rows of a tile spread over all banks).
//
// Epilogues replace the elementwise passes of the unfused graph:
//   DSC pair  (EPI 0): both DSC 1x1 GEMMs of the RMB in one launch (group 0 =
//       reinforce, 1 = normal); + BN-folded bias; stores x_r (pre-activation,
//       SiLU is applied by the transition's prologue) / Hardswish(x_n) into the
//       [x_r | x_n] rows; accumulates per-ROI column sums of SiLU(x_r) (SE
//       squeeze) and Hardswish(x_n) (GAP).
//   transition (EPI 1): A prologue applies SiLU(x_r) * s[roi] (SE excitation)
//       to the first kscale columns while staging; epilogue + bias, SiLU,
//       per-ROI column sums only (the GAP is all the head needs; T is never
//       written).
// Per-ROI sums are int64 fixed point (2^-24) updated with 64-bit atomics:
// exact integer addition, so the result does not depend on the order in
// which tiles finish (deterministic run to run).
#include "trk_common.h"

namespace {

typedef __bf16 bf8_t __attribute__((ext_vector_type(8)));
typedef float f16_t __attribute__((ext_vector_type(16)));

constexpr int BK = 32, LDK = BK + 8;  // padded LDS row: 80 B
constexpr float kFix = 16777216.0f;  // 2^24

struct EncGemmArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;       // [groups][N][K]
  const float* bias;       // [groups * N]
  uint16_t* C;             // EPI 0 output, row stride ldc, group g at column g * N
  int64_t ldc;
  long long* sums;         // [nroi][ld_sums]: group g's columns at g * N
  int ld_sums;
  const float* scale;      // EPI 1: s [nroi][kscale]
  int M, N, K, P, groups, kscale;
};

// bf16-path activations: hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32), a
// few ulp of f32 -- far below the bf16 rounding these kernels feed
__device__ __forceinline__ float silu_f(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * v));
}
__device__ __forceinline__ float hswish_f(float v) {
  return v * fminf(fmaxf(v + 3.0f, 0.0f), 6.0f) * (1.0f / 6.0f);
}

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t nx = 8;
  if (nwg < nx) return bid;
  int64_t q = nwg / nx, r = nwg % nx, x = bid % nx;
  int64_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return (uint32_t)trk::f32_to_bf16(a) | ((uint32_t)trk::f32_to_bf16(b) << 16);
}

// EPI 1 prologue on one staged 16-B piece (8 consecutive k of one row)
__device__ __forceinline__ uint4 silu_scale_piece(uint4 v, const float* s8) {
  const float4 s0 = *reinterpret_cast<const float4*>(s8);
  const float4 s1 = *reinterpret_cast<const float4*>(s8 + 4);
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = __uint_as_float(w[q] << 16), b = __uint_as_float(w[q] & 0xffff0000u);
    w[q] = pack_bf16x2(silu_f(a) * sv[2 * q], silu_f(b) * sv[2 * q + 1]);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int EPI, int BM, int BN>
__global__ void __launch_bounds__(512) enc_gemm_kernel(EncGemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 4, TM = WM / 32, TN = WN / 32;  // 8 waves: 2 (M) x 4 (N)
  constexpr int APT = BM / 128, BPT = BN / 128;                          // 16-B pieces per thread
  __shared__ __align__(16) uint16_t As[2][BM * LDK];
  __shared__ __align__(16) uint16_t Bs[2][BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntile_n = a.N / BN;
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = (int)(lb % (ntile_n * a.groups));
  const int64_t mt = lb / (ntile_n * a.groups);
  const int g = nt / ntile_n, n0 = (nt % ntile_n) * BN;
  const int64_t m0 = mt * BM;
  const uint16_t* Ag = a.A + (int64_t)g * a.K;  // group g's K columns of the A rows
  const uint16_t* Bg = a.B + (int64_t)g * a.N * a.K;

  // staging: APT 16-B A pieces and BPT B pieces per thread per K step
  const int sr = tid >> 2, sk = (tid & 3) * 8;
  const uint16_t* ap[APT];
  const float* srow[APT];
#pragma unroll
  for (int q = 0; q < APT; ++q) {
    const int64_t arow = min(m0 + sr + 128 * q, (int64_t)a.M - 1);  // clamp: rows >= M are never stored
    ap[q] = Ag + arow * a.lda + sk;
    srow[q] = EPI == 1 ? a.scale + (int64_t)(arow / a.P) * a.kscale + sk : nullptr;
  }
  const uint16_t* bp = Bg + (int64_t)(n0 + sr) * a.K + sk;
  uint4 ra[APT], rb[BPT];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < APT; ++q) ra[q] = *reinterpret_cast<const uint4*>(ap[q] + k0);
#pragma unroll
    for (int q = 0; q < BPT; ++q) rb[q] = *reinterpret_cast<const uint4*>(bp + (int64_t)128 * q * a.K + k0);
  };
  auto swrite = [&](int buf, int k0) {
#pragma unroll
    for (int q = 0; q < APT; ++q) {
      if (EPI == 1 && k0 + sk < a.kscale) ra[q] = silu_scale_piece(ra[q], srow[q] + k0);
      *reinterpret_cast<uint4*>(&As[buf][(sr + 128 * q) * LDK + sk]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < BPT; ++q) *reinterpret_cast<uint4*>(&Bs[buf][(sr + 128 * q) * LDK + sk]) = rb[q];
  };

  f16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  swrite(0, 0);
  __syncthreads();
  const int nk = a.K / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int kk = ks * 16 + 8 * (lane >> 5);
      bf8_t bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf8_t*>(&Bs[buf][(wn * WN + j * 32 + (lane & 31)) * LDK + kk]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf8_t af = *reinterpret_cast<const bf8_t*>(&As[buf][(wm * WM + i * 32 + (lane & 31)) * LDK + kk]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) swrite(buf ^ 1, (kt + 1) * BK);
    __syncthreads();
  }

  // epilogue: lane = column, registers = rows (row = (r&3) + 8(r>>2) + 4(lane>>5)).
  // Per-ROI column sums: each 32-row tile splits into <= 2 ROI segments (P >= 32);
  // segments are accumulated in LDS as int64 fixed point per (ROI slot, column)
  // -- the workgroup's 128 rows touch at most kSlots ROIs -- then one 64-bit
  // global atomic per touched (ROI, column).  Integer adds: order-independent.
  constexpr int kSlots = BM / 32 + 1;
  static_assert(kSlots * BN * 8 <= 2 * BM * LDK * 2, "ROI sums must fit the A operand LDS");
  __syncthreads();  // operand LDS is reused for the sums
  unsigned long long* red = reinterpret_cast<unsigned long long*>(&As[0][0]);  // [kSlots][BN]
  for (int q = tid; q < kSlots * BN; q += 512) red[q] = 0ull;
  __syncthreads();
  const int64_t roi_base = m0 / a.P;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col_l = wn * WN + j * 32 + (lane & 31);
    const int col = n0 + col_l;
    const float bv = a.bias[g * a.N + col];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t r0 = m0 + wm * WM + i * 32;  // first row of this 32-row tile
      const int64_t roi0 = r0 / a.P;
      const int64_t split = (roi0 + 1) * a.P;    // first row of the next ROI
      float s_lo = 0.f, s_hi = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = r0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= a.M) continue;
        const float v = acc[i][j][r] + bv;
        float act;
        if (EPI == 0) {
          if (g == 0) {
            act = silu_f(v);
            a.C[row * a.ldc + col] = trk::f32_to_bf16(v);
          } else {
            act = hswish_f(v);
            a.C[row * a.ldc + (int64_t)a.N + col] = trk::f32_to_bf16(act);
          }
        } else {
          act = silu_f(v);
        }
        if (row < split) s_lo += act;
        else s_hi += act;
      }
      s_lo += __shfl_xor(s_lo, 32);
      s_hi += __shfl_xor(s_hi, 32);
      if (lane < 32 && r0 < a.M) {
        const int slot = (int)(roi0 - roi_base);
        atomicAdd(&red[slot * BN + col_l], (unsigned long long)llrintf(s_lo * kFix));
        if (split < r0 + 32 && split < a.M)
          atomicAdd(&red[(slot + 1) * BN + col_l], (unsigned long long)llrintf(s_hi * kFix));
      }
    }
  }
  __syncthreads();
  const int64_t last_row = min(m0 + BM, (int64_t)a.M) - 1;
  const int nslot = (int)(last_row / a.P - roi_base) + 1;
  for (int q = tid; q < nslot * BN; q += 512) {
    const int slot = q / BN, c = q % BN;
    atomicAdd(reinterpret_cast<unsigned long long*>(a.sums + (roi_base + slot) * a.ld_sums + g * a.N + n0 + c),
              red[q]);
  }
}

constexpr int kBM = 128, kBN = 128;

int launch(const EncGemmArgs& a, int epi, hipStream_t st) {
  const int64_t mt = ((int64_t)a.M + kBM - 1) / kBM;
  const int64_t nwg = mt * (a.N / kBN) * a.groups;
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_gemm: too many workgroups");
  if (epi == 0) hipLaunchKernelGGL((enc_gemm_kernel<0, kBM, kBN>), dim3((unsigned)nwg), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((enc_gemm_kernel<1, kBM, kBN>), dim3((unsigned)nwg), dim3(512), 0, st, a);
  return trk::check_launch("enc_gemm_kernel");
}

}  // namespace

extern "C" int trk_enc_dsc_gemm(const void* Y2, int64_t M, int64_t P, int64_t Kg, const void* W2,
                                const float* bias, int64_t Ng, void* XRN, long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 32 && Kg % BK == 0 && Kg > 0 && Ng % kBN == 0 && Ng > 0,
              "enc_dsc_gemm: need P >= 32, K %% 32 == 0, N %% 128 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(Y2 && W2 && bias && XRN && sums, "enc_dsc_gemm: null pointer");
  const int64_t nroi = (M + P - 1) / P;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(sums, 0, sizeof(long long) * nroi * 2 * Ng, st) != hipSuccess) {
    trk::set_error("enc_dsc_gemm: memset failed");
    return TRK_ELAUNCH;
  }
  EncGemmArgs a{};
  a.A = (const uint16_t*)Y2; a.lda = 2 * Kg;
  a.B = (const uint16_t*)W2; a.bias = bias;
  a.C = (uint16_t*)XRN; a.ldc = 2 * Ng;
  a.sums = sums; a.ld_sums = (int)(2 * Ng);
  a.M = (int)M; a.N = (int)Ng; a.K = (int)Kg; a.P = (int)P; a.groups = 2; a.kscale = 0;
  return launch(a, 0, st);
}

extern "C" int trk_enc_transition_gemm(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s,
                                       int64_t kscale, const void* Wt, const float* bias, int64_t N,
                                       long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 32 && K % BK == 0 && K > 0 && N % kBN == 0 && N > 0 && kscale % 8 == 0 &&
                  kscale <= K,
              "enc_transition_gemm: need P >= 32, K %% 32 == 0, N %% 128 == 0, kscale %% 8 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(XRN && s && Wt && bias && sums, "enc_transition_gemm: null pointer");
  const int64_t nroi = (M + P - 1) / P;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(sums, 0, sizeof(long long) * nroi * N, st) != hipSuccess) {
    trk::set_error("enc_transition_gemm: memset failed");
    return TRK_ELAUNCH;
  }
  EncGemmArgs a{};
  a.A = (const uint16_t*)XRN; a.lda = K;
  a.B = (const uint16_t*)Wt; a.bias = bias;
  a.C = nullptr; a.ldc = 0;
  a.sums = sums; a.ld_sums = (int)N;
  a.scale = s;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.P = (int)P; a.groups = 1; a.kscale = (int)kscale;
  return launch(a, 1, st);
}
