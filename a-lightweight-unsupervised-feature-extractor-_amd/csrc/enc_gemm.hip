// bf16 GEMMs of the encoder (reference model/utils/modules/card.py: DSC :48-57,
// SEBlock :73-78, RMB.forward :128-148) for gfx950, with the elementwise work
// of the eval graph fused into their prologues / epilogues.
//
// C = A . B^T on MFMA 32x32x16 bf16 (f32 accumulate): A = activation rows
// [M, K] (row stride lda), B = weights [N, K] (the conv weight's [out, in]
// layout, K contiguous).  Workgroup tile 256 x 256, BK = 32, 8 waves as
// 2 (M) x 4 (N), each wave 128 x 64 (4 x 2 accumulators): 0.75 KB of LDS
// fragment reads per MFMA, inside the ~1 KB / 32-cycle MFMA the CU's LDS
// delivers (64 x 32 wave tiles were LDS-bound at 1.5 KB).
//
// K loop: operands are staged with LDS-DMA (global_load_lds, 16 B per lane)
// into a three-stage LDS ring; the wave writes its 1 KB lane-linearly and the XOR
// swizzle of the image is applied to the per-lane SOURCE address (chunk c of
// row r at position r*4 + (c ^ ((r >> 2) & 3))), so the 16-B fragment reads of
// 16 consecutive rows hit 16 distinct bank groups.  Two K steps stay in flight
// (counted vmcnt + raw s_barrier); no staging registers.
//
// Epilogue:
//   * per-ROI column sums of the activation straight from the accumulators
//     (lane = column, registers = rows; a 32-row tile spans <= 2 ROIs since
//     P >= 32), as int64 fixed point (x 2^24) in LDS, then one 64-bit global
//     atomic per (ROI, column): integer adds, so the sums are identical
//     whatever order tiles finish in;
//   * stores through an f32 LDS block [64][264] (row stride chosen so the two
//     lane halves of a write hit disjoint banks) as 16-B bf16 vectors.
// Variants:
//   EPI_DSC   both DSC 1x1 GEMMs (group 0 = reinforce, 1 = normal) + BN-folded
//             bias; stores SiLU(x_r) / Hardswish(x_n) into the [x_r | x_n]
//             rows; sums SiLU(x_r) (SE squeeze) / Hardswish(x_n) (GAP).
//   EPI_TRANS transition: the SE excitation (x_r * s[roi]) is applied in LDS to
//             the staged A tiles of the first kscale columns; + bias, sums
//             SiLU(T); T is never stored.
//   EPI_PLAIN plain bf16 store (the four first 1x1 convs as one GEMM).
#include "trk_common.h"

unsigned long long* g_enc_prof = nullptr;  // trk_enc_set_prof (diagnostics: gemm8 / gemm4 phase stamps)
int g_enc_g4_narrow = 0;  // trk_set_tuning("enc_g4_narrow"): 1 = 3-slot ROI sums even for P >= 64 (A/B)
int g_enc_gemm = 1;      // trk_set_tuning("enc_gemm"): 1 = gemm4 (default), 0 = the 128 x 128 / 128 x 256 kernels
int g_enc_gemm_dbg = 0;     // trk_set_tuning("enc_gemm_dbg"): experiments (1 skip epilogue, 2 stores, 4 sums, 8 sum
                            // writes; g1dw: 16 no depthwise, 32 two K steps only)
int g_g1dw_persist = 0;     // trk_set_tuning("g1dw_persist"): 0 = one workgroup per tile; v > 0 = persistent
                            // tile queue, 2 workgroups per CU, the second started (v - 1) x 2048 cycles late
int g_g1dw_mode = 7;        // trk_set_tuning("g1dw_mode"): 7 (default) = g1dw4_kernel (4-wave workgroups, 16x16x32
                            // MFMAs; Y1 summed in another order); the 32x32x16 g1dw_kernel variants, bit-identical
                            // to each other: where the K loop issues its LDS-DMA (0 top, 1 after the MFMAs,
                            // 2 interleaved); 4 = warp-specialised DMA waves; 5 = 256-wide N tiles; 6 = role-split
int g_dsc_split = 1;        // trk_set_tuning("dsc_split"): 1 = gemm4's DSC tiles compiled per activation (SiLU /
                            // Hardswish), 0 = one tile body with a per-element select
int g_enc_gemm_offset = 0;  // trk_set_tuning("enc_gemm_offset"): > 0 runs gemm4 persistent (2 workgroups per CU)
                            // with each CU's second workgroup started that many x 2048 cycles late

namespace {

typedef __bf16 bf8_t __attribute__((ext_vector_type(8)));
typedef float f16_t __attribute__((ext_vector_type(16)));
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

enum { EPI_DSC = 0, EPI_TRANS = 1, EPI_PLAIN = 2 };

constexpr int BK = 32;
constexpr int CPR = BK / 8;                 // 16-B chunks per tile row
constexpr int NSTAGE = 3;                   // LDS-DMA ring: two K steps in flight
constexpr int EROWS = 64;                   // rows per epilogue store block

// Tile configuration: workgroup BM x BN, 8 waves as 2 (M) x 4 (N).  Measured
// per variant (M = 204800, K = 512 / 1024): 256 x 256 (wave 128 x 64, 0.75 KB of
// LDS fragment reads per MFMA) for the plain GEMM; 128 x 256 (wave 64 x 64) for
// the transition; 128 x 128 (wave 64 x 32) for the DSC pair, whose store +
// activation epilogue overlaps best with 3 workgroups per CU.
template <int BM_, int BN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_;
  static constexpr int WM = BM / 2, WN = BN / 4, TM = WM / 32, TN = WN / 32;
  static constexpr int AI = BM * CPR / 512, BI = BN * CPR / 512;  // DMA ops per thread per stage
  static constexpr int TLD = BN + 8;                               // epilogue block row stride (floats)
  static constexpr int kSlots = BM / 32 + 1;                       // ROIs a tile can touch (P >= 32)
  static constexpr size_t kStageBytes = NSTAGE * (size_t)(BM + BN) * CPR * 16;
  static constexpr size_t kEpiBytes = (size_t)EROWS * TLD * 4 + (size_t)kSlots * BN * 8;
  static constexpr size_t kLds = kStageBytes > kEpiBytes ? kStageBytes : kEpiBytes;
};
constexpr float kFix = 16777216.0f;         // 2^24
// per-ROI sums leave the GEMMs as int64 partials, one per 128-row M tile that
// covers the ROI (<= 3 for P <= 256), written with plain stores (no atomics,
// no memset); consumers add the 1..3 partials of a ROI (trk_enc_sums_reduce,
// trk_enc_se, trk_enc_head) -- integer adds, so the totals do not depend on
// tile order
constexpr int kPart = TRK_ENC_PARTS, kPartRows = 128;

struct EncGemmArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;       // [groups][N][K]
  const float* bias;       // [groups * N] or null
  uint16_t* C;             // output rows, stride ldc; group g at column g * N
  int64_t ldc;
  long long* sums;         // per-ROI partial sums [nroi][kPart][ld_sums] (one per 128-row tile
  int ld_sums;             // covering the ROI); group g at column g * N
  const float* scale;      // EPI_TRANS: s [nroi][kscale]
  int M, N, K, P, groups, kscale;
  int dbg;                 // g_enc_gemm_dbg
  int hsplit;              // g_dsc_split: gemm4 DSC tiles instantiated per activation
  unsigned long long* prof;  // trk_enc_set_prof (gemm4: per-workgroup phase stamps; diagnostics)
};

// bf16-path activations: hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32), a
// few ulp of f32 -- far below the bf16 rounding these kernels feed
__device__ __forceinline__ float silu_f(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * v));
}
__device__ __forceinline__ float hswish_f(float v) {
  return v * fminf(fmaxf(v + 3.0f, 0.0f), 6.0f) * (1.0f / 6.0f);
}
__device__ __forceinline__ unsigned long long eg_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// cross-lane exchanges without the LDS pipe (ds_bpermute): DPP quad_perm for lane ^ 1,
// gfx950's v_permlane16/32_swap for the half-row / half-wave sums; a + b in either
// order, so the sums equal x + __shfl_xor(x, 16 / 32) bit for bit
__device__ __forceinline__ float lane_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t nx = 8;
  if (nwg < nx) return bid;
  int64_t q = nwg / nx, r = nwg % nx, x = bid % nx;
  int64_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

// chunk c (of CPR = 4) of row r lives at r*4 + (c ^ ((r >> 2) & 3)): 16 consecutive
// rows of one chunk land in 16 distinct 16-B bank groups
typedef float dw_pair_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int swz(int r, int c) { return r * CPR + (c ^ ((r >> 2) & 3)); }
__device__ __forceinline__ int unswz_c(int p) { return (p % CPR) ^ (((p / CPR) >> 2) & 3); }

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return trk::pack2_bf16(a, b);
}

template <int EPI, int BM_, int BN_>
__global__ void __launch_bounds__(512) enc_gemm_kernel(EncGemmArgs a) {
  using T = Tile<BM_, BN_>;
  constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, TM = T::TM, TN = T::TN;
  constexpr int AI = T::AI, BI = T::BI, TLD = T::TLD, kSlots = T::kSlots;
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);  // [NSTAGE][BM * CPR]
  uint4* Bs = As + NSTAGE * BM * CPR;           // [NSTAGE][BN * CPR]
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

  // LDS-DMA sources: the lane writes LDS position (wave*AI + q)*64 + lane, which
  // holds (row, chunk) = inverse swizzle of that position
  const uint16_t* asrc[AI];
  const uint16_t* bsrc[BI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int p = (wave * AI + q) * 64 + lane, r = p / CPR, c = unswz_c(p);
    const int64_t row = min(m0 + r, (int64_t)a.M - 1);  // clamp: rows >= M are never stored
    asrc[q] = Ag + row * a.lda + c * 8;
  }
#pragma unroll
  for (int q = 0; q < BI; ++q) {
    const int p = (wave * BI + q) * 64 + lane, r = p / CPR, c = unswz_c(p);
    bsrc[q] = Bg + (int64_t)(n0 + r) * a.K + c * 8;
  }
  auto issue = [&](int stage, int k0) {
#pragma unroll
    for (int q = 0; q < AI; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + k0), LPTR(As + stage * BM * CPR + (wave * AI + q) * 64), 16,
                                       0, 0);
#pragma unroll
    for (int q = 0; q < BI; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + k0), LPTR(Bs + stage * BN * CPR + (wave * BI + q) * 64), 16,
                                       0, 0);
  };
  // EPI_TRANS: x_r * s[roi] on a staged A tile whose K range is < kscale.  The
  // thread's s values for step k are loaded during step k-1 (sv registers), so
  // the transform never waits on a global load.
  constexpr int TPT = BM * CPR / 512;  // A pieces per thread per step
  float4 sv[TPT][2];
  auto sload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
      const int p = tid + 512 * q, r = p / CPR, c = unswz_c(p);
      const int64_t row = min(m0 + r, (int64_t)a.M - 1);
      const float* sp = a.scale + (row / a.P) * a.kscale + k0 + c * 8;
      sv[q][0] = *reinterpret_cast<const float4*>(sp);
      sv[q][1] = *reinterpret_cast<const float4*>(sp + 4);
    }
  };
  auto transform = [&](int stage) {
    uint4* as = As + stage * BM * CPR;
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
      const int p = tid + 512 * q;
      const float s8[8] = {sv[q][0].x, sv[q][0].y, sv[q][0].z, sv[q][0].w,
                           sv[q][1].x, sv[q][1].y, sv[q][1].z, sv[q][1].w};
      uint4 v = as[p];
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x0 = __uint_as_float(w[e] << 16), x1 = __uint_as_float(w[e] & 0xffff0000u);
        w[e] = pack_bf16x2(x0 * s8[2 * e], x1 * s8[2 * e + 1]);
      }
      as[p] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  };

  f16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // K loop over an NSTAGE ring.  Each stage is 2 LDS-DMA ops per thread
  // (AI + BI); waiting for stage kt while stage kt+1 stays in flight is a
  // counted vmcnt(AI + BI), and the barrier is a raw s_barrier (__syncthreads would
  // drain every DMA in flight with vmcnt(0), MI355X guide "glds ... across a
  // barrier").  Stage (kt+2) % 3 is refilled right after the barrier of step
  // kt: every wave has finished reading it (step kt-1) by then.
  static_assert(AI + BI >= 2 && AI + BI <= 4, "vmcnt immediates below assume 2..4 DMA ops per stage");
  const int nk = a.K / BK;
  issue(0, 0);
  if (nk > 1) issue(1, BK);
  if (EPI == EPI_TRANS && a.kscale > 0) sload(0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt % NSTAGE;
    if (kt + 1 < nk) {
      if constexpr (AI + BI == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (AI + BI == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (EPI == EPI_TRANS && kt * BK < a.kscale) {
      transform(st);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (kt + 2 < nk) issue((kt + 2) % NSTAGE, (kt + 2) * BK);
    if (EPI == EPI_TRANS && (kt + 1) * BK < a.kscale) sload((kt + 1) * BK);
    const uint4* as = As + st * BM * CPR;
    const uint4* bs = Bs + st * BN * CPR;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + (lane >> 5);
      bf8_t bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * WN + j * 32 + (lane & 31), c)]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(wm * WM + i * 32 + (lane & 31), c)]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // all LDS reads of the ring done before the epilogue reuses it

  // ---- epilogue
  float* tile = reinterpret_cast<float*>(smem);                                                  // [EROWS][TLD]
  unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + (size_t)EROWS * TLD * 4);  // [kSlots][BN]
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn * WN + j * 32 + (lane & 31);
    const float bv = a.bias ? a.bias[g * a.N + n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // the activation, once: both the ROI sums and the stores use it
        const float v = acc[i][j][r] + bv;
        acc[i][j][r] = EPI == EPI_PLAIN ? v : (EPI == EPI_DSC && g == 1) ? hswish_f(v) : silu_f(v);
      }
  }

  if (EPI != EPI_PLAIN) {
    // per-ROI column sums of the activation from the registers (lane = column,
    // registers = 16 rows of a 32-row tile; <= 2 ROI segments per tile)
    for (int q = tid; q < kSlots * BN; q += 512) red[q] = 0ull;
    __syncthreads();
    const int64_t roi_base = m0 / a.P;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn * WN + j * 32 + (lane & 31);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int64_t r0 = m0 + wm * WM + i * 32;
        const int64_t roi0 = r0 / a.P;
        const int64_t split = (roi0 + 1) * a.P;
        float s_lo = 0.f, s_hi = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = r0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const float act = acc[i][j][r];
          if (row < a.M) {
            if (row < split) s_lo += act;
            else s_hi += act;
          }
        }
        s_lo = sum_xor32(s_lo);
        s_hi = sum_xor32(s_hi);
        if (lane < 32 && r0 < a.M) {
          const int slot = (int)(roi0 - roi_base);
          atomicAdd(&red[slot * BN + cl], (unsigned long long)llrintf(s_lo * kFix));
          if (split < r0 + 32 && split < a.M)
            atomicAdd(&red[(slot + 1) * BN + cl], (unsigned long long)llrintf(s_hi * kFix));
        }
      }
    }
    __syncthreads();
    const int64_t last_row = min(m0 + BM, (int64_t)a.M) - 1;
    const int nslot = (int)(last_row / a.P - roi_base) + 1;
    for (int q = tid; q < nslot * BN; q += 512) {
      const int slot = q / BN, c = q % BN;
      const int64_t roi = roi_base + slot;
      const int j = (int)(m0 / kPartRows - roi * a.P / kPartRows);  // this tile among the ROI's tiles
      a.sums[(roi * kPart + j) * a.ld_sums + g * a.N + n0 + c] = (long long)red[q];
    }
  }
  if (EPI == EPI_TRANS) return;

  // stores: 64-row blocks through the f32 LDS tile, then 16-B bf16 vectors per
  // thread (coalesced rows).  Block h holds rows [64h, 64h + 64): wave row-group
  // wm = h / (WM / 64), its accumulator tiles i = 2 (h % (WM / 64)) .. + 1.
  constexpr int HPW = WM / EROWS;  // store blocks per wave row-group
  const int64_t cbase = (int64_t)(EPI == EPI_DSC ? g * a.N : 0) + n0;
#pragma unroll
  for (int h = 0; h < BM / EROWS; ++h) {
    if (wm == h / HPW) {
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        const int i = 2 * (h % HPW) + i2;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cl = wn * WN + j * 32 + (lane & 31);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = i2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            tile[rl * TLD + cl] = acc[i][j][r];
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < EROWS * BN / 8 / 512; ++q) {
      const int p = tid + 512 * q, rl = p / (BN / 8), c8 = (p % (BN / 8)) * 8;
      const int64_t row = m0 + h * EROWS + rl;
      if (row < a.M) {
        const float4 v0 = *reinterpret_cast<const float4*>(&tile[rl * TLD + c8]);
        const float4 v1 = *reinterpret_cast<const float4*>(&tile[rl * TLD + c8 + 4]);
        *reinterpret_cast<uint4*>(a.C + row * a.ldc + cbase + c8) =
            make_uint4(pack_bf16x2(v0.x, v0.y), pack_bf16x2(v0.z, v0.w), pack_bf16x2(v1.x, v1.y),
                       pack_bf16x2(v1.z, v1.w));
      }
    }
    __syncthreads();
  }
}

template <int EPI, int BM, int BN>
int launch(const EncGemmArgs& a, hipStream_t st) {
  using T = Tile<BM, BN>;
  const int64_t mt = ((int64_t)a.M + BM - 1) / BM;
  const int64_t nwg = mt * (a.N / BN) * a.groups;
  TRK_REQUIRE(a.N % BN == 0, "enc_gemm: N must be a multiple of %d", BN);
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_gemm: too many workgroups");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(enc_gemm_kernel<EPI, BM, BN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)T::kLds);
    attr = true;
  }
  hipLaunchKernelGGL((enc_gemm_kernel<EPI, BM, BN>), dim3((unsigned)nwg), dim3(512), T::kLds, st, a);
  return trk::check_launch("enc_gemm_kernel");
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Persistent tile queue: tiles are dealt from 8 per-XCD ranges (tile order as
// xcd_remap, so one XCD's L2 sees contiguous M tiles); a workgroup takes tiles of
// its own range first (blockIdx % 8, the dispatcher's round-robin -- placement is a
// speed hint only) and then steals from the others, so workgroups that start late
// -- behind CUs another stream still holds -- just take fewer tiles.  The last
// workgroup to leave resets the counters for the next launch using this slot.
constexpr int kQueues = 64;                 // launch slots (round-robin on the host)
__device__ unsigned int g_tileq[kQueues][10];  // [0..7] next index per XCD range, [8] workgroups done

struct TileQueue {
  unsigned int* q;
  int64_t ntiles;
  __device__ int64_t range_lo(int x) const {
    const int64_t b = ntiles / 8, r = ntiles % 8;
    return x * b + (x < r ? x : r);
  }
  // next tile for this workgroup (uniform), or -1; tid 0 fetches, LDS broadcast
  __device__ int64_t next(int* slot, int& cur) const {
    if (threadIdx.x == 0) {
      int64_t t = -1;
      for (; cur < 8 && t < 0; ) {
        const int x = (int)((blockIdx.x + cur) & 7);
        const int64_t lo = range_lo(x), n = range_lo(x + 1) - lo;
        const unsigned int i = atomicAdd(&q[x], 1u);
        if ((int64_t)i < n) t = lo + i;
        else ++cur;
      }
      *slot = (int)t;
    }
    __syncthreads();
    const int t = *slot;
    __syncthreads();
    return t;
  }
  __device__ void finish() const {
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(&q[8], 1u) == gridDim.x - 1) {
        for (int x = 0; x < 9; ++x) atomicExch(&q[x], 0u);
        __threadfence();
      }
    }
  }
};

int next_queue_slot() {
  static int s = 0;
  s = (s + 1) % kQueues;
  return s;
}

// ---------------------------------------------------------------------------
// First 1x1 convs + the four depthwise 5x5 convs in one kernel (10x10 ROIs).
//
// The M tile is two whole ROIs (200 rows, computed as 7 MFMA row tiles of 32;
// rows 200..223 belong to the next tile and are discarded), so the 5x5
// neighbourhood of every output pixel is inside the tile: Y1 = X . W1^T is
// rounded to bf16 into LDS (exactly what the plain GEMM would store) and the
// depthwise conv runs from there with dwconv5_rows2_kernel's f32 FMA order (taps
// in the zero padding skipped), writing only Y2.  Y1 never reaches HBM.  N tile =
// 128 channels; 8 waves: wave w owns column tile w & 3 and row tiles (w >> 2) +
// 2t.  K loop as enc_gemm_kernel (LDS-DMA ring, NSTAGE = 3).
constexpr int G1_ROWS = 224, G1_BN = 128, G1_S = 10, G1_P = 100;
constexpr int G1_AP = G1_ROWS * CPR;               // A 16-B pieces per stage (896)
constexpr size_t G1_STAGE = (size_t)(G1_ROWS + G1_BN) * CPR * 16;
constexpr size_t G1_TILE = (size_t)2 * G1_P * (G1_BN / 2) * 4;   // bf16 pairs [200][64]
constexpr size_t G1_W = (size_t)25 * (G1_BN / 2) * 8;            // f32 pairs [25][64]
constexpr size_t G1_LDS = NSTAGE * G1_STAGE > G1_TILE + G1_W ? NSTAGE * G1_STAGE : G1_TILE + G1_W;

// Depthwise 5x5 of output rows [OY0, OY1) x columns [X0, X0 + 5) of a 10x10
// ROI for the lane's channel pair: input rows / columns clipped to the ROI (the
// zero padding's taps are skipped at compile time), weights read from LDS.  Each
// output accumulates its taps in ascending input row, then ascending kx --
// dwconv5_rows2_kernel's order, so Y2 is bit-identical.
template <int OY0, int OY1, int X0>
__device__ __forceinline__ void dw5_block(const uint32_t* __restrict__ src, const dw_pair_t* __restrict__ w,
                                          uint32_t* __restrict__ dst, int ldd) {
  constexpr int NY = OY1 - OY0;
  constexpr int IY0 = OY0 - 2 < 0 ? 0 : OY0 - 2, IY1 = OY1 + 1 > G1_S - 1 ? G1_S - 1 : OY1 + 1;
  constexpr int IX0 = X0 - 2 < 0 ? 0 : X0 - 2, IX1 = X0 + 6 > G1_S - 1 ? G1_S - 1 : X0 + 6;
  constexpr int NX = IX1 - IX0 + 1;
  dw_pair_t acc[NY][5];
#pragma unroll
  for (int oy = 0; oy < NY; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) acc[oy][ox] = dw_pair_t{0.f, 0.f};
  // input rows are software-pipelined: row iy + 1 is read from LDS while row iy is used
  uint32_t nxt[NX];
#pragma unroll
  for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[(IY0 * G1_S + IX0 + ix) * (G1_BN / 2)];
#pragma unroll 1
  for (int iy = IY0; iy <= IY1; ++iy) {  // rolled: one input row's values live at a time
    dw_pair_t in[NX];
#pragma unroll
    for (int ix = 0; ix < NX; ++ix) in[ix] = dw_pair_t{__uint_as_float(nxt[ix] << 16), __uint_as_float(nxt[ix] & 0xffff0000u)};
    const int iyn = iy < IY1 ? iy + 1 : iy;
#pragma unroll
    for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[(iyn * G1_S + IX0 + ix) * (G1_BN / 2)];
#pragma unroll
    for (int oy = 0; oy < NY; ++oy) {
      const int ky = iy - (OY0 + oy) + 2;
      if (ky < 0 || ky > 4) continue;
      dw_pair_t wr[5];  // weight row ky (LDS)
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) wr[kx] = w[(ky * 5 + kx) * (G1_BN / 2)];
#pragma unroll
      for (int ox = 0; ox < 5; ++ox)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) {
          const int ix = X0 + ox + kx - 2;
          if (ix >= IX0 && ix <= IX1)
            acc[oy][ox] = __builtin_elementwise_fma(wr[kx], in[ix - IX0], acc[oy][ox]);
        }
    }
  }
#pragma unroll
  for (int oy = 0; oy < NY; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) {
      const uint32_t v = pack_bf16x2(acc[oy][ox].x, acc[oy][ox].y);
      if (ldd > 0) dst[((OY0 + oy) * G1_S + X0 + ox) * ldd] = v;
      else asm volatile("" ::"v"(v));  // experiment (enc_gemm_dbg 256): no Y2 stores
    }
}

// one 5x5 output quadrant (QY, QX), in two row blocks (fewer live accumulators)
template <int QY, int QX>
__device__ __forceinline__ void dw5_quadrant(const uint32_t* __restrict__ src, const dw_pair_t* __restrict__ w,
                                             uint32_t* __restrict__ dst, int ldd) {
  dw5_block<5 * QY, 5 * QY + 3, 5 * QX>(src, w, dst, ldd);
  dw5_block<5 * QY + 3, 5 * QY + 5, 5 * QX>(src, w, dst, ldd);
}

template <int MODE>
__device__ __forceinline__ void g1dw_tile(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                          const float* __restrict__ wdw, uint16_t* __restrict__ Y2, int M, int N,
                                          int dbg, int64_t lb, unsigned char* smem) {
  uint4* As = reinterpret_cast<uint4*>(smem);       // [NSTAGE][224 * CPR]
  uint4* Bs = As + NSTAGE * G1_AP;                   // [NSTAGE][128 * CPR]
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));                      // per tile: keep lane addresses out of the tile loop
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3, wr = wave >> 2;
  const int ntile_n = N / G1_BN;
  const int n0 = (int)(lb % ntile_n) * G1_BN;
  const int64_t m0 = (lb / ntile_n) * (2 * G1_P);   // two ROIs per tile
  constexpr int K = 512;

  // DMA sources: A pieces p = q*512 + tid (q = 0: all waves; q = 1: waves 0..5)
  const uint16_t* asrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = min(q * 512 + tid, G1_AP - 1), r = p / CPR, c = unswz_c(p);
    const int64_t row = min(m0 + r, (int64_t)M - 1);
    asrc[q] = X + row * K + c * 8;
  }
  const uint16_t* bsrc;
  {
    const int p = tid, r = p / CPR, c = unswz_c(p);
    bsrc = W1 + (int64_t)(n0 + r) * K + c * 8;
  }
  // DMA op j (0: A rows 0..127, 1: A rows 128..223 (waves 0..5), 2: B) of a stage
  auto issue_op = [&](int j, int stage, int k0) {
    if (dbg & 128) return;  // experiment: no operand loads
    if (j == 0)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[0] + k0), LPTR(As + stage * G1_AP + wave * 64), 16, 0, 0);
    else if (j == 1) {
      if (wave < (G1_AP - 512) / 64)
        __builtin_amdgcn_global_load_lds(GPTR(asrc[1] + k0), LPTR(As + stage * G1_AP + 512 + wave * 64), 16, 0, 0);
    } else {
      __builtin_amdgcn_global_load_lds(GPTR(bsrc + k0), LPTR(Bs + stage * G1_BN * CPR + wave * 64), 16, 0, 0);
    }
  };
  auto issue = [&](int stage, int k0) {
    issue_op(0, stage, k0);
    issue_op(1, stage, k0);
    issue_op(2, stage, k0);
  };
  // row tiles of this wave: wr, wr + 2, wr + 4 (+ wr + 6 for wr == 0)
  constexpr int TMX = 4;
  const int ntm = wr == 0 ? 4 : 3;
  f16_t acc[TMX];
#pragma unroll
  for (int i = 0; i < TMX; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  // waves 0..5 issue 3 DMA ops per stage, waves 6..7 issue 2
  const int nk = (dbg & 32) ? 2 : K / BK;
  issue(0, 0);
  issue(1, BK);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt % NSTAGE;
    if (kt + 1 < nk) {
      if (wave < (G1_AP - 512) / 64) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool pf = kt + 2 < nk;
    const int pst = (kt + 2) % NSTAGE, pk = (kt + 2) * BK;
    if (MODE == 0 && pf) issue(pst, pk);
    const uint4* as = As + st * G1_AP;
    const uint4* bs = Bs + st * G1_BN * CPR;
    if (!(dbg & 64)) {  // dbg 64 (experiment): no MFMAs
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int c = ks * 2 + (lane >> 5);
        const bf8_t bfr = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * 32 + (lane & 31), c)]);
#pragma unroll
        for (int i = 0; i < TMX; ++i) {
          if (i < ntm) {
            const int rt = wr + 2 * i;
            const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(rt * 32 + (lane & 31), c)]);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[i], 0, 0, 0);
          }
          // MODE 2: the stage's three DMA ops interleaved with the MFMAs
          if (MODE == 2 && pf && ((ks == 0 && (i == 0 || i == 2)) || (ks == 1 && i == 0))) {
            __builtin_amdgcn_sched_barrier(0);
            issue_op(ks == 0 ? i / 2 : 2, pst, pk);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
    if (MODE == 1 && pf) {  // after this step's MFMAs are issued
      __builtin_amdgcn_sched_barrier(0);
      issue(pst, pk);
    }
  }
  __syncthreads();

  const int cp = lane;
  // depthwise weights [25][64 channel pairs] of the tile: global loads issued now,
  // written to LDS after Y1 (their latency hides behind the Y1 writes)
  dw_pair_t* wl = reinterpret_cast<dw_pair_t*>(smem + G1_TILE);
  constexpr int NWQ = (25 * (G1_BN / 2) + 511) / 512;
  dw_pair_t wreg[NWQ];
#pragma unroll
  for (int j = 0; j < NWQ; ++j) {
    const int q = min(j * 512 + tid, 25 * (G1_BN / 2) - 1), k = q / (G1_BN / 2), pp = q % (G1_BN / 2);
    wreg[j] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * pp);
  }
  // Y1 (bf16-rounded, rows < 200 of the tile) -> LDS [200][64 channel pairs]
  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem);
  {
    const int cl = wn * 32 + (lane & 31);  // channel within the tile
#pragma unroll
    for (int i = 0; i < TMX; ++i) {
      if (i < ntm) {
        const int rt = wr + 2 * i;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (rl < 2 * G1_P) reinterpret_cast<uint16_t*>(y1)[rl * G1_BN + cl] = trk::f32_to_bf16(acc[i][r]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NWQ; ++j)
    if (j * 512 + tid < 25 * (G1_BN / 2)) wl[j * 512 + tid] = wreg[j];
  __syncthreads();

  // depthwise 5x5: wave = (ROI, 5x5 output quadrant): 8 equal tasks, lane = channel pair
  if (dbg & 16) return;
  {
    const int roi = wave >> 2, quad = wave & 3;
    const int64_t rbase = m0 + roi * G1_P;
    if (rbase < M) {
      const uint32_t* src = y1 + roi * G1_P * (G1_BN / 2) + cp;
      const dw_pair_t* wq = wl + cp;
      uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + rbase * N + n0) + cp;
      const int ldd = (dbg & 256) ? 0 : N / 2;
      switch (quad) {
        case 0: dw5_quadrant<0, 0>(src, wq, dst, ldd); break;
        case 1: dw5_quadrant<0, 1>(src, wq, dst, ldd); break;
        case 2: dw5_quadrant<1, 0>(src, wq, dst, ldd); break;
        default: dw5_quadrant<1, 1>(src, wq, dst, ldd); break;
      }
    }
  }
}

template <int MODE>
__global__ void __launch_bounds__(512) g1dw_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                   const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                   int M, int N, int dbg) {
  extern __shared__ __align__(16) unsigned char smem[];
  g1dw_tile<MODE>(X, W1, wdw, Y2, M, N, dbg, xcd_remap(blockIdx.x, gridDim.x), smem);
}

// ---------------------------------------------------------------------------
// g1dw, warp-specialised: 10 waves = 8 MFMA waves (the tile split of g1dw_tile)
// + 2 DMA waves that issue the whole stage (22 LDS-DMA wave-instructions).  The
// K loop is L2->LDS bound (~27 TB/s chip-wide for this tile shape) and a wave
// that issues LDS-DMA stalls while the memory pipeline is full; with the issue
// on waves of their own, the MFMA waves keep the matrix pipe busy meanwhile.
// One s_barrier per K step for all 10 waves: the DMA waves wait (vmcnt) for
// stage kt, the barrier publishes it, then they issue stage kt + 2 while the
// MFMA waves consume stage kt.  The depthwise phase runs on all 10 waves, one
// (ROI, output row pair) task each.  Same arithmetic as g1dw_kernel.
__global__ void __launch_bounds__(640, 5) g1dw_ws_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                      const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                      int M, int N) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);       // [NSTAGE][224 * CPR]
  uint4* Bs = As + NSTAGE * G1_AP;                   // [NSTAGE][128 * CPR]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntile_n = N / G1_BN;
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = (int)(lb % ntile_n) * G1_BN;
  const int64_t m0 = (lb / ntile_n) * (2 * G1_P);
  constexpr int K = 512, NK = K / BK, NBLK = (G1_AP + G1_BN * CPR) / 64;  // 22 blocks of 64 pieces
  constexpr int NI = NBLK / 2;                                             // per DMA wave (11)
  static_assert(NBLK % 2 == 0 && G1_AP % 64 == 0, "DMA blocks");
  const bool dmaw = wave >= 8;

  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem);
  dw_pair_t* wl = reinterpret_cast<dw_pair_t*>(smem + G1_TILE);
  if (dmaw) {
    // ---- DMA waves: piece q = 64 b + lane of a block sits at row 16 b + lane / 4 (of A,
    // or of B past the A blocks), chunk unswz_c(lane); 32-bit element offsets from the
    // uniform operand bases (M * 512 < 2^31: checked on the host)
    const int p = wave - 8;
    const int lrow = lane >> 2, lcol = unswz_c(lane) * 8;
    auto issue = [&](int stage, int k0) {
      int lr = lrow;
      asm volatile("" : "+v"(lr));  // offsets rebuilt per stage: no hoisted per-block state
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int b = 2 * i + p;
        if (b < G1_AP / 64) {
          const int row = min((int)m0 + 16 * b + lr, M - 1);
          __builtin_amdgcn_global_load_lds(GPTR(X + (row * K + lcol + k0)), LPTR(As + stage * G1_AP + b * 64), 16,
                                           0, 0);
        } else {
          const int row = n0 + 16 * (b - G1_AP / 64) + lr;
          __builtin_amdgcn_global_load_lds(GPTR(W1 + (row * K + lcol + k0)),
                                           LPTR(Bs + stage * G1_BN * CPR + (b - G1_AP / 64) * 64), 16, 0, 0);
        }
      }
    };
    issue(0, 0);
    issue(1, BK);
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      if (kt + 1 < NK) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");   // stage kt landed, kt + 1 in flight
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 2 < NK) issue((kt + 2) % NSTAGE, (kt + 2) * BK);  // buffer last read in step kt - 1
    }
    __syncthreads();
  } else {
    // ---- MFMA waves: the g1dw_tile split (wave: column tile wave & 3, row tiles (wave >> 2) + 2t)
    constexpr int TMX = 4;
    const int wn = wave & 3, wr = wave >> 2;
    const int ntm = wr == 0 ? 4 : 3;
    f16_t acc[TMX];
#pragma unroll
    for (int i = 0; i < TMX; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const uint4* as = As + (kt % NSTAGE) * G1_AP;
      const uint4* bs = Bs + (kt % NSTAGE) * G1_BN * CPR;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int c = ks * 2 + (lane >> 5);
        const bf8_t bfr = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * 32 + (lane & 31), c)]);
#pragma unroll
        for (int i = 0; i < TMX; ++i) {
          if (i < ntm) {
            const int rt = wr + 2 * i;
            const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(rt * 32 + (lane & 31), c)]);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[i], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
    const int cl = wn * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TMX; ++i) {
      if (i < ntm) {
        const int rt = wr + 2 * i;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (rl < 2 * G1_P) reinterpret_cast<uint16_t*>(y1)[rl * G1_BN + cl] = trk::f32_to_bf16(acc[i][r]);
        }
      }
    }
  }
  for (int q = tid; q < 25 * (G1_BN / 2); q += 640) {
    const int k = q / (G1_BN / 2), pp = q % (G1_BN / 2);
    wl[q] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * pp);
  }
  __syncthreads();

  // depthwise 5x5: one (ROI, output row pair) task per wave
  {
    const int roi = wave / (G1_S / 2), y0 = 2 * (wave % (G1_S / 2));
    const int64_t rbase = m0 + roi * G1_P;
    if (rbase < M) {
      const uint32_t* src = y1 + roi * G1_P * (G1_BN / 2);
      dw_pair_t a0[G1_S], a1[G1_S];
#pragma unroll
      for (int x = 0; x < G1_S; ++x) { a0[x] = dw_pair_t{0.f, 0.f}; a1[x] = dw_pair_t{0.f, 0.f}; }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const int yy = y0 - 2 + r;
        if (yy < 0 || yy >= G1_S) continue;
        dw_pair_t rr[G1_S];
#pragma unroll
        for (int x = 0; x < G1_S; ++x) {
          const uint32_t v = src[(yy * G1_S + x) * (G1_BN / 2) + lane];
          rr[x] = dw_pair_t{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
        }
        if (r <= 4) {
          dw_pair_t wv[5];
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(r * 5 + kx) * (G1_BN / 2) + lane];
#pragma unroll
          for (int x = 0; x < G1_S; ++x)
#pragma unroll
            for (int kx = 0; kx < 5; ++kx)
              if (x + kx >= 2 && x + kx < G1_S + 2) a0[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a0[x]);
        }
        if (r >= 1) {
          dw_pair_t wv[5];
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[((r - 1) * 5 + kx) * (G1_BN / 2) + lane];
#pragma unroll
          for (int x = 0; x < G1_S; ++x)
#pragma unroll
            for (int kx = 0; kx < 5; ++kx)
              if (x + kx >= 2 && x + kx < G1_S + 2) a1[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a1[x]);
        }
      }
      uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + rbase * N + n0);
#pragma unroll
      for (int x = 0; x < G1_S; ++x) {
        dst[(y0 * G1_S + x) * (N / 2) + lane] = pack_bf16x2(a0[x].x, a0[x].y);
        dst[((y0 + 1) * G1_S + x) * (N / 2) + lane] = pack_bf16x2(a1[x].x, a1[x].y);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// g1dw with 256-channel N tiles (g1dw_mode 5): one 16-wave workgroup per CU per
// tile of 2 ROIs x 256 channels.  Against the 128-channel tile it halves the
// L2 -> LDS traffic of the A operand (each X row is staged 4 instead of 8 times:
// 1.9 instead of 2.95 GB per launch), which the K loop pays for one-to-one
// (DESIGN.md §4).  Waves: row parity wr = wave >> 3 (row tiles wr + 2t), column
// tile wave & 7 (the g1dw_tile split over 8 column tiles).  Depthwise: 20 tasks
// (ROI, output row pair, 128-channel half) over the 16 waves.  LDS: Y1 [200][128
// pairs] + weights [25][128] (128 KiB), the operand ring aliased below it.
constexpr int G2_BN = 256;
constexpr size_t G2_STAGE = (size_t)(G1_ROWS + G2_BN) * CPR * 16;      // 30 KiB
constexpr size_t G2_TILE = (size_t)2 * G1_P * (G2_BN / 2) * 4;         // 100 KiB
constexpr size_t G2_W = (size_t)25 * (G2_BN / 2) * 8;                  // 25 KiB
constexpr size_t G2_LDS = NSTAGE * G2_STAGE > G2_TILE + G2_W ? NSTAGE * G2_STAGE : G2_TILE + G2_W;
static_assert(G2_LDS <= 160 * 1024, "g1dw256 LDS");

__global__ void __launch_bounds__(1024) g1dw256_kernel(const uint16_t* __restrict__ X,
                                                       const uint16_t* __restrict__ W1,
                                                       const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                       int M, int N) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);          // [NSTAGE][224 * CPR]
  uint4* Bs = As + NSTAGE * G1_AP;                      // [NSTAGE][256 * CPR]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 7, wr = wave >> 3;
  const int ntile_n = N / G2_BN;
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = (int)(lb % ntile_n) * G2_BN;
  const int64_t m0 = (lb / ntile_n) * (2 * G1_P);
  constexpr int K = 512, NK = K / BK;
  constexpr int BP = G2_BN * CPR;                       // B pieces per stage (1024)

  // DMA: A pieces 0..895 (threads 0..895), B pieces 0..1023 (all threads)
  const uint16_t* asrc;
  {
    const int p = min(tid, G1_AP - 1), r = p / CPR, c = unswz_c(p);
    asrc = X + min(m0 + r, (int64_t)M - 1) * K + c * 8;
  }
  const uint16_t* bsrc = W1 + (int64_t)(n0 + tid / CPR) * K + unswz_c(tid) * 8;
  const bool adma = wave < G1_AP / 64;                  // waves 0..13 stage A pieces
  auto issue = [&](int stage, int k0) {
    if (adma) __builtin_amdgcn_global_load_lds(GPTR(asrc + k0), LPTR(As + stage * G1_AP + wave * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(GPTR(bsrc + k0), LPTR(Bs + stage * BP + wave * 64), 16, 0, 0);
  };
  constexpr int TMX = 4;
  const int ntm = wr == 0 ? 4 : 3;
  f16_t acc[TMX];
#pragma unroll
  for (int i = 0; i < TMX; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  issue(0, 0);
  issue(1, BK);
  for (int kt = 0; kt < NK; ++kt) {
    if (kt + 1 < NK) {
      if (adma) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const uint4* as = As + (kt % NSTAGE) * G1_AP;
    const uint4* bs = Bs + (kt % NSTAGE) * BP;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + (lane >> 5);
      const bf8_t bfr = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * 32 + (lane & 31), c)]);
#pragma unroll
      for (int i = 0; i < TMX; ++i) {
        if (i < ntm) {
          const int rt = wr + 2 * i;
          const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(rt * 32 + (lane & 31), c)]);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[i], 0, 0, 0);
        }
      }
    }
    if (kt + 2 < NK) {  // after this step's MFMAs (g1dw_mode 1); the buffer was last read in step kt - 1
      __builtin_amdgcn_sched_barrier(0);
      issue((kt + 2) % NSTAGE, (kt + 2) * BK);
    }
  }
  __syncthreads();

  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem);
  dw_pair_t* wl = reinterpret_cast<dw_pair_t*>(smem + G2_TILE);
  {
    const int cl = wn * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TMX; ++i) {
      if (i < ntm) {
        const int rt = wr + 2 * i;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (rl < 2 * G1_P) reinterpret_cast<uint16_t*>(y1)[rl * G2_BN + cl] = trk::f32_to_bf16(acc[i][r]);
        }
      }
    }
  }
  for (int q = tid; q < 25 * (G2_BN / 2); q += 1024) {
    const int k = q / (G2_BN / 2), pp = q % (G2_BN / 2);
    wl[q] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * pp);
  }
  __syncthreads();

  // depthwise 5x5: task = (ROI, output row pair, 128-channel half), lane = channel pair
  for (int task = wave; task < 20; task += 16) {
    const int roi = task / 10, rem = task % 10, y0 = 2 * (rem % 5), cp = (rem / 5) * 64 + lane;
    const int64_t rbase = m0 + roi * G1_P;
    if (rbase >= M) continue;
    const uint32_t* src = y1 + roi * G1_P * (G2_BN / 2);
    dw_pair_t a0[G1_S], a1[G1_S];
#pragma unroll
    for (int x = 0; x < G1_S; ++x) { a0[x] = dw_pair_t{0.f, 0.f}; a1[x] = dw_pair_t{0.f, 0.f}; }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int yy = y0 - 2 + r;
      if (yy < 0 || yy >= G1_S) continue;
      dw_pair_t rr[G1_S];
#pragma unroll
      for (int x = 0; x < G1_S; ++x) {
        const uint32_t v = src[(yy * G1_S + x) * (G2_BN / 2) + cp];
        rr[x] = dw_pair_t{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
      }
      if (r <= 4) {
        dw_pair_t wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(r * 5 + kx) * (G2_BN / 2) + cp];
#pragma unroll
        for (int x = 0; x < G1_S; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx)
            if (x + kx >= 2 && x + kx < G1_S + 2) a0[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a0[x]);
      }
      if (r >= 1) {
        dw_pair_t wv[5];
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[((r - 1) * 5 + kx) * (G2_BN / 2) + cp];
#pragma unroll
        for (int x = 0; x < G1_S; ++x)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx)
            if (x + kx >= 2 && x + kx < G1_S + 2) a1[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a1[x]);
      }
    }
    uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + rbase * N + n0);
#pragma unroll
    for (int x = 0; x < G1_S; ++x) {
      dst[(y0 * G1_S + x) * (N / 2) + cp] = pack_bf16x2(a0[x].x, a0[x].y);
      dst[((y0 + 1) * G1_S + x) * (N / 2) + cp] = pack_bf16x2(a1[x].x, a1[x].y);
    }
  }
}

// persistent: two workgroups per CU take tiles from the queue; each CU's second
// workgroup starts offset x 2048 cycles late so its K loop runs beside the first
// one's depthwise phase
__global__ void __launch_bounds__(512) g1dw_persist_kernel(const uint16_t* __restrict__ X,
                                                           const uint16_t* __restrict__ W1,
                                                           const float* __restrict__ wdw,
                                                           uint16_t* __restrict__ Y2, int M, int N, int dbg,
                                                           int64_t ntiles, int qslot, int offset) {
  extern __shared__ __align__(16) unsigned char smem[];
  const TileQueue tq{g_tileq[qslot], ntiles};
  if (offset > 0 && blockIdx.x >= gridDim.x / 2)
    for (int i = 0; i < offset; ++i) __builtin_amdgcn_s_sleep(32);
  int cur = 0;
  for (;;) {
    const int64_t t = tq.next(reinterpret_cast<int*>(smem), cur);  // LDS is free between tiles
    if (t < 0) break;
    g1dw_tile<0>(X, W1, wdw, Y2, M, N, dbg, t, smem);
    __syncthreads();  // the next tile's DMA reuses the LDS the depthwise phase read
  }
  tq.finish();
}


// ---------------------------------------------------------------------------
// g1dw, interleaved (persistent, one workgroup per CU): the depthwise 5x5 of
// the previous tile runs INSIDE the K loop of the current tile's GEMM, so its
// VALU work fills the MFMA / LDS-DMA latency of the K loop instead of running
// as a separate phase.  LDS: a 4-stage operand ring (three K steps in flight),
// the previous tile's Y1 [200][64 pairs] and its depthwise weights.
//   per tile t:  K step kt: barrier, DMA of step kt + 3, MFMAs of tile t, and on
//                even kt one depthwise input-row step of tile t - 1;
//                barrier; Y1(t) and weights(t) -> LDS; next tile.
// Depthwise work per tile = 10 (ROI, output row pair) tasks = 52 valid input-row
// steps: waves 0..5 own one interior task each (6 steps), waves 6..7 own the
// two border tasks of one ROI (4 + 4 steps); every wave is done by K step 14.
// Same arithmetic as g1dw_kernel (bit-identical).
constexpr int IL_NST = 4;
constexpr size_t IL_RING = (size_t)IL_NST * G1_STAGE;                 // 90112
constexpr size_t IL_LDS = IL_RING + G1_TILE + G1_W + 16;               // 154128
static_assert(IL_LDS <= 160 * 1024, "g1dw_il: one workgroup per CU");

// one input row yy (kernel rows r / r - 1 for output rows y0 / y0 + 1)
__device__ __forceinline__ void il_dw_row(const uint32_t* __restrict__ src, const dw_pair_t* __restrict__ wl, int yy,
                                          int r, dw_pair_t (&a0)[G1_S], dw_pair_t (&a1)[G1_S], int cp) {
  dw_pair_t rr[G1_S];
#pragma unroll
  for (int x = 0; x < G1_S; ++x) {
    const uint32_t v = src[(yy * G1_S + x) * (G1_BN / 2) + cp];
    rr[x] = dw_pair_t{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
  }
  if (r <= 4) {
    dw_pair_t wv[5];
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[(r * 5 + kx) * (G1_BN / 2) + cp];
#pragma unroll
    for (int x = 0; x < G1_S; ++x)
#pragma unroll
      for (int kx = 0; kx < 5; ++kx)
        if (x + kx >= 2 && x + kx < G1_S + 2) a0[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a0[x]);
  }
  if (r >= 1) {
    dw_pair_t wv[5];
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) wv[kx] = wl[((r - 1) * 5 + kx) * (G1_BN / 2) + cp];
#pragma unroll
    for (int x = 0; x < G1_S; ++x)
#pragma unroll
      for (int kx = 0; kx < 5; ++kx)
        if (x + kx >= 2 && x + kx < G1_S + 2) a1[x] = __builtin_elementwise_fma(wv[kx], rr[x + kx - 2], a1[x]);
  }
}

__global__ void __launch_bounds__(512) g1dw_il_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                      const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                      int M, int N, int64_t ntiles, int qslot) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);                     // [IL_NST][224 * CPR]
  uint4* Bs = As + IL_NST * G1_AP;                                 // [IL_NST][128 * CPR]
  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem + IL_RING);      // previous tile's Y1
  dw_pair_t* wl = reinterpret_cast<dw_pair_t*>(smem + IL_RING + G1_TILE);
  int* slot = reinterpret_cast<int*>(smem + IL_RING + G1_TILE + G1_W);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3, wr = wave >> 2;
  const int ntile_n = N / G1_BN;
  constexpr int K = 512, NK = K / BK;
  const TileQueue tq{g_tileq[qslot], ntiles};
  int cur = 0;
  // depthwise plan of this wave: (roi, y0, first / last input-row step r)
  const int d_roi = wave < 6 ? wave / 3 : wave - 6;
  const int d_y0a = wave < 6 ? 2 * (1 + wave % 3) : 0;    // interior pair, or border pair 0
  const int ops = wave < (G1_AP - 512) / 64 ? 3 : 2;      // DMA ops per stage of this wave

  int64_t t = tq.next(slot, cur), tp = -1;
  while (t >= 0 || tp >= 0) {
    const bool gemm = t >= 0;
    const int n0 = gemm ? (int)(t % ntile_n) * G1_BN : 0;
    const int64_t m0 = gemm ? (t / ntile_n) * (2 * G1_P) : 0;
    const uint16_t* asrc[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = min(q * 512 + tid, G1_AP - 1), r = p / CPR, c = unswz_c(p);
      asrc[q] = X + min(m0 + r, (int64_t)M - 1) * K + c * 8;
    }
    const uint16_t* bsrc = W1 + (int64_t)(n0 + tid / CPR) * K + unswz_c(tid) * 8;
    auto issue = [&](int stage, int k0) {
      __builtin_amdgcn_global_load_lds(GPTR(asrc[0] + k0), LPTR(As + stage * G1_AP + wave * 64), 16, 0, 0);
      if (ops == 3)
        __builtin_amdgcn_global_load_lds(GPTR(asrc[1] + k0), LPTR(As + stage * G1_AP + 512 + wave * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(GPTR(bsrc + k0), LPTR(Bs + stage * G1_BN * CPR + wave * 64), 16, 0, 0);
    };
    // previous tile's depthwise target
    const int pn0 = tp >= 0 ? (int)(tp % ntile_n) * G1_BN : 0;
    const int64_t prbase = tp >= 0 ? (tp / ntile_n) * (2 * G1_P) + d_roi * G1_P : M;
    const bool dw = tp >= 0 && prbase < M;
    const uint32_t* dsrc = y1 + d_roi * G1_P * (G1_BN / 2);
    uint32_t* ddst = reinterpret_cast<uint32_t*>(Y2 + (dw ? prbase : 0) * N + pn0);
    dw_pair_t a0[G1_S], a1[G1_S];

    constexpr int TMX = 4;
    const int ntm = wr == 0 ? 4 : 3;
    f16_t acc[TMX];
#pragma unroll
    for (int i = 0; i < TMX; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    if (gemm) {
      issue(0, 0);
      issue(1, BK);
      issue(2, 2 * BK);
    }
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      if (gemm) {
        // stage kt landed; kt + 1, kt + 2 (and at most one step's Y2 stores) may stay in flight
        if (kt + 2 < NK) {
          if (ops == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else if (kt + 1 < NK) {
          if (ops == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (gemm) {
        if (kt + 3 < NK) issue((kt + 3) % IL_NST, (kt + 3) * BK);
        const uint4* as = As + (kt % IL_NST) * G1_AP;
        const uint4* bs = Bs + (kt % IL_NST) * G1_BN * CPR;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
          const int c = ks * 2 + (lane >> 5);
          const bf8_t bfr = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * 32 + (lane & 31), c)]);
#pragma unroll
          for (int i = 0; i < TMX; ++i) {
            if (i < ntm) {
              const int rt = wr + 2 * i;
              const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(rt * 32 + (lane & 31), c)]);
              acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[i], 0, 0, 0);
            }
          }
        }
      }
      // one depthwise input-row step of the previous tile on even K steps
      if (dw && !(kt & 1)) {
        const int s = kt >> 1;
        int y0, r;
        if (wave < 6) { y0 = d_y0a; r = s; }
        else if (s < 4) { y0 = 0; r = s + 2; }          // border pair 0: input rows 0..3
        else { y0 = 8; r = s - 4; }                      // border pair 4: input rows 6..9
        const bool active = wave < 6 ? s < 6 : true;
        if (active) {
          const bool first = wave < 6 ? s == 0 : (s == 0 || s == 4);
          const bool last = wave < 6 ? s == 5 : (s == 3 || s == 7);
          if (first) {
#pragma unroll
            for (int x = 0; x < G1_S; ++x) { a0[x] = dw_pair_t{0.f, 0.f}; a1[x] = dw_pair_t{0.f, 0.f}; }
          }
          il_dw_row(dsrc, wl, y0 - 2 + r, r, a0, a1, lane);
          if (last) {
#pragma unroll
            for (int x = 0; x < G1_S; ++x) {
              ddst[(y0 * G1_S + x) * (N / 2) + lane] = pack_bf16x2(a0[x].x, a0[x].y);
              ddst[((y0 + 1) * G1_S + x) * (N / 2) + lane] = pack_bf16x2(a1[x].x, a1[x].y);
            }
          }
        }
      }
    }
    __syncthreads();  // every read of Y1(tp) / weights(tp) and of the ring is done
    if (gemm) {
      const int cl = wn * 32 + (lane & 31);
#pragma unroll
      for (int i = 0; i < TMX; ++i) {
        if (i < ntm) {
          const int rt = wr + 2 * i;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (rl < 2 * G1_P) reinterpret_cast<uint16_t*>(y1)[rl * G1_BN + cl] = trk::f32_to_bf16(acc[i][r]);
          }
        }
      }
      for (int q = tid; q < 25 * (G1_BN / 2); q += 512) {
        const int k = q / (G1_BN / 2), pp = q % (G1_BN / 2);
        wl[q] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * pp);
      }
    }
    tp = t;
    t = gemm ? tq.next(slot, cur) : -1;  // next() ends with a barrier: Y1 / weights visible
    if (!gemm) break;                     // the drain pass ran the last tile's depthwise
  }
  tq.finish();
}

// ---------------------------------------------------------------------------
// g1dw, role-split (g1dw_mode 6; persistent, one 16-wave workgroup per CU):
// waves 0..7 run the GEMM of tile t (the g1dw_il_kernel K loop, 4-stage ring),
// waves 8..15 run the depthwise 5x5 of tile t - 1 from LDS at the same time,
// as g1dw_kernel's straight-line (ROI, quadrant) tasks.  An MFMA holds its
// SIMD's vector issue for 8 of its 32 cycles, so the depthwise VALU of the
// partner waves can fill the other 24 (MI355X_MICROARCH.md, vector-instruction
// issue cost).  The GEMM waves do not use s_barrier inside the K loop (the
// depthwise waves would have to take part): each arrives on an LDS counter
// once its DMA pieces of the step have landed and waits until all 8 have
// (also the ring's write-after-read guard: a wave arrives after its reads of
// the previous step).  Tile boundaries use s_barrier for all 16 waves.
// Bit-identical to g1dw_kernel.  Measured (tools/exp/enc_breakdown.py, 2048 ROIs):
// 646-721 us against g1dw_kernel<1>'s 486-492.  The depthwise does overlap (it adds
// 70-120 us here, 180 there), but the counter handshake costs ~900 cycles per K
// step (406 us with neither MFMAs nor depthwise); an earlier form that kept the K
// loop's s_barrier for all 16 waves (one depthwise input row per two K steps)
// measured 711 us: the coupled row steps were latency-bound.  Kept as a knob.
__device__ __forceinline__ void sp_arrive_wait(uint32_t addr, uint32_t target) {
  asm volatile("s_waitcnt lgkmcnt(0)\n\tds_add_u32 %0, %1" ::"v"(addr), "v"(1u) : "memory");
  uint32_t v;
  for (;;) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    if (__builtin_amdgcn_readfirstlane(v) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ void __launch_bounds__(1024) g1dw_sp_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                       const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                       int M, int N, int64_t ntiles, int qslot, int dbg) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);                     // [IL_NST][224 * CPR]
  uint4* Bs = As + IL_NST * G1_AP;                                 // [IL_NST][128 * CPR]
  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem + IL_RING);      // previous tile's Y1
  dw_pair_t* wl = reinterpret_cast<dw_pair_t*>(smem + IL_RING + G1_TILE);
  int* slot = reinterpret_cast<int*>(smem + IL_RING + G1_TILE + G1_W);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(slot + 1);           // K-step arrivals (64 per wave)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool mma = wave < 8;
  const int wn = wave & 3, wr = (wave >> 2) & 1;
  const int ntile_n = N / G1_BN;
  constexpr int K = 512, NK = K / BK;
  const TileQueue tq{g_tileq[qslot], ntiles};
  int cur = 0;
  const int ops = wave < (G1_AP - 512) / 64 ? 3 : 2;
  if (threadIdx.x == 0) *cnt = 0;
  uint32_t arrivals = 0;                                           // steps this wave has completed

  int64_t t = tq.next(slot, cur), tp = -1;                         // next() ends with a barrier
  while (t >= 0 || tp >= 0) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // per tile: keep lane addresses out of the tile loop (no spills)
    const int lane = tid & 63;
    const bool gemm = t >= 0;
    const int n0 = gemm ? (int)(t % ntile_n) * G1_BN : 0;
    const int64_t m0 = gemm ? (t / ntile_n) * (2 * G1_P) : 0;
    if (mma) {
      constexpr int TMX = 4;
      const int ntm = wr == 0 ? 4 : 3;
      f16_t acc[TMX];
      const uint16_t* asrc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int p = min(q * 512 + tid, G1_AP - 1), r = p / CPR, c = unswz_c(p);
        asrc[q] = X + min(m0 + r, (int64_t)M - 1) * K + c * 8;
      }
      const uint16_t* bsrc = W1 + (int64_t)(n0 + tid / CPR) * K + unswz_c(tid) * 8;
      auto issue = [&](int stage, int k0) {
        __builtin_amdgcn_global_load_lds(GPTR(asrc[0] + k0), LPTR(As + stage * G1_AP + wave * 64), 16, 0, 0);
        if (ops == 3)
          __builtin_amdgcn_global_load_lds(GPTR(asrc[1] + k0), LPTR(As + stage * G1_AP + 512 + wave * 64), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(GPTR(bsrc + k0), LPTR(Bs + stage * G1_BN * CPR + wave * 64), 16, 0, 0);
      };
#pragma unroll
      for (int i = 0; i < TMX; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      if (gemm) {
        issue(0, 0);
        issue(1, BK);
        issue(2, 2 * BK);
#pragma unroll 1
        for (int kt = 0; kt < NK; ++kt) {
          if (kt + 2 < NK) {
            if (ops == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          } else if (kt + 1 < NK) {
            if (ops == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          ++arrivals;
          sp_arrive_wait((uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)cnt), arrivals * 8 * 64);
          if (dbg & 64) continue;  // experiment: no MFMAs / further loads
          if (kt + 3 < NK) issue((kt + 3) % IL_NST, (kt + 3) * BK);
          const uint4* as = As + (kt % IL_NST) * G1_AP;
          const uint4* bs = Bs + (kt % IL_NST) * G1_BN * CPR;
#pragma unroll
          for (int ks = 0; ks < BK / 16; ++ks) {
            const int c = ks * 2 + (lane >> 5);
            const bf8_t bfr = *reinterpret_cast<const bf8_t*>(&bs[swz(wn * 32 + (lane & 31), c)]);
#pragma unroll
            for (int i = 0; i < TMX; ++i) {
              if (i < ntm) {
                const int rt = wr + 2 * i;
                const bf8_t af = *reinterpret_cast<const bf8_t*>(&as[swz(rt * 32 + (lane & 31), c)]);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[i], 0, 0, 0);
              }
            }
          }
        }
      }
      __syncthreads();  // (with the depthwise waves') every read of Y1(tp) and of the ring is done
      if (gemm) {
        const int cl = wn * 32 + (lane & 31);
#pragma unroll
        for (int i = 0; i < TMX; ++i) {
          if (i < ntm) {
            const int rt = wr + 2 * i;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
              if (rl < 2 * G1_P) reinterpret_cast<uint16_t*>(y1)[rl * G1_BN + cl] = trk::f32_to_bf16(acc[i][r]);
            }
          }
        }
      }
    } else {
      // depthwise 5x5 of the previous tile: wave = (ROI, 5x5 output quadrant), lane = channel pair
      const int dwv = wave - 8, roi = dwv >> 2, quad = dwv & 3;
      const int64_t rbase = tp >= 0 ? (tp / ntile_n) * (2 * G1_P) + roi * G1_P : M;
      if (rbase < M && !(dbg & 16)) {   // dbg 16 (experiment): no depthwise
        const int pn0 = (int)(tp % ntile_n) * G1_BN;
        const uint32_t* src = y1 + roi * G1_P * (G1_BN / 2) + lane;
        const dw_pair_t* wq = wl + lane;
        uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + rbase * N + pn0) + lane;
        switch (quad) {
          case 0: dw5_quadrant<0, 0>(src, wq, dst, N / 2); break;
          case 1: dw5_quadrant<0, 1>(src, wq, dst, N / 2); break;
          case 2: dw5_quadrant<1, 0>(src, wq, dst, N / 2); break;
          default: dw5_quadrant<1, 1>(src, wq, dst, N / 2); break;
        }
      }
      __syncthreads();  // (with the GEMM waves') every read of weights(tp) is done
      if (gemm) {
        for (int q = tid - 512; q < 25 * (G1_BN / 2); q += 512) {
          const int kk = q / (G1_BN / 2), pp = q % (G1_BN / 2);
          wl[q] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)kk * N + n0 + 2 * pp);
        }
      }
    }
    tp = t;
    t = gemm ? tq.next(slot, cur) : -1;  // next() ends with a barrier: Y1 / weights visible
    if (!gemm) break;                     // the drain pass ran the last tile's depthwise
  }
  tq.finish();
}

typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

// LDS image of a 64-B-row operand tile read as mfma_f32_16x16x32 fragments
// (lane l: row l & 15, chunk l >> 4; ds_read_b128 serves lanes in the groups
// {0-3,12-15,20-27} {4-11,16-19,28-31} {32-35,44-47,52-59} {36-43,48-51,60-63},
// MI355X_MICROARCH.md §LDS): chunk c of row r sits at 16-B slot c ^ x16(r), which
// gives each group 16 distinct slots of the 256-B bank row
__device__ __forceinline__ int x16(int r) { return ((r >> 3) & 1) << 1; }

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(const T* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)p);
}
__device__ __forceinline__ u32x4 lds_read128(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ void lds_write128(uint32_t addr, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v silu2(f2v v) {
  const f2v e = v * f2v{-1.44269504088896341f, -1.44269504088896341f};
  const f2v d = f2v{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)} + f2v{1.0f, 1.0f};
  return v * f2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ f2v hswish2(f2v v) {
  const f2v c = v + f2v{3.0f, 3.0f};
  const f2v r = f2v{fminf(fmaxf(c.x, 0.0f), 6.0f), fminf(fmaxf(c.y, 0.0f), 6.0f)};
  return (v * r) * f2v{1.0f / 6.0f, 1.0f / 6.0f};
}

__device__ __forceinline__ void g4_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// gemm4: 128 x 256 tiles on 4-wave workgroups, two workgroups per CU, so one
// workgroup's epilogue (activation, ROI sums, the bf16 stores) runs under the
// other's MFMA loop.  Waves 2 (M) x 2 (N), wave tile 64 x 128 = 4 x 8 MFMA
// 16x16x32 tiles (0.375 KB of fragment reads per MFMA).  BK = 32 in a
// 3-buffer LDS-DMA ring, tile kt + 2 issued at the top of step kt (its buffer
// was last read in step kt - 1, before the barrier that ends it); the counted
// vmcnt(6) at the end of step kt retires tile kt + 1 and leaves kt + 2 in
// flight; one raw s_barrier per K step.  LDS 80 KiB per workgroup.
constexpr int G4_SLD = 132;                 // stage row stride (u32): conflict-free pair writes
constexpr int G4_BUF = 1536;                // uint4 per buffer: A 512 (128 rows) | B 1024 (256 rows)
constexpr size_t G4_RING = (size_t)3 * G4_BUF * 16;     // 72 KiB
constexpr int G4_SLOTS = 4;                 // ROIs a 128-row tile spans (P >= 43)
constexpr int G4_WSLOTS = 3;                // ROIs a wave's 64 rows span (P >= 43)
constexpr int G4_SQ = 2;                    // s-tile DMA per thread (8 KiB)
constexpr size_t G4_STILE = (size_t)G4_SQ * 256 * 16;
constexpr size_t G4_STAGE = (size_t)128 * G4_SLD * 4;   // 66 KiB
constexpr size_t G4_RED = (size_t)G4_SLOTS * 256 * 8;   // 8 KiB
constexpr size_t G4_LDS = (G4_RING + G4_STILE) > (G4_STAGE + G4_RED) ? (G4_RING + G4_STILE) : (G4_STAGE + G4_RED);
static_assert(G4_LDS <= 80 * 1024, "two gemm4 workgroups per CU");

// WIDE (P >= 64): a wave's 64 rows span at most 2 ROIs and a tile's 128 at most 3, so
// the ROI-sum epilogue keeps 2 slots per wave instead of 3 (a third fewer reductions)
template <int EPI, bool WIDE = false, int HSWM = -1>
__device__ __forceinline__ void gemm4_tile(const EncGemmArgs& a, int64_t lb, unsigned char* smem) {
  uint4* ring = reinterpret_cast<uint4*>(smem);
  // opaque per tile: keeps the compiler from hoisting lane-dependent addresses
  // out of the persistent tile loop (they would stay live across the MFMA loop)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntile_n = a.N / 256;
  const int ntl = (int)(lb % (ntile_n * a.groups));
  const int64_t mt = lb / (ntile_n * a.groups);
  const int g = ntl / ntile_n, n0 = (ntl % ntile_n) * 256;
  const int64_t m0 = mt * 128;
  const uint16_t* Ag = a.A + (int64_t)g * a.K;
  const uint16_t* Bg = a.B + (int64_t)g * a.N * a.K;
  const int nk = a.K / BK;
  const int64_t roi_base = m0 / a.P;

  const uint16_t* asrc[2];
  const uint16_t* bsrc[4];
  int arow[2], achk[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    arow[q] = r;
    achk[q] = c;
    asrc[q] = Ag + min(m0 + r, (int64_t)a.M - 1) * a.lda + c * 8;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    bsrc[q] = Bg + (int64_t)(n0 + r) * a.K + c * 8;
  }
  auto issue = [&](int kt) {
    uint4* d = ring + (kt % 3) * G4_BUF + wave * 64;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * 256), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * BK), LPTR(d + 512 + q * 256), 16, 0, 0);
  };

  const float* stile = reinterpret_cast<const float*>(smem + G4_RING);
  const float* srow[2] = {stile, stile};
  if constexpr (EPI == EPI_TRANS) {
    const int per = a.kscale / 4;
    const int64_t nroi = ((int64_t)a.M + a.P - 1) / a.P;
#pragma unroll
    for (int q = 0; q < G4_SQ; ++q) {
      const int p = q * 256 + tid;
      const int slot = min(p / per, G4_SLOTS - 1);
      const int64_t roi = min(roi_base + slot, nroi - 1);
      const float* src = a.scale + roi * a.kscale + (p % per) * 4;
      __builtin_amdgcn_global_load_lds(GPTR(src), LPTR(reinterpret_cast<uint4*>(smem + G4_RING) + q * 256 + wave * 64),
                                       16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t row = min(m0 + arow[q], (int64_t)a.M - 1);
      srow[q] = stile + (int)(row / a.P - roi_base) * a.kscale + achk[q] * 8;
    }
  }
  auto transform = [&](int kt) {
    if constexpr (EPI == EPI_TRANS) {
      if (kt * BK < a.kscale) {
        const uint32_t d = lds_addr(ring + (kt % 3) * G4_BUF + tid);
        u32x4 v[2], s4[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          v[q] = lds_read128(d + q * 256 * 16);
          const uint32_t sa = lds_addr(srow[q] + kt * BK);
          s4[q][0] = lds_read128(sa);
          s4[q][1] = lds_read128(sa + 16);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(s4[0][0]), "+v"(s4[0][1]),
                     "+v"(s4[1][0]), "+v"(s4[1][1])::"memory");
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float s_lo = __uint_as_float(s4[q][e >> 1][(2 * e) & 3]);
            const float s_hi = __uint_as_float(s4[q][e >> 1][(2 * e + 1) & 3]);
            o[e] = pack_bf16x2(__uint_as_float(v[q][e] << 16) * s_lo, __uint_as_float(v[q][e] & 0xffff0000u) * s_hi);
          }
          lds_write128(d + q * 256 * 16, o);
        }
      }
    }
  };

  const int fr = lane & 15, fc = lane >> 4;
  const int lterm = fr * 4 + (fc ^ x16(fr));
  const int aoff = (wr * 64) * 4 + lterm;            // + mt * 64
  const int boff = 512 + (wc * 128) * 4 + lterm;     // + nt * 64

  f4v acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};

  // diagnostics (trk_enc_set_prof): wave 0's [start, K loop, activation, ROI sums,
  // staging + barrier, sums stores, output stores drained] per workgroup
  unsigned long long pst[8];
  const bool prof = a.prof != nullptr;
  if (prof) pst[0] = eg_stamp();
  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  transform(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g4_barrier();

  // tile kt + 2's DMA is issued after step kt's MFMAs (its buffer was last read in
  // step kt - 1): the MFMAs start as soon as the fragments are read, and the DMA
  // issue -- which stalls while the memory pipeline is full -- runs beside them
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * G4_BUF;
    bf8v bfr[8], afr[4];
#pragma unroll
    for (int t = 0; t < 8; ++t) bfr[t] = *reinterpret_cast<const bf8v*>(buf + boff + t * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) afr[i] = *reinterpret_cast<const bf8v*>(buf + aoff + i * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[t], acc[i][t], 0, 0, 0);
    if (kt + 2 < nk) {
      __builtin_amdgcn_sched_barrier(0);
      issue(kt + 2);
    }
    if (kt + 1 < nk) {
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      transform(kt + 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_barrier();
  }

  if (prof) pst[1] = eg_stamp();
  if (a.dbg & 1) {
    if (tid == 0 && acc[0][0][0] == 12345.f) a.sums[0] = 1;
    return;
  }
  // ---- epilogue (the ring is free: every DMA retired, all reads done at the last barrier)
  const int colq = wc * 128 + fr;  // + t * 16
  // HSWM: -1 = the DSC group decides per tile (a select per element pair, which the compiler
  // turns into 64 branches, each a dependent exp / rcp chain padded with s_nops); 0 / 1 = the
  // tile's activation is known at compile time (straight-line SiLU or Hardswish)
  const bool hsw = HSWM < 0 ? (EPI == EPI_DSC && g == 1) : HSWM == 1;
  float bias8[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) bias8[t] = a.bias[g * a.N + n0 + colq + t * 16];  // one batch of loads
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f2v b2 = {bias8[t], bias8[t]};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2v v = f2v{acc[i][t][2 * h], acc[i][t][2 * h + 1]} + b2;
        v = hsw ? hswish2(v) : silu2(v);
        acc[i][t][2 * h] = v.x;
        acc[i][t][2 * h + 1] = v.y;
      }
  }
  if (prof) {
    asm volatile("" ::"v"(acc[3][7][3]));
    pst[2] = eg_stamp();
  }
  // per-ROI column sums: each row-half wave (wr) writes its f32 partials for every tile
  // slot (0 where it has no rows) with plain stores -- no zeroing pass, no atomics; the
  // consumer adds llrintf(p0 * 2^24) + llrintf(p1 * 2^24) (the former int64 atomics' sum)
  float* part = reinterpret_cast<float*>(smem + (EPI == EPI_DSC ? G4_STAGE : (size_t)0));  // [2][SLOTS][256]
  if (!(a.dbg & 4)) {
    const int64_t r0w = m0 + wr * 64;
    const int64_t roiw = r0w / a.P;
    const int wslot0 = (int)(roiw - roi_base);
    const int P = a.P;
    const int nxt0 = P - (int)(r0w - roiw * P);
    const bool full = r0w + 64 <= (int64_t)a.M;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      constexpr int WS = WIDE ? 2 : G4_WSLOTS, TS = WIDE ? 3 : G4_SLOTS;
      float ssum[WS];
#pragma unroll
      for (int q = 0; q < WS; ++q) ssum[q] = 0.f;
      int slot = 0, nxt = nxt0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f4v v = acc[k][t];
        if (full && nxt >= 16 * k + 16) {
          const float x = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
          for (int q = 0; q < WS; ++q)
            if (q == slot) ssum[q] += x;
        } else {
          float lo = 0.f, hi = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * k + fc * 4 + e;
            const float x = (r0w + row < a.M) ? v[e] : 0.f;
            if (row < nxt) lo += x;
            else hi += x;
          }
#pragma unroll
          for (int q = 0; q < WS; ++q) {
            if (q == slot) ssum[q] += lo;
            if (q == slot + 1) ssum[q] += hi;
          }
        }
        if (nxt <= 16 * k + 16) {
          ++slot;
          nxt += P;
        }
      }
#pragma unroll
      for (int q = 0; q < WS; ++q) {
        ssum[q] = sum_xor16(ssum[q]);
        ssum[q] = sum_xor32(ssum[q]);
      }
      if (lane < 16) {
#pragma unroll
        for (int ts = 0; ts < TS; ++ts) {
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < WS; ++q)
            if (q <= slot && wslot0 + q == ts) v = ssum[q];
          part[(wr * G4_SLOTS + ts) * 256 + colq + t * 16] = v;
        }
      }
    }
  }
  if (prof) pst[3] = eg_stamp();
  if (EPI == EPI_DSC && !(a.dbg & 2)) {
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem);
    const bool odd = fr & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const f4v v = acc[i][t];
        const float x0 = lane_xor1(odd ? v[0] : v[2]);
        const float x1 = lane_xor1(odd ? v[1] : v[3]);
        const int rb = wr * 64 + i * 16 + fc * 4 + (odd ? 2 : 0);
        const int cp = (wc * 128 + t * 16 + fr) >> 1;
        stage[rb * G4_SLD + cp] = odd ? pack_bf16x2(x0, v[2]) : pack_bf16x2(v[0], x0);
        stage[(rb + 1) * G4_SLD + cp] = odd ? pack_bf16x2(x1, v[3]) : pack_bf16x2(v[1], x1);
      }
  }
  __syncthreads();
  if (prof) pst[4] = eg_stamp();
  {
    const int64_t last_row = min(m0 + 128, (int64_t)a.M) - 1;
    const int nslot = (int)(last_row / a.P - roi_base) + 1;
    if (!(a.dbg & 8))
      for (int q = tid; q < nslot * 256; q += 256) {
        const int slot = q >> 8, c = q & 255;
        const int64_t roi = roi_base + slot;
        const int j = (int)(m0 / kPartRows - roi * a.P / kPartRows);
        a.sums[(roi * kPart + j) * a.ld_sums + g * a.N + n0 + c] =
            llrintf(part[slot * 256 + c] * kFix) + llrintf(part[(G4_SLOTS + slot) * 256 + c] * kFix);
      }
  }
  if (prof) pst[5] = eg_stamp();
  if (EPI == EPI_DSC && !(a.dbg & 2)) {
    const uint32_t* stage = reinterpret_cast<const uint32_t*>(smem);
    const int64_t cbase = (int64_t)g * a.N + n0;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int p = q * 256 + tid, rl = p >> 5, c8 = (p & 31) * 8;
      const int64_t row = m0 + rl;
      if (row < a.M)
        *reinterpret_cast<uint4*>(a.C + row * a.ldc + cbase + c8) =
            *reinterpret_cast<const uint4*>(stage + rl * G4_SLD + c8 / 2);
    }
  }
  if (prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pst[6] = eg_stamp();
    if (tid == 0) {
      unsigned long long* o = a.prof + lb * 8;
      for (int q = 0; q < 6; ++q) o[q] = pst[q + 1] - pst[q];
      o[6] = pst[6] - pst[0];
      o[7] = 0;
    }
  }
}

// Persistent: 2 workgroups per CU walk the tiles (XCD-remapped).  The second
// resident of each CU starts a fraction of a tile late (enc_gemm_offset x
// 2048-cycle sleeps), so the two workgroups sharing a CU stay out of phase:
// one's MFMA loop runs under the other's VALU / store epilogue instead of both
// alternating between them in lockstep.
template <int EPI, bool WIDE>
__global__ void __launch_bounds__(256, 2) gemm4_kernel(EncGemmArgs a, int64_t ntiles, int offset, int qslot) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (qslot < 0) {  // one workgroup per tile
    const int64_t lb = xcd_remap(blockIdx.x, ntiles);
    if (EPI == EPI_DSC && a.hsplit) {  // the tile's group (SiLU / Hardswish) as a template argument
      if ((lb % (a.N / 256 * a.groups)) / (a.N / 256) == 1) gemm4_tile<EPI, WIDE, 1>(a, lb, smem);
      else gemm4_tile<EPI, WIDE, 0>(a, lb, smem);
    } else {
      gemm4_tile<EPI, WIDE>(a, lb, smem);
    }
    return;
  }
  const TileQueue tq{g_tileq[qslot], ntiles};
  if (offset > 0 && blockIdx.x >= gridDim.x / 2)
    for (int i = 0; i < offset; ++i) __builtin_amdgcn_s_sleep(32);
  int cur = 0;
  for (;;) {
    const int64_t t = tq.next(reinterpret_cast<int*>(smem), cur);  // LDS is free between tiles
    if (t < 0) break;
    gemm4_tile<EPI, WIDE>(a, t, smem);
    __syncthreads();  // the next tile's DMA reuses the LDS the epilogue read
  }
  tq.finish();
}

// ---------------------------------------------------------------------------
// g1dw4 (g1dw_mode 7): g1dw_kernel's first 1x1 convs + depthwise 5x5 on 4-wave
// workgroups with gemm4's operand image and 16x16x32 MFMAs.  The M tile is two
// ROIs (200 rows) computed as 13 row tiles of 16 (208 rows; 200..207 belong to
// the next tile and are discarded -- 4 % padding against g1dw_kernel's 12 %), the
// N tile 128 channels.  Waves 2 (M) x 2 (N): wave (wr, wc) owns row tiles
// 7 wr .. 7 wr + 6 (six for wr = 1) x 64 columns, a 112 x 64 wave tile with
// 11 fragment reads per 28 MFMAs (24 B of LDS reads per kflop; g1dw_kernel's
// 112 x 32 wave tiles of 32x32x16 read 39).  The K loop is L2->LDS + LDS bound,
// so bytes per flop is what this variant cuts.  DMA ring as gemm4 (BK 32, three
// buffers, tile kt + 2 issued after step kt's MFMAs); two workgroups per CU so
// one's depthwise (VALU) runs under the other's K loop.  Epilogue: Y1 rounded
// to bf16 pairs into LDS [200][64 pairs] (lane_xor1 pairing as gemm4's staging),
// depthwise weights behind it, then the 8 (ROI, quadrant) depthwise tasks of
// g1dw_kernel, two per wave (same FMA order).  Y1 sums its 512 products in
// another order than the 32x32x16 path, so Y1 (and Y2) may differ from
// g1dw_kernel's by bf16 rounding of f32 ties; tested against the fp32 GEMM.
constexpr int G1Q_ROWS = 208;                                   // 13 row tiles of 16
constexpr int G1Q_AP = G1Q_ROWS * 4;                            // A 16-B slots per buffer (832)
constexpr int G1Q_BUF = G1Q_AP + G1_BN * 4;                     // + B (512) = 1344 slots
constexpr size_t G1Q_RING = (size_t)3 * G1Q_BUF * 16;           // 63 KiB
// Y1 rows of 64 bf16 pairs at a 68-dword stride: a Y1 store's 32-lane group writes rows
// {0, 2, 4, 6} + base x 8 consecutive pairs, which the 4-dword row shift spreads over all 32
// banks (a 64-dword stride put the four rows on the same 8 banks: 4-way conflicts); the
// depthwise reads 64 consecutive dwords of one row either way
constexpr int G1Q_YS = 68;
constexpr size_t G1Q_Y1 = (size_t)2 * G1_P * G1Q_YS * 4;
constexpr size_t G1Q_LDS = G1Q_RING > G1Q_Y1 ? G1Q_RING : G1Q_Y1;   // Y1 reuses the ring
static_assert(2 * G1Q_LDS <= 160 * 1024, "two g1dw4 workgroups per CU");

// Depthwise 5x5 of one 5x5 output quadrant (QY, QX) of a 10x10 ROI for the lane's
// channel pair, weights in registers, all 25 accumulators live: each input row of the
// quadrant's (clipped) 7 x 7 window is read from LDS and unpacked once (dw5_block reads
// the window's rows in two overlapping blocks).  Same per-output order as dw5_block
// (ascending input row, then ascending kx), so equal Y1 gives equal Y2.
template <int QY, int QX, int YS>
__device__ __forceinline__ void dw5q_regs(const uint32_t* __restrict__ src, const dw_pair_t (&w)[25],
                                          uint32_t* __restrict__ dst, int ldd) {
  constexpr int OY0 = 5 * QY, X0 = 5 * QX;
  constexpr int IY0 = OY0 - 2 < 0 ? 0 : OY0 - 2, IY1 = OY0 + 6 > G1_S - 1 ? G1_S - 1 : OY0 + 6;
  constexpr int IX0 = X0 - 2 < 0 ? 0 : X0 - 2, IX1 = X0 + 6 > G1_S - 1 ? G1_S - 1 : X0 + 6;
  constexpr int NX = IX1 - IX0 + 1;
  dw_pair_t acc[5][5];
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) acc[oy][ox] = dw_pair_t{0.f, 0.f};
  uint32_t nxt[NX];
#pragma unroll
  for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[(IY0 * G1_S + IX0 + ix) * YS];
#pragma unroll
  for (int iy = IY0; iy <= IY1; ++iy) {
    dw_pair_t in[NX];
#pragma unroll
    for (int ix = 0; ix < NX; ++ix) in[ix] = dw_pair_t{__uint_as_float(nxt[ix] << 16), __uint_as_float(nxt[ix] & 0xffff0000u)};
    if (iy < IY1) {
#pragma unroll
      for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[((iy + 1) * G1_S + IX0 + ix) * YS];
    }
    // groups of up to 5 independent FMAs (the 5 outputs of a row for one tap), each group
    // closed by an empty asm on its accumulators: left to itself the compiler ran every
    // output's taps as one dependent chain (an s_nop between dependent v_pk_fma_f32) at 2
    // waves per SIMD (a sched_barrier alone does not hold: the FMAs have no chain edge)
#pragma unroll
    for (int oy = 0; oy < 5; ++oy) {
      const int ky = iy - (OY0 + oy) + 2;
      if (ky < 0 || ky > 4) continue;
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
#pragma unroll
        for (int ox = 0; ox < 5; ++ox) {
          const int ix = X0 + ox + kx - 2;
          if (ix >= IX0 && ix <= IX1)
            acc[oy][ox] = __builtin_elementwise_fma(w[ky * 5 + kx], in[ix - IX0], acc[oy][ox]);
        }
        asm volatile("" : "+v"(acc[oy][0]), "+v"(acc[oy][1]), "+v"(acc[oy][2]), "+v"(acc[oy][3]), "+v"(acc[oy][4]));
      }
    }
  }
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) {
      const uint32_t v = pack_bf16x2(acc[oy][ox].x, acc[oy][ox].y);
      if (ldd > 0) dst[((OY0 + oy) * G1_S + X0 + ox) * ldd] = v;
      else asm volatile("" ::"v"(v));  // experiment (enc_gemm_dbg 256): no Y2 stores
    }
}

__global__ void __launch_bounds__(256, 2) g1dw4_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                        const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                        int M, int N, int dbg) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntile_n = N / G1_BN;
  const int n0 = (int)(lb % ntile_n) * G1_BN;
  const int64_t m0 = (lb / ntile_n) * (2 * G1_P);
  constexpr int K = 512, NK = K / BK;

  // DMA: A slots p = q * 256 + tid (q = 0..2 every wave, q = 3 wave 0 only: 832 slots),
  // B slots 832 + q * 256 + tid (q = 0, 1); slot p holds row p >> 2, chunk (p & 3) ^ x16(row)
  const uint16_t* asrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = min(q * 256 + tid, G1Q_AP - 1), r = p >> 2, c = (p & 3) ^ x16(r);
    asrc[q] = X + min(m0 + r, (int64_t)M - 1) * K + c * 8;
  }
  const uint16_t* bsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    bsrc[q] = W1 + (int64_t)(n0 + r) * K + c * 8;
  }
  auto issue = [&](int kt) {
    if (dbg & 128) return;  // experiment: no operand loads
    uint4* d = ring + (kt % 3) * G1Q_BUF + wave * 64;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * 256), 16, 0, 0);
    if (wave == 0) __builtin_amdgcn_global_load_lds(GPTR(asrc[3] + kt * BK), LPTR(d + 3 * 256), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * BK), LPTR(d + G1Q_AP + q * 256), 16, 0, 0);
  };
  // retire all but the newest stage's DMA ops (wave 0 issues 6 per stage, the others 5)
  auto wait_prev = [&]() {
    if (dbg & 128) return;
    if (wave == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  };

  const int fr = lane & 15, fc = lane >> 4;
  const int lterm = fr * 4 + (fc ^ x16(fr));
  const int aoff = (wr * 112) * 4 + lterm;           // + i * 64
  const int boff = G1Q_AP + (wc * 64) * 4 + lterm;   // + t * 64
  const int ntm = wr == 0 ? 7 : 6;

  f4v acc[7][4];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};

  const int nk = (dbg & 32) ? 2 : NK;
  issue(0);
  issue(1);
  wait_prev();
  g4_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * G1Q_BUF;
    if (!(dbg & 64)) {  // dbg 64 (experiment): no MFMAs
      // 11 fragment reads up front (wr = 1's seventh reads B slots, unused), then counted
      // lgkmcnt waits: row tile i's MFMAs start once its A fragment has landed
      const uint32_t bb = lds_addr(buf + boff), ab = lds_addr(buf + aoff);
      u32x4 bq[4], aq[7];
#pragma unroll
      for (int t = 0; t < 4; ++t) bq[t] = lds_read128(bb + t * 1024);
#pragma unroll
      for (int i = 0; i < 7; ++i) aq[i] = lds_read128(ab + i * 1024);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        __builtin_amdgcn_sched_barrier(0);  // keep each wait in front of its own row tile's MFMAs
        if (i == 0) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(aq[0]));
        else if (i == 1) asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(aq[1]));
        else if (i == 2) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(aq[2]));
        else if (i == 3) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(aq[3]));
        else if (i == 4) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(aq[4]));
        else if (i == 5) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(aq[5]));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aq[6]));
        if (i < ntm) {
          const bf8v a = __builtin_bit_cast(bf8v, aq[i]);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8v, bq[t]), acc[i][t], 0, 0, 0);
        }
      }
    }
    if (kt + 2 < nk) {
      __builtin_amdgcn_sched_barrier(0);
      issue(kt + 2);
    }
    if (kt + 1 < nk) {
      if (kt + 2 < nk) wait_prev();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_barrier();
  }

  // depthwise weights: every wave needs the same 25 taps of its lane's channel pair, so
  // each lane loads them straight into registers (issued now, used after the Y1 writes)
  dw_pair_t wreg[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) wreg[k] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * lane);
  // Y1 (bf16 pairs, rows < 200) -> LDS [200][64]: lane pairs (fr, fr ^ 1) trade values so each
  // lane writes two column pairs: even fr rows +0, +1, odd fr rows +2, +3 (as gemm4's staging)
  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem);
  {
    const bool odd = fr & 1;
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if (i < ntm)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f4v v = acc[i][t];
          const float x0 = lane_xor1(odd ? v[0] : v[2]);
          const float x1 = lane_xor1(odd ? v[1] : v[3]);
          const int rb = wr * 112 + i * 16 + fc * 4 + (odd ? 2 : 0);
          const int cp = (wc * 64 + t * 16 + fr) >> 1;
          if (rb < 2 * G1_P) y1[rb * G1Q_YS + cp] = odd ? pack_bf16x2(x0, v[2]) : pack_bf16x2(v[0], x0);
          if (rb + 1 < 2 * G1_P) y1[(rb + 1) * G1Q_YS + cp] = odd ? pack_bf16x2(x1, v[3]) : pack_bf16x2(v[1], x1);
        }
  }
  __syncthreads();

  if (dbg & 16) return;
  // depthwise 5x5: wave = output quadrant, for each of the two ROIs; lane = channel pair
  const int ldd = (dbg & 256) ? 0 : N / 2;
#pragma unroll 1
  for (int roi = 0; roi < 2; ++roi) {
    const int64_t rbase = m0 + roi * G1_P;
    if (rbase >= M) break;
    int l = ldd;
    asm volatile("" : "+s"(l));  // per ROI: keeps the 25 store offsets out of the loop (SGPR spills)
    const uint32_t* src = y1 + roi * G1_P * G1Q_YS + lane;
    uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + rbase * N + n0) + lane;
    switch (wave) {
      case 0: dw5q_regs<0, 0, G1Q_YS>(src, wreg, dst, l); break;
      case 1: dw5q_regs<0, 1, G1Q_YS>(src, wreg, dst, l); break;
      case 2: dw5q_regs<1, 0, G1Q_YS>(src, wreg, dst, l); break;
      default: dw5q_regs<1, 1, G1Q_YS>(src, wreg, dst, l); break;
    }
  }
}

// ---------------------------------------------------------------------------
// gemm8: 256 x 256 tiles, BK = 64, one 8-wave workgroup per CU (waves 2 (M) x 4
// (N), wave tile 128 x 64 = 8 x 4 MFMA 16x16x32 tiles: 0.375 KB of fragment
// reads per MFMA).  Both operands are staged by LDS-DMA into two 64 KiB K-tile
// buffers: tile kt + 1's 8 loads per thread are issued at the top of step kt
// and have the whole step's MFMAs to land; one vmcnt(0) + barrier per step.
// The LDS image of a 256 x 64 operand is 16-B chunk c of row r at r * 8 + (c ^
// ((r >> 1) & 7)) -- the 16-lane groups of every ds_read_b128 hit 16 distinct
// bank groups -- laid down lane-linearly by the DMA (the XOR is applied to the
// per-lane source address).  The SE scale of the transition is applied in LDS by
// the thread that staged each chunk (its own vmcnt(0) orders it), before the
// step's barrier.  Epilogue (transition): bias + SiLU + per-ROI column sums; a
// wave's 128 rows are exactly one 128-row partial tile of the ROI sums.
constexpr int G8_BM = 256, G8_BN = 256, G8_BK = 64, G8_CH = G8_BK / 8;
constexpr int G8_POS = G8_BM * G8_CH;                          // 16-B slots of one operand image (2048)
constexpr size_t G8_BUF = (size_t)2 * G8_POS * 16;             // A + B images of one K tile: 64 KiB
constexpr int G8_SROI = 4;                                      // ROIs a 256-row tile spans (P >= 86)
constexpr size_t G8_STILE = (size_t)G8_SROI * 512 * 4;          // s rows of those ROIs (kscale <= 512)
constexpr size_t G8_LDS = 2 * G8_BUF + G8_STILE;               // 136 KiB

__device__ __forceinline__ int g8_swz(int r, int c) { return r * G8_CH + (c ^ ((r >> 1) & 7)); }

__device__ __forceinline__ unsigned long long g8_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// PROF (trk_enc_set_prof, diagnostics only): waves 0 and 4 of each workgroup record
// [start, prologue done, K loop done, end, sum of the per-step vmcnt waits, sum of
// the per-step barrier waits, hw id, 0] at prof[(wg * 2 + wave / 4) * 8]
// MF = 0: v_mfma_f32_16x16x32_bf16, wave tile 8 x 4 MFMA tiles; MF = 1:
// v_mfma_f32_32x32x16_bf16, 4 x 2 tiles (half the MFMA instructions; at two waves
// per SIMD a 32x32x16 retires 33 % more flops per cycle than two 16x16x32 --
// tools/exp/clock_probe.hip).  Same LDS images and fragment bytes.
template <int EPI, bool PROF, int MF>
__global__ void __launch_bounds__(512) gemm8_kernel(EncGemmArgs a, int64_t ntiles, unsigned long long* prof) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* bufs = reinterpret_cast<uint4*>(smem);                // [2][A 2048 | B 2048] uint4
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t lb = xcd_remap(blockIdx.x, ntiles);
  const int ntile_n = a.N / G8_BN;
  const int ntl = (int)(lb % (ntile_n * a.groups));
  const int64_t mt = lb / (ntile_n * a.groups);
  const int g = ntl / ntile_n, n0 = (ntl % ntile_n) * G8_BN;
  const int64_t m0 = mt * G8_BM;
  const uint16_t* Ag = a.A + (int64_t)g * a.K;
  const uint16_t* Bg = a.B + (int64_t)g * a.N * a.K;
  const int nk = a.K / G8_BK;
  const int64_t roi_base = m0 / a.P;

  // DMA sources: slot p = q * 512 + tid of each image (row p >> 3, data chunk by the swizzle)
  const uint16_t* asrc[4];
  const uint16_t* bsrc[4];
  int achunk[4], arow[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = q * 512 + tid, r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
    arow[q] = r;
    achunk[q] = c;
    asrc[q] = Ag + min(m0 + r, (int64_t)a.M - 1) * a.lda + c * 8;
    bsrc[q] = Bg + (int64_t)(n0 + r) * a.K + c * 8;
  }
  auto issue = [&](int kt) {
    uint4* d = bufs + (kt & 1) * (2 * G8_POS) + wave * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * G8_BK), LPTR(d + q * 512), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * G8_BK), LPTR(d + G8_POS + q * 512), 16, 0, 0);
  };

  // transition: the SE scales of the tile's ROIs (LDS, [G8_SROI][kscale] f32) and, per staged
  // chunk, the s row it is scaled with
  const float* stile = reinterpret_cast<const float*>(smem + 2 * G8_BUF);
  int srow[4];
  if constexpr (EPI == EPI_TRANS) {
    const int per = a.kscale / 4;                       // 16-B pieces per s row
    const int64_t nroi = ((int64_t)a.M + a.P - 1) / a.P;
    for (int p = tid; p < G8_SROI * per; p += 512) {
      const int slot = p / per;
      const int64_t roi = min(roi_base + slot, nroi - 1);
      reinterpret_cast<float4*>(smem + 2 * G8_BUF)[p] =
          *reinterpret_cast<const float4*>(a.scale + roi * a.kscale + (p % per) * 4);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = min(m0 + arow[q], (int64_t)a.M - 1);
      srow[q] = (int)(row / a.P - roi_base) * a.kscale + achunk[q] * 8;
    }
  }
  auto transform = [&](int kt) {  // x_f columns of K tile kt: bf16(x * s[roi][k])
    if constexpr (EPI == EPI_TRANS) {
      if (kt * G8_BK < a.kscale) {
        uint4* d = bufs + (kt & 1) * (2 * G8_POS);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint4 v = d[q * 512 + tid];
          const float4 s0 = *reinterpret_cast<const float4*>(stile + srow[q] + kt * G8_BK);
          const float4 s1 = *reinterpret_cast<const float4*>(stile + srow[q] + kt * G8_BK + 4);
          const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            w[e] = pack_bf16x2(__uint_as_float(w[e] << 16) * sv[2 * e], __uint_as_float(w[e] & 0xffff0000u) * sv[2 * e + 1]);
          d[q * 512 + tid] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    }
  };

  typename std::conditional<MF == 0, f4v[8][4], f16_t[4][2]>::type acc;
  if constexpr (MF == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][t][e] = 0.f;
  }

  const int fr = lane & 15, fc = lane >> 4;
  const int f32r = lane & 31, f32h = lane >> 5;
  unsigned long long p_t0 = 0, p_t1 = 0, p_t2 = 0, p_w = 0, p_b = 0;
  if constexpr (PROF) p_t0 = g8_stamp();
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // s tile (plain stores) visible before the first transform
  transform(0);
  __syncthreads();
  if constexpr (PROF) p_t1 = g8_stamp();
  // K step: 16 MFMA groups s = (k half h, row tile i), 4 MFMAs each; the A fragment of
  // group s + 1 (and the next half's B fragments) are read while group s runs, and the
  // next K tile's 8 LDS-DMA pieces are issued one per odd group, between MFMAs
  for (int kt = 0; kt < nk; ++kt) {
    const bool pf = kt + 1 < nk;
    const uint4* ab = bufs + (kt & 1) * (2 * G8_POS);
    const uint4* bb = ab + G8_POS;
    uint4* dn = bufs + ((kt + 1) & 1) * (2 * G8_POS) + wave * 64;
    auto issue_piece = [&](int q) {  // piece q: A slots q*512.. (q < 4), B slots (q - 4)*512..
      if (q < 4)
        __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + (kt + 1) * G8_BK), LPTR(dn + q * 512), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(GPTR(bsrc[q - 4] + (kt + 1) * G8_BK), LPTR(dn + G8_POS + (q - 4) * 512), 16, 0, 0);
    };
    if constexpr (MF == 0) {
      auto rd_a = [&](int s) { return *reinterpret_cast<const bf8v*>(ab + g8_swz(wr * 128 + (s & 7) * 16 + fr, (s >> 3) * 4 + fc)); };
      bf8v bfr[2][4];
  #pragma unroll
      for (int t = 0; t < 4; ++t) bfr[0][t] = *reinterpret_cast<const bf8v*>(bb + g8_swz(wc * 64 + t * 16 + fr, fc));
      bf8v afr = rd_a(0);
  #pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int h = s >> 3, i = s & 7;
        bf8v anext = afr;
        if (s < 15) anext = rd_a(s + 1);
        if (s == 4) {
  #pragma unroll
          for (int t = 0; t < 4; ++t) bfr[1][t] = *reinterpret_cast<const bf8v*>(bb + g8_swz(wc * 64 + t * 16 + fr, 4 + fc));
        }
  #pragma unroll
        for (int t = 0; t < 4; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[h][t], acc[i][t], 0, 0, 0);
        if (pf && (s & 1)) issue_piece(s >> 1);
        afr = anext;
      }
    } else {
      // 16 groups s = (k step ks = s >> 2, row tile i = s & 3), 2 MFMAs each; lane (r, h)
      // reads 16 B of row r at chunk 2 ks + h
      auto rd_a = [&](int s) { return *reinterpret_cast<const bf8v*>(ab + g8_swz(wr * 128 + (s & 3) * 32 + f32r, (s >> 2) * 2 + f32h)); };
      auto rd_b = [&](int ks, int t) { return *reinterpret_cast<const bf8v*>(bb + g8_swz(wc * 64 + t * 32 + f32r, ks * 2 + f32h)); };
      const bool top = a.dbg & 512;  // experiment: the next K tile's 8 DMA pieces all before the MFMAs
      if (pf && top) {
#pragma unroll
        for (int q = 0; q < 8; ++q) issue_piece(q);
      }
      bf8v bfr[2][2];
      bfr[0][0] = rd_b(0, 0);
      bfr[0][1] = rd_b(0, 1);
      bf8v afr = rd_a(0);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int ks = s >> 2, i = s & 3;
        bf8v anext = afr;
        if (s < 15) anext = rd_a(s + 1);
        if (i == 1 && ks < 3) {
          bfr[(ks + 1) & 1][0] = rd_b(ks + 1, 0);
          bfr[(ks + 1) & 1][1] = rd_b(ks + 1, 1);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr, bfr[ks & 1][t], acc[i][t], 0, 0, 0);
        if (pf && !top && (s & 1)) issue_piece(s >> 1);
        afr = anext;
      }
    }
    unsigned long long pa = 0, pb = 0;
    if constexpr (PROF) pa = g8_stamp();
    if (kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PROF) pb = g8_stamp();
      transform(kt + 1);
    } else if constexpr (PROF) {
      pb = pa;
    }
    __syncthreads();
    if constexpr (PROF) {
      const unsigned long long pc = g8_stamp();
      p_w += pb - pa;
      p_b += pc - pb;
    }
  }
  if constexpr (PROF) p_t2 = g8_stamp();

  if constexpr (EPI == EPI_TRANS) {
    // bias + SiLU + per-ROI column sums over this wave's 128 rows (one partial tile)
    const int64_t r0 = m0 + wr * 128;
    const int P = a.P;
    const int64_t roi0 = r0 / P;
    const int nxt = P - (int)(r0 - roi0 * P);   // first row (within the 128) of ROI roi0 + 1
    const bool full = r0 + 128 <= (int64_t)a.M;
    const int64_t last = min(r0 + 128, (int64_t)a.M) - 1;
    const int nslot = (int)(last / P - roi0) + 1;
    const int64_t th = r0 / kPartRows;
    if constexpr (MF == 0) {
      float bias4[4];
  #pragma unroll
      for (int t = 0; t < 4; ++t) bias4[t] = a.bias[n0 + wc * 64 + t * 16 + fr];
  #pragma unroll
      for (int t = 0; t < 4; ++t) {
        float sm[3] = {0.f, 0.f, 0.f};
  #pragma unroll
        for (int i = 0; i < 8; ++i) {
          f4v v = acc[i][t];
  #pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = silu_f(v[e] + bias4[t]);
          const int lo = i * 16;
          if (full && lo + 16 <= nxt) {
            sm[0] += (v[0] + v[1]) + (v[2] + v[3]);
          } else if (full && lo >= nxt && lo + 16 <= nxt + P) {
            sm[1] += (v[0] + v[1]) + (v[2] + v[3]);
          } else if (full && lo >= nxt + P) {
            sm[2] += (v[0] + v[1]) + (v[2] + v[3]);
          } else {
  #pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int ro = lo + fc * 4 + e;
              const float x = (r0 + ro < a.M) ? v[e] : 0.f;
              sm[0] += ro < nxt ? x : 0.f;
              sm[1] += (ro >= nxt && ro < nxt + P) ? x : 0.f;
              sm[2] += ro >= nxt + P ? x : 0.f;
            }
          }
        }
  #pragma unroll
        for (int q = 0; q < 3; ++q) sm[q] = sum_xor32(sum_xor16(sm[q]));
        if (fc == 0) {
  #pragma unroll
          for (int q = 0; q < 3; ++q) {
            if (q < nslot) {
              const int64_t roi = roi0 + q;
              const int j = (int)(th - roi * P / kPartRows);
              a.sums[(roi * kPart + j) * a.ld_sums + (int64_t)g * a.N + n0 + wc * 64 + t * 16 + fr] =
                  llrintf(sm[q] * kFix);
            }
          }
        }
      }
    } else {
      // 32x32 tiles: lane (c = lane & 31, h) holds rows (r & 3) + 8 (r >> 2) + 4 h of
      // column c in register r
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int col = n0 + wc * 64 + t * 32 + f32r;
        const float bias = a.bias[col];
        float sm[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f16_t v = acc[i][t];
#pragma unroll
          for (int e = 0; e < 16; ++e) v[e] = silu_f(v[e] + bias);
          const int lo = i * 32;
          if (full && (lo + 32 <= nxt || (lo >= nxt && lo + 32 <= nxt + P) || lo >= nxt + P)) {
            float x = 0.f;
#pragma unroll
            for (int e = 0; e < 16; e += 4) x += (v[e] + v[e + 1]) + (v[e + 2] + v[e + 3]);
            const int q = lo + 32 <= nxt ? 0 : lo + 32 <= nxt + P ? 1 : 2;
            sm[0] += q == 0 ? x : 0.f;
            sm[1] += q == 1 ? x : 0.f;
            sm[2] += q == 2 ? x : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int ro = lo + (e & 3) + 8 * (e >> 2) + 4 * f32h;
              const float x = (r0 + ro < a.M) ? v[e] : 0.f;
              sm[0] += ro < nxt ? x : 0.f;
              sm[1] += (ro >= nxt && ro < nxt + P) ? x : 0.f;
              sm[2] += ro >= nxt + P ? x : 0.f;
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) sm[q] = sum_xor32(sm[q]);
        if (f32h == 0) {
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            if (q < nslot) {
              const int64_t roi = roi0 + q;
              const int j = (int)(th - roi * P / kPartRows);
              a.sums[(roi * kPart + j) * a.ld_sums + (int64_t)g * a.N + col] = llrintf(sm[q] * kFix);
            }
          }
        }
      }
    }
  }
  if constexpr (PROF) {
    const unsigned long long p_t3 = g8_stamp();
    if ((wave & 3) == 0 && lane == 0) {
      unsigned long long* o = prof + ((int64_t)blockIdx.x * 2 + (wave >> 2)) * 8;
      unsigned hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      o[0] = p_t0; o[1] = p_t1; o[2] = p_t2; o[3] = p_t3; o[4] = p_w; o[5] = p_b; o[6] = hw; o[7] = 0;
    }
  }
}


template <int EPI, int MF>
int launch8(const EncGemmArgs& a, hipStream_t st) {
  const int64_t nwg = ((int64_t)a.M + G8_BM - 1) / G8_BM * (a.N / G8_BN) * a.groups;
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_gemm8: too many workgroups");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<EPI, false, MF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G8_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<EPI, true, MF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G8_LDS);
    attr = true;
  }
  if (g_enc_prof)
    hipLaunchKernelGGL((gemm8_kernel<EPI, true, MF>), dim3((unsigned)nwg), dim3(512), G8_LDS, st, a, nwg, g_enc_prof);
  else
    hipLaunchKernelGGL((gemm8_kernel<EPI, false, MF>), dim3((unsigned)nwg), dim3(512), G8_LDS, st, a, nwg, nullptr);
  return trk::check_launch("gemm8_kernel");
}

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int EPI>
int launch4(const EncGemmArgs& a, hipStream_t st) {
  const int64_t nwg = ((int64_t)a.M + 127) / 128 * (a.N / 256) * a.groups;
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_gemm4: too many workgroups");
  // persistent grid (enc_gemm_offset > 0) or one workgroup per tile (0, the default: in the
  // pipeline the GEMMs share the GPU with the tracker's kernels, and a persistent grid then
  // waits for CUs the tracker still holds)
  const int64_t grid = g_enc_gemm_offset > 0 ? std::min<int64_t>(nwg, 2 * (int64_t)cu_count()) : nwg;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm4_kernel<EPI, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G4_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm4_kernel<EPI, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G4_LDS);
    attr = true;
  }
  EncGemmArgs b = a;
  b.dbg = g_enc_gemm_dbg;
  b.hsplit = g_dsc_split;
  b.prof = g_enc_prof;
  const int qs = g_enc_gemm_offset > 0 ? next_queue_slot() : -1;
  if (a.P >= 64 && !g_enc_g4_narrow)
    hipLaunchKernelGGL((gemm4_kernel<EPI, true>), dim3((unsigned)grid), dim3(256), G4_LDS, st, b, nwg,
                       g_enc_gemm_offset, qs);
  else
    hipLaunchKernelGGL((gemm4_kernel<EPI, false>), dim3((unsigned)grid), dim3(256), G4_LDS, st, b, nwg,
                       g_enc_gemm_offset, qs);
  return trk::check_launch("gemm4_kernel");
}


// out[roi][c] = (float)(sum_j part[roi][j][c] * 2^-24) over the 1..3 partials
__global__ void __launch_bounds__(256) sums_reduce_kernel(const long long* __restrict__ part, int64_t R, int P,
                                                          int ld, float* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= R * ld) return;
  const int64_t roi = q / ld;
  const int c = (int)(q % ld);
  const int cnt = (int)((roi * P + P - 1) / kPartRows - roi * P / kPartRows) + 1;
  long long v = 0;
  for (int j = 0; j < cnt; ++j) v += part[(roi * kPart + j) * ld + c];
  out[q] = (float)((double)v * (1.0 / 16777216.0));
}

}  // namespace

extern "C" int trk_enc_sums_reduce(const long long* part, int64_t R, int64_t P, int64_t ld, float* out,
                                   void* stream) {
  TRK_REQUIRE(R >= 0 && P >= 1 && P <= 256 && ld > 0, "enc_sums_reduce: need R >= 0, 1 <= P <= 256, ld > 0");
  if (R == 0) return TRK_OK;
  TRK_REQUIRE(part && out, "enc_sums_reduce: null pointer");
  hipLaunchKernelGGL(sums_reduce_kernel, dim3((unsigned)((R * ld + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), part, R, (int)P, (int)ld, out);
  return trk::check_launch("sums_reduce_kernel");
}

extern "C" int trk_enc_gemm(const void* A, int64_t M, int64_t K, int64_t lda, const void* B, int64_t N, void* C,
                            int64_t ldc, void* stream) {
  TRK_REQUIRE(M >= 0 && K % BK == 0 && K > 0 && N % 256 == 0 && N > 0 && lda >= K && ldc >= N && lda % 8 == 0 &&
                  ldc % 8 == 0,
              "enc_gemm: need K %% 32 == 0, N %% 256 == 0, lda/ldc multiples of 8");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(A && B && C && aligned16(A) && aligned16(B) && aligned16(C), "enc_gemm: null or unaligned pointer");
  EncGemmArgs a{};
  a.A = (const uint16_t*)A; a.lda = lda;
  a.B = (const uint16_t*)B; a.bias = nullptr;
  a.C = (uint16_t*)C; a.ldc = ldc;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.P = 1; a.groups = 1;
  return launch<EPI_PLAIN, 256, 256>(a, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int trk_enc_dsc_gemm(const void* Y2, int64_t M, int64_t P, int64_t Kg, const void* W2,
                                const float* bias, int64_t Ng, void* XRN, long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 32 && P <= 256 && Kg % BK == 0 && Kg > 0 && Ng % 128 == 0 && Ng > 0,
              "enc_dsc_gemm: need 32 <= P <= 256, K %% 32 == 0, N %% 128 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(Y2 && W2 && bias && XRN && sums && aligned16(Y2) && aligned16(W2) && aligned16(XRN),
              "enc_dsc_gemm: null or unaligned pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EncGemmArgs a{};
  a.A = (const uint16_t*)Y2; a.lda = 2 * Kg;
  a.B = (const uint16_t*)W2; a.bias = bias;
  a.C = (uint16_t*)XRN; a.ldc = 2 * Ng;
  a.sums = sums; a.ld_sums = (int)(2 * Ng);
  a.M = (int)M; a.N = (int)Ng; a.K = (int)Kg; a.P = (int)P; a.groups = 2; a.kscale = 0;
  if (g_enc_gemm == 1 && P >= 43 && Ng % 256 == 0) return launch4<EPI_DSC>(a, st);
  return launch<EPI_DSC, 128, 128>(a, st);
}

extern "C" int trk_enc_transition_gemm(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s,
                                       int64_t kscale, const void* Wt, const float* bias, int64_t N,
                                       long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 32 && P <= 256 && K % BK == 0 && K > 0 && N % 256 == 0 && N > 0 &&
                  kscale % BK == 0 && kscale <= K,
              "enc_transition_gemm: need 32 <= P <= 256, K %% 32 == 0, N %% 256 == 0, kscale %% 32 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(XRN && s && Wt && bias && sums && aligned16(XRN) && aligned16(Wt) && aligned16(s),
              "enc_transition_gemm: null or unaligned pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EncGemmArgs a{};
  a.A = (const uint16_t*)XRN; a.lda = K;
  a.B = (const uint16_t*)Wt; a.bias = bias;
  a.sums = sums; a.ld_sums = (int)N;
  a.scale = s;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.P = (int)P; a.groups = 1; a.kscale = (int)kscale;
  if (g_enc_gemm >= 2 && P >= 86 && K % 64 == 0 && kscale % 64 == 0 && kscale <= 512)
    return g_enc_gemm == 2 ? launch8<EPI_TRANS, 0>(a, st) : launch8<EPI_TRANS, 1>(a, st);
  if (g_enc_gemm >= 1 && P >= 43 && kscale * G4_SLOTS <= G4_SQ * 256 * 4) return launch4<EPI_TRANS>(a, st);
  return launch<EPI_TRANS, 128, 256>(a, st);
}

extern "C" int trk_enc_g1_dwconv(const void* X, int64_t M, const void* W1, int64_t N, const float* wdw, void* Y2,
                                 void* stream) {
  TRK_REQUIRE(M >= 0 && M % 100 == 0 && N % 128 == 0 && N > 0,
              "enc_g1_dwconv: 10x10 ROIs (M %% 100 == 0), K = 512, N %% 128 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(X && W1 && wdw && Y2 && aligned16(X) && aligned16(W1) && aligned16(Y2) && aligned16(wdw),
              "enc_g1_dwconv: null or unaligned pointer");
  const int64_t nwg = (M / 200 + (M % 200 ? 1 : 0)) * (N / 128);
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_g1_dwconv: too many workgroups");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_kernel<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_kernel<1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_kernel<2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_persist_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1_LDS);
    attr = true;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (g_g1dw_persist == 66) {   // interleaved depthwise, one workgroup per CU
    static bool attr_il = false;
    if (!attr_il) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_il_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)IL_LDS);
      attr_il = true;
    }
    const int64_t grid = std::min<int64_t>(nwg, (int64_t)cu_count());
    hipLaunchKernelGGL(g1dw_il_kernel, dim3((unsigned)grid), dim3(512), IL_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N, nwg, next_queue_slot());
    return trk::check_launch("g1dw_il_kernel");
  }
  if (g_g1dw_mode == 6) {   // role-split: GEMM waves + depthwise waves, one workgroup per CU
    static bool attr_sp = false;
    if (!attr_sp) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_sp_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)IL_LDS);
      attr_sp = true;
    }
    const int64_t grid = std::min<int64_t>(nwg, (int64_t)cu_count());
    hipLaunchKernelGGL(g1dw_sp_kernel, dim3((unsigned)grid), dim3(1024), IL_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N, nwg, next_queue_slot(), g_enc_gemm_dbg);
    return trk::check_launch("g1dw_sp_kernel");
  }
  if (g_g1dw_persist > 0) {
    const int64_t grid = std::min<int64_t>(nwg, 2 * (int64_t)cu_count());
    hipLaunchKernelGGL(g1dw_persist_kernel, dim3((unsigned)grid), dim3(512), G1_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N, g_enc_gemm_dbg, nwg,
                       next_queue_slot(), g_g1dw_persist - 1);
    return trk::check_launch("g1dw_persist_kernel");
  }
  if (g_g1dw_mode == 5 && N % 256 == 0) {
    static bool attr_256 = false;
    if (!attr_256) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw256_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)G2_LDS);
      attr_256 = true;
    }
    const int64_t nwg2 = (M / 200 + (M % 200 ? 1 : 0)) * (N / 256);
    hipLaunchKernelGGL(g1dw256_kernel, dim3((unsigned)nwg2), dim3(1024), G2_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N);
    return trk::check_launch("g1dw256_kernel");
  }
  if (g_g1dw_mode == 7) {   // 4-wave workgroups, 112 x 64 wave tiles of 16x16x32
    static bool attr_q = false;
    if (!attr_q) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw4_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1Q_LDS);
      attr_q = true;
    }
    hipLaunchKernelGGL(g1dw4_kernel, dim3((unsigned)nwg), dim3(256), G1Q_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N, g_enc_gemm_dbg);
    return trk::check_launch("g1dw4_kernel");
  }
  if (g_g1dw_mode == 4) {
    TRK_REQUIRE(M * 512 < (int64_t)1 << 31, "enc_g1_dwconv: M * 512 must stay below 2^31");
    static bool attr_ws = false;
    if (!attr_ws) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw_ws_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1_LDS);
      attr_ws = true;
    }
    hipLaunchKernelGGL(g1dw_ws_kernel, dim3((unsigned)nwg), dim3(640), G1_LDS, st, (const uint16_t*)X,
                       (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N);
    return trk::check_launch("g1dw_ws_kernel");
  }
  auto kern = g_g1dw_mode == 1 ? g1dw_kernel<1> : g_g1dw_mode == 2 ? g1dw_kernel<2> : g1dw_kernel<0>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(512), G1_LDS, st, (const uint16_t*)X,
                     (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N, g_enc_gemm_dbg);
  return trk::check_launch("g1dw_kernel");
}

// diagnostics: gemm8 per-workgroup timestamps (PROF variant above); buf holds
// >= 16 * workgroups u64, nullptr switches back to the plain kernel
extern "C" int trk_enc_set_prof(unsigned long long* buf) {
  g_enc_prof = buf;
  return TRK_OK;
}
