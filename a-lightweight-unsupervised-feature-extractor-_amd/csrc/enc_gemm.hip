// bf16 GEMMs of the encoder (reference model/utils/modules/card.py: DSC :48-57,
// SEBlock :73-78, RMB.forward :128-148) for gfx950, with the elementwise work
// of the eval graph fused into their prologues / epilogues.  All on MFMA
// 16x16x32 bf16 with f32 accumulation:
//   rmb_front3 (trk_enc_rmb_front_means, the default front): per 10x10 ROI and DSC
//             group, the first 1x1 convs + depthwise 5x5 + the DSC 1x1 GEMM + BN +
//             activation, Y1 / Y2 only in LDS; writes [x_r | x_n] rows and the SE's
//             squeeze means.  A persistent grid, two workgroups per ROI on one XCD.
//   g1dw4 + gemm4<EPI_DSC> (trk_enc_g1_dwconv + trk_enc_dsc_gemm): the same front as two
//             kernels with Y2 in HBM (the alternative the front's tests compare against).
//   trans4 / gemm4<EPI_TRANS> (trk_enc_transition_gemm2): the SE excitation applied to
//             the staged x_f tiles, the transition GEMM + bias + SiLU and the per-ROI
//             sums of SiLU(T); T is never stored.  trans4 reads its weights straight
//             into VGPRs as pre-packed fragments; gemm4 streams them through LDS.
// Per-ROI sums leave the GEMMs as int64 fixed point (x 2^24) partials written with plain
// stores, so they do not depend on the order tiles finish in.
#include "trk_common.h"
#include "rb_linear.h"

#include <utility>

trk::DiagBuf g_enc_prof;  // trk_enc_set_prof (diagnostics: per-workgroup phase stamps)
int g_rf3_groups = 0;  // trk_set_tuning("rf3_groups"): rmb_front3 workgroup pairs per XCD (0 = CUs / 16 - 2)
int g_rf3_chunks = 1;  // trk_set_tuning("rf3_chunks"): rmb_front3 generations (each pair's ROIs in that many
                       // chunks, one workgroup each; 1 = one persistent generation)
int g_rf_pf = 1;  // trk_set_tuning("rf_pf"): rmb_front3 reads each K step's first X / Y fragment one step ahead
int g_enc_trans = 1;  // trk_set_tuning("enc_trans"): 1 = trans4 (weights straight into VGPRs, needs the
                      // packed fragments: trk_enc_transition_gemm2; 247.6 vs 281.5 us isolated, pipeline
                      // 1.981/1.939/1.968M vs 1.894/1.881/1.911M ROIs/s interleaved), 0 = gemm4 (through LDS)

namespace {

#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

enum { EPI_DSC = 0, EPI_TRANS = 1 };

constexpr int BK = 32;
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
  unsigned long long* prof;  // trk_enc_set_prof (gemm4: per-workgroup phase stamps; diagnostics)
};

__device__ __forceinline__ unsigned long long eg_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// lane ^ 1 without the LDS pipe (ds_bpermute): DPP quad_perm
__device__ __forceinline__ float lane_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t nx = 8;
  if (nwg < nx) return bid;
  int64_t q = nwg / nx, r = nwg % nx, x = bid % nx;
  int64_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

typedef float dw_pair_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return trk::pack2_bf16(a, b);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

constexpr int G1_BN = 128, G1_S = 10, G1_P = 100;  // g1dw4: N tile, ROI side, ROI rows

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
  // v_med3_f32 (one op) = min(max(c, 0), 6) for every non-NaN c
  const f2v r = f2v{__builtin_amdgcn_fmed3f(c.x, 0.0f, 6.0f), __builtin_amdgcn_fmed3f(c.y, 0.0f, 6.0f)};
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
constexpr int G4_SQ = 2;                    // s-tile DMA per thread (8 KiB)
constexpr size_t G4_STILE = (size_t)G4_SQ * 256 * 16;
constexpr size_t G4_STAGE = (size_t)128 * G4_SLD * 4;   // 66 KiB
constexpr size_t G4_RED = (size_t)G4_SLOTS * 256 * 8;   // 8 KiB
constexpr size_t G4_LDS = (G4_RING + G4_STILE) > (G4_STAGE + G4_RED) ? (G4_RING + G4_STILE) : (G4_STAGE + G4_RED);
static_assert(G4_LDS <= 80 * 1024, "two gemm4 workgroups per CU");

// HSWM: the DSC tile's activation (1 = Hardswish, the normal group), a compile-time constant
template <int EPI, int HSWM>
__device__ __forceinline__ void gemm4_tile(const EncGemmArgs& a, int64_t lb, unsigned char* smem) {
  constexpr int WMV = 2;                           // waves along M
  constexpr int NT = 128 * WMV, BM = 64 * WMV;   // threads, tile rows
  constexpr int ABUF = BM * 4, BUF = ABUF + 1024;  // uint4: A | B (256 rows) per ring stage
  constexpr int NB = 1024 / NT;                    // B DMA ops per thread per stage (A: 2)
  constexpr size_t RING = (size_t)3 * BUF * 16;
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
  const int64_t m0 = mt * BM;
  const uint16_t* Ag = a.A + (int64_t)g * a.K;
  const uint16_t* Bg = a.B + (int64_t)g * a.N * a.K;
  const int nk = a.K / BK;
  const int64_t roi_base = m0 / a.P;

  const uint16_t* asrc[2];
  const uint16_t* bsrc[NB];
  int arow[2], achk[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * NT + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    arow[q] = r;
    achk[q] = c;
    asrc[q] = Ag + min(m0 + r, (int64_t)a.M - 1) * a.lda + c * 8;
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int p = q * NT + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    bsrc[q] = Bg + (int64_t)(n0 + r) * a.K + c * 8;
  }
  auto issue = [&](int kt) {
    uint4* d = ring + (kt % 3) * BUF + wave * 64;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * NT), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < NB; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * BK), LPTR(d + ABUF + q * NT), 16, 0, 0);
  };
  // retire the oldest of two issued stages: the other stage's 2 + NB ops may stay in flight
  auto wait_older_stage = []() {
    if constexpr (NB == 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  };

  const float* stile = reinterpret_cast<const float*>(smem + RING);
  const float* srow[2] = {stile, stile};
  if constexpr (EPI == EPI_TRANS) {
    const int per = a.kscale / 4;
    const int64_t nroi = ((int64_t)a.M + a.P - 1) / a.P;
    // only the slots a tile can span (ceil(127 / P) + 1): the launch sizes LDS for them
    const int tslots = min(G4_SLOTS, (BM - 1 + a.P - 1) / a.P + 1);
#pragma unroll
    for (int q = 0; q < G4_SQ * 256 / NT; ++q) {
      const int p = q * NT + tid;
      if (p >= tslots * per) continue;
      const int slot = min(p / per, G4_SLOTS - 1);
      const int64_t roi = min(roi_base + slot, nroi - 1);
      const float* src = a.scale + roi * a.kscale + (p % per) * 4;
      __builtin_amdgcn_global_load_lds(GPTR(src), LPTR(reinterpret_cast<uint4*>(smem + RING) + q * NT + wave * 64),
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
        const uint32_t d = lds_addr(ring + (kt % 3) * BUF + tid);
        u32x4 v[2], s4[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          v[q] = lds_read128(d + q * NT * 16);
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
          lds_write128(d + q * NT * 16, o);
        }
      }
    }
  };

  const int fr = lane & 15, fc = lane >> 4;
  const int lterm = fr * 4 + (fc ^ x16(fr));
  const int aoff = (wr * 64) * 4 + lterm;            // + mt * 64
  const int boff = ABUF + (wc * 128) * 4 + lterm;    // + nt * 64

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
    wait_older_stage();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // the transition's s tile was landed by every wave's DMA, and transform reads any slot of
  // it: one barrier after each wave's own wait (the A elements it scales are its own DMA's)
  if constexpr (EPI == EPI_TRANS) g4_barrier();
  transform(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g4_barrier();

  // tile kt + 2's DMA is issued after step kt's MFMAs (its buffer was last read in
  // step kt - 1): the MFMAs start as soon as the fragments are read, and the DMA
  // issue -- which stalls while the memory pipeline is full -- runs beside them
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * BUF;
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
      if (kt + 2 < nk) wait_older_stage();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      transform(kt + 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_barrier();
  }

  if (prof) pst[1] = eg_stamp();
  // ---- epilogue (the ring is free: every DMA retired, all reads done at the last barrier)
  const int colq = wc * 128 + fr;  // + t * 16
  // HSWM: the tile's activation, known at compile time (straight-line SiLU or Hardswish)
  const bool hsw = EPI == EPI_DSC && HSWM == 1;
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
  float* part = reinterpret_cast<float*>(smem + (EPI == EPI_DSC ? G4_STAGE : (size_t)0));  // [WMV][SLOTS][256]
  {
    // the same partials on the MFMA: S[slot][col] = sum_rows mask[slot][row] * act[row][col]
    // as 16x16x32 bf16 MFMAs whose B operand is the accumulator fragments themselves --
    // lane (fr, fc) holds rows 4 fc + e of row tiles 2p and 2p + 1 for column fr, which
    // is exactly a B fragment (k = 8 fc + j) once the k -> row order below is used for
    // the mask too (A: lane (m = fr, fc), k = 8 fc + j -> row tile 2p + j / 4, row
    // 4 fc + j % 4).  The activations enter as a bf16 pair hi + lo (hi = bf16(x), lo =
    // bf16(x - hi): 16 significant bits, products with 1.0 exact, f32 accumulation).
    // Row rl of the tile belongs to slot (off + rl) / P, off = m0 - roi_base * P; P >= 43
    // so a 128-row tile holds at most 4 slots.  Lanes 0..15 end up with slots 0..3 (e).
    const int P = a.P;
    const int off = (int)(m0 - roi_base * P);
    bf8v mask[2];
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rl = wr * 64 + (2 * p2 + (j >> 2)) * 16 + 4 * fc + (j & 3);
        const int x = off + rl;
        const int slot = (x >= P) + (x >= 2 * P) + (x >= 3 * P);
        const bool on = slot == fr && m0 + rl < (int64_t)a.M;
        mask[p2][j] = on ? (__bf16)1.0f : (__bf16)0.0f;
      }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      f4v sacc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const f4v u = acc[2 * p2][t], v = acc[2 * p2 + 1][t];
        bf8v hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hi[e] = (__bf16)u[e];
          hi[4 + e] = (__bf16)v[e];
          lo[e] = (__bf16)(u[e] - (float)hi[e]);
          lo[4 + e] = (__bf16)(v[e] - (float)hi[4 + e]);
        }
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mask[p2], hi, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mask[p2], lo, sacc, 0, 0, 0);
      }
      if (lane < 16) {
#pragma unroll
        for (int ts = 0; ts < G4_SLOTS; ++ts) part[(wr * G4_SLOTS + ts) * 256 + colq + t * 16] = sacc[ts];
      }
    }
  }
  if (prof) pst[3] = eg_stamp();
  if (EPI == EPI_DSC) {
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
    const int64_t last_row = min(m0 + BM, (int64_t)a.M) - 1;
    const int nslot = (int)(last_row / a.P - roi_base) + 1;
    for (int q = tid; q < nslot * 256; q += NT) {
      const int slot = q >> 8, c = q & 255;
      const int64_t roi = roi_base + slot;
      long long v = 0;
#pragma unroll
      for (int w = 0; w < WMV; ++w) v += llrintf(part[(w * G4_SLOTS + slot) * 256 + c] * kFix);
      // partial j = the ROI's 128-row block index (the tile's own block)
      const int64_t rb0 = roi * a.P / kPartRows;
      const int64_t tb0 = max(m0 / kPartRows, rb0);
      a.sums[(roi * kPart + (tb0 - rb0)) * a.ld_sums + g * a.N + n0 + c] = v;
    }
  }
  if (prof) pst[5] = eg_stamp();
  if (EPI == EPI_DSC) {
    const uint32_t* stage = reinterpret_cast<const uint32_t*>(smem);
    const int64_t cbase = (int64_t)g * a.N + n0;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int p = q * NT + tid, rl = p >> 5, c8 = (p & 31) * 8;
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

// one workgroup per tile (XCD-remapped); a DSC tile's group (SiLU / Hardswish) is a
// template argument of its body, so each body is straight-line (a per-element select
// was compiled into 64 branches of nop-padded exp / rcp chains)
template <int EPI>
__global__ void __launch_bounds__(256, 2) gemm4_kernel(EncGemmArgs a, int64_t ntiles) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t lb = xcd_remap(blockIdx.x, ntiles);
  if (EPI == EPI_DSC && (lb % (a.N / 256 * a.groups)) / (a.N / 256) == 1) gemm4_tile<EPI, 1>(a, lb, smem);
  else gemm4_tile<EPI, 0>(a, lb, smem);
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
      dst[((OY0 + oy) * G1_S + X0 + ox) * ldd] = v;
    }
}


__global__ void __launch_bounds__(256, 2) g1dw4_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                        const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                        int M, int N) {
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

  const int nk = NK;
  issue(0);
  issue(1);
  wait_prev();
  g4_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * G1Q_BUF;
    {
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
  // L2 prefetch of the A rows of the tile this slot most likely
  // runs next (xcd_remap's order: logical tile lb + 64 runs on this XCD after lb), an eighth
  // of its M tile per N tile, issued now so the depthwise below covers its HBM latency
  // (28 us of 389 isolated); retired by the kernel's end, nothing waits on it before
  uint32_t pf = 0;
  {
    const int64_t tn = lb + 64;
    const int64_t xs = (int64_t)gridDim.x / 8;   // logical tiles per XCD range (remap: contiguous)
    if (tn / xs == lb / xs && tn < (int64_t)gridDim.x && tid < 208) {
      const int part = (int)(tn % ntile_n);
      const int64_t row = min((tn / ntile_n) * (2 * G1_P) + (part * 26 + (tid >> 3)), (int64_t)M - 1);
      const uint16_t* pa = X + row * K + (tid & 7) * 64;
      // (an inline-asm load's destination is written when the load returns: pf stays live,
      // so its register is not reused, until the wait at the end)
      asm volatile("global_load_dword %0, %1, off" : "+v"(pf) : "v"(pa) : "memory");
    }
  }

  // depthwise 5x5: wave = output quadrant, for each of the two ROIs; lane = channel pair
  const int ldd = N / 2;
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
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(pf)::"memory");
}


// ---------------------------------------------------------------------------
// rmb_front3: one DSC of the RMB end to end for 10x10 ROIs (card.py:28-57: the
// branch's first 1x1 convs, the depthwise 5x5, depth.2 + point.2 with eval-BN folded,
// the activation, and the SE's squeeze means).  Y1 and Y2 live only in LDS; HBM sees X
// and the [x_r | x_n] rows (XRN).  A workgroup runs one DSC group G (0 reinforce /
// SiLU, 1 normal / Hardswish) for the ROIs roi0, roi0 + stride, ... (persistent grid).
//
// 8 waves, one workgroup per CU.  Wave w owns output columns 64 w .. 64 w + 63 of the
// group's 512 in BOTH GEMMs and all 112 rows (7 row tiles of 16; rows 100..111 are
// padding whose results are dropped): a 112 x 64 wave tile of 16x16x32 MFMAs, 112
// accumulator registers.  No weight element is used by two waves, so weights do not go
// through LDS: they are pre-packed on the host in MFMA fragment order ([g][k step][16-col
// tile][lane] x 16 B), and a wave's four fragments of a K step are one contiguous 4 KiB
// read straight into VGPRs, two steps ahead.  The ROI's X rows (shared by the 8 waves)
// are staged by LDS-DMA into the LDS image Y1 and Y2 use later: K blocks of 32 channels,
// 100 rows x 64 B per block (row r's 16-B chunk c at slot r*4 + (c ^ sw(r)), sw(r) =
// (r >> 1) & 3: conflict-free ds_read_b128 fragment reads, 2-way 8-B row writes), block
// stride 6464 B so the depthwise's 4-B channel-pair reads of two blocks fall on different
// banks.  X arrives in four groups of four blocks, each issued four K steps ahead (a
// per-step barrier kept the 8 waves' LDS reads in lockstep).  Both GEMMs are computed
// transposed (weights = A operand), so a lane holds 4 consecutive channels of one pixel.
// Same MFMA shape, K order and roundings (Y1 and Y2 to bf16) as g1dw4 + gemm4<DSC>: XRN is
// bit-identical to the two-kernel path; the means add the same f32 activations in
// another order.
constexpr int RF_S = 100;                                      // rows per ROI
constexpr int RF_KBS = 1616;                                   // block stride (dwords): 6400 B + 64

// s_waitcnt vmcnt(n) for a (compile-time after unrolling) n, tied to the four fragment registers
__device__ __forceinline__ void rf_vmwait(int n, u32x4 (&b)[4]) {
#define RF_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])::"memory"); break;
  switch (n) {
    RF_VMW(1) RF_VMW(2) RF_VMW(3) RF_VMW(4) RF_VMW(5) RF_VMW(6) RF_VMW(7) RF_VMW(8) RF_VMW(9) RF_VMW(10)
    RF_VMW(11) RF_VMW(12) RF_VMW(13) RF_VMW(14) RF_VMW(15) RF_VMW(16) RF_VMW(17) RF_VMW(18) RF_VMW(19)
    RF_VMW(20) RF_VMW(21) RF_VMW(22) RF_VMW(23) RF_VMW(24)
    default: asm volatile("s_waitcnt vmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])::"memory");
  }
#undef RF_VMW
}

struct RfArgs {
  const uint16_t* X;    // [R * 100][512] bf16 NHWC ROI rows
  const uint4* W1p;     // [2][16][32][64] 16-B fragments of W1 (group g: rows 512 g ..)
  const float* wdw;     // [25][1024] depthwise taps
  const uint4* W2p;     // [2][16][32][64] fragments of the BN-folded DSC weights
  const float* bias;    // [1024] BN-folded bias
  uint16_t* XRN;        // [R * 100][1024] = [SiLU(x_r) | Hardswish(x_n)]
  float *m_r, *m_n;     // [R][512] the squeeze means of SiLU(x_r) / Hardswish(x_n) (trk_enc_se's)
  int64_t R;            // ROIs
  int pairs, chunks;    // rmb_front3's grid: workgroup pairs per XCD, generations (ROI chunks)
  unsigned long long* prof;  // trk_enc_set_prof: every wave's phase cycles per ROI (diagnostics)
  uint32_t* progress;        // the launch's `progress` argument: +1 per finished ROI (group 0's workgroup), or null
};

__device__ __forceinline__ int rf_sw(int s) { return (s >> 1) & 3; }
// depthwise 5x5 of output quadrant (QY, QX) for the lane's channel pair, results
// held as packed bf16 pairs (the caller writes them back in place after a barrier);
// same per-output FMA order as dw5q_regs.  Pixel s sits at dword b[rf_sw(s)] + 16 s (s is
// a constant after unrolling).
template <int QY, int QX>
__device__ __forceinline__ void rf_dw5q(const uint32_t* y, const int (&b)[4], const dw_pair_t (&w)[25],
                                        uint32_t (&out)[25]) {
  constexpr int OY0 = 5 * QY, X0 = 5 * QX;
  constexpr int IY0 = OY0 - 2 < 0 ? 0 : OY0 - 2, IY1 = OY0 + 6 > G1_S - 1 ? G1_S - 1 : OY0 + 6;
  constexpr int IX0 = X0 - 2 < 0 ? 0 : X0 - 2, IX1 = X0 + 6 > G1_S - 1 ? G1_S - 1 : X0 + 6;
  constexpr int NX = IX1 - IX0 + 1;
  auto at = [&](int s) { return y[b[rf_sw(s)] + s * 16]; };
  dw_pair_t acc[5][5];
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) acc[oy][ox] = dw_pair_t{0.f, 0.f};
  uint32_t nxt[NX];
#pragma unroll
  for (int ix = 0; ix < NX; ++ix) nxt[ix] = at(IY0 * G1_S + IX0 + ix);
#pragma unroll
  for (int iy = IY0; iy <= IY1; ++iy) {
    dw_pair_t in[NX];
#pragma unroll
    for (int ix = 0; ix < NX; ++ix) in[ix] = dw_pair_t{__uint_as_float(nxt[ix] << 16), __uint_as_float(nxt[ix] & 0xffff0000u)};
    if (iy < IY1) {
#pragma unroll
      for (int ix = 0; ix < NX; ++ix) nxt[ix] = at((iy + 1) * G1_S + IX0 + ix);
    }
#pragma unroll
    for (int oy = 0; oy < 5; ++oy) {
      const int ky = iy - (OY0 + oy) + 2;
      if (ky < 0 || ky > 4) continue;
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
#pragma unroll
        for (int ox = 0; ox < 5; ++ox) {
          const int ix = X0 + ox + kx - 2;
          if (ix >= IX0 && ix <= IX1) {
            acc[oy][ox] = __builtin_elementwise_fma(w[ky * 5 + kx], in[ix - IX0], acc[oy][ox]);
          }
        }
        asm volatile("" : "+v"(acc[oy][0]), "+v"(acc[oy][1]), "+v"(acc[oy][2]), "+v"(acc[oy][3]), "+v"(acc[oy][4]));
      }
    }
  }
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) out[oy * 5 + ox] = pack_bf16x2(acc[oy][ox].x, acc[oy][ox].y);
}
template <int QY, int QX>
__device__ __forceinline__ void rf_dw5q_store(uint32_t* y, const int (&b)[4], const uint32_t (&out)[25]) {
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) {
      const int s = (5 * QY + oy) * G1_S + 5 * QX + ox;
      y[b[rf_sw(s)] + s * 16] = out[oy * 5 + ox];
    }
}

// the wave's four B fragments of k step kt (4 KiB contiguous): asm loads, so the issue order
// is the program order and the caller's counted vmcnt waits are exact
__device__ __forceinline__ void rf_loadB(const uint4* bp, int kt, u32x4 (&d)[4]) {
  asm volatile("" : "+v"(bp));  // per call: keeps the compiler from hoisting all 32 step addresses
  const uint4* p = bp + kt * 32 * 64;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d[0]) : "v"(p) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(d[1]) : "v"(p) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off offset:2048" : "=v"(d[2]) : "v"(p) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off offset:3072" : "=v"(d[3]) : "v"(p) : "memory");
}

// one K step of the wave's 64-channel x 112-pixel tile, computed transposed (C = W . X^T:
// the weight fragments are the A operand, the activation rows the B operand, so lane
// (fr, fc) of tile (i, t) ends up with channels 16 t + 4 fc .. + 3 of pixel 16 i + fr, four
// consecutive channels of one pixel = one 8-B LDS store).  The 7 pixel-tile fragments
// (tile i at byte ab + 1024 i of an LDS image) are read up front, then each tile's 4 MFMAs
// wait (counted lgkmcnt) for its own fragment only, as g1dw4
__device__ __forceinline__ void rf_mfma_step(uint32_t ab, const u32x4 (&b)[4], f4v (&acc)[7][4]) {
  u32x4 aq[7];
  asm volatile("ds_read_b128 %0, %1" : "=v"(aq[0]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(aq[1]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(aq[2]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(aq[3]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(aq[4]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(aq[5]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(aq[6]) : "v"(ab) : "memory");
  // the waits are not tied to aq[i] ("+v" made the compiler treat the asm as a VALU write of
  // the MFMA's B operand and pad every wait with an s_nop: 224 per wave and ROI); the
  // scheduling barriers keep each tile's MFMAs behind its wait (tests/test_isa.py checks
  // the compiled order)
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    if (i == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
    else if (i == 1) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
    else if (i == 2) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    else if (i == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
    else if (i == 4) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    else if (i == 5) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bf8v xf = __builtin_bit_cast(bf8v, aq[i]);
#pragma unroll
    for (int t = 0; t < 4; ++t)
      acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, b[t]), xf, acc[i][t], 0, 0, 0);
  }
}

// rf_mfma_step with the first fragment read one step ahead: PRE, tile 0's fragment is already in
// `pre` (its ds_read issued during the previous step, possibly still in flight: it is older than
// this step's six reads, so the tile-0 wait lgkmcnt(6) retires it); NEXT, the next step's tile-0
// fragment (LDS byte address nab) is read into `pre` after tile 3's MFMAs, so the next step's
// first MFMAs do not wait for an LDS read the partner wave may not cover (the read is younger
// than tiles 4..6's: their waits count it).  The caller passes NEXT only where the next step's
// block is already in LDS without a wait in between (not across an X group boundary or the
// Y2(B) hand-off)
template <bool PRE, bool NEXT>
__device__ __forceinline__ void rf_mfma_step_pf(uint32_t ab, const u32x4 (&b)[4], f4v (&acc)[7][4], u32x4& pre,
                                                uint32_t nab) {
  u32x4 aq[7];
  if constexpr (!PRE) asm volatile("ds_read_b128 %0, %1" : "=v"(aq[0]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(aq[1]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(aq[2]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:3072" : "=v"(aq[3]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(aq[4]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:5120" : "=v"(aq[5]) : "v"(ab) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(aq[6]) : "v"(ab) : "memory");
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    if (i == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
    else if (i == 1) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
    else if (i == 2) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    else if (i == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
    else if (i == 4) {
      if constexpr (NEXT) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    } else if (i == 5) {
      if constexpr (NEXT) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
    } else {
      if constexpr (NEXT) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    const bf8v xf = __builtin_bit_cast(bf8v, (PRE && i == 0) ? pre : aq[i]);
#pragma unroll
    for (int t = 0; t < 4; ++t)
      acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, b[t]), xf, acc[i][t], 0, 0, 0);
    if constexpr (NEXT) {
      if (i == 3) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("ds_read_b128 %0, %1" : "=v"(pre) : "v"(nab) : "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}
// one K step with the prefetch flags as compile-time constants of the unrolled loops
__device__ __forceinline__ void rf_step_pf(bool pre_in, bool next, uint32_t ab, const u32x4 (&b)[4],
                                           f4v (&acc)[7][4], u32x4& pre, uint32_t nab) {
  if (pre_in) {
    if (next) rf_mfma_step_pf<true, true>(ab, b, acc, pre, nab);
    else rf_mfma_step_pf<true, false>(ab, b, acc, pre, nab);
  } else {
    if (next) rf_mfma_step_pf<false, true>(ab, b, acc, pre, nab);
    else rf_mfma_step_pf<false, false>(ab, b, acc, pre, nab);
  }
}

// Decoupled halves: half A (waves 0..3, one per SIMD) produces Y1 / Y2 channels 0..255 and
// half B (waves 4..7) channels 256..511; the depthwise of a half only reads its own half's Y1,
// so the only cross-half dependencies are GEMM2's K steps 8..15 (Y2(B)) and the LDS regions
// the halves reuse.  Those are tracked by LDS counters (a wave adds 1 after its LDS writes or
// DMA have landed; a waiter polls with s_sleep) that count on across the workgroup's ROIs
// (targets 4 (it + 1)).  B starts GEMM1 behind A's (they share every SIMD's matrix pipe), so
// on every SIMD one wave's depthwise / activation VALU runs beside its partner's MFMAs.
// LDS (blocks of RF_KBS dwords): blocks 0..15 = X for GEMM1 (both halves), blocks 16..23 =
// Y(A); once both halves finished GEMM1, blocks 8..15 = Y(B) and blocks 0..7 = A's output
// staging; B stages over Y(A) after both halves' GEMM2.
constexpr int RF2_NB = 24;
constexpr size_t RF2_CTR = (size_t)(RF2_NB - 1) * RF_KBS * 4 + 112 * 64;  // past block 23's row-111 reads
enum { RF2_CX = 0, RF2_CG1 = 4, RF2_CY1 = 6, RF2_CDW = 8, RF2_CY2 = 12, RF2_CG2 = 14, RF2_CST = 16, RF2_CSD = 18,
       RF2_NCTR = 20 };
constexpr size_t RF2_LDS = RF2_CTR + RF2_NCTR * 4;
constexpr int RF2_SROW = 128;  // output staging row (dwords): 256 channels, 16-B chunks XOR-swizzled by row
static_assert(RF2_LDS <= 160 * 1024, "one rmb_front workgroup per CU");
static_assert((size_t)RF_S * RF2_SROW * 4 <= (size_t)8 * RF_KBS * 4, "a half's staging fits 8 blocks");
constexpr uint32_t kRf2Spin = 1u << 22;  // poll bound (~0.1 s): a lost signal ends the wait, never hangs

// Y block of K block kb (32 channels): channels 0..255 in blocks 16..23, 256..511 in 8..15
__device__ __forceinline__ int rf2_yblk(int kb) { return kb < 8 ? kb + 16 : kb; }
__device__ __forceinline__ int rf2_yaddr(int s, int col) {
  const int kb = col >> 5, c = (col & 31) >> 3, d = (col & 7) >> 1;
  return rf2_yblk(kb) * RF_KBS + s * 16 + ((c ^ rf_sw(s)) << 2) + d;
}
// this wave's LDS writes (and any LDS-DMA it waited for) have landed: count it (lane 0
// only).  Both hand-off halves are single asm statements: a C++ loop or lane branch here
// splits the unrolled K loops' scheduling regions (1.2 KB of spills per lane)
__device__ __forceinline__ void rf2_signal(uint32_t* ctr, int) {
  uint64_t saved;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 %[e], exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %[a], %[one]\n\t"
      "s_mov_b64 exec, %[e]"
      : [e] "=&s"(saved)
      : [a] "v"(lds_addr(ctr)), [one] "v"(1u)
      : "memory");
}
// poll the counter until it reaches target (bounded: a lost signal ends the wait)
__device__ __forceinline__ void rf2_wait(uint32_t* ctr, uint32_t target) {
  uint32_t v, sv, n;
  asm volatile(
      "s_mov_b32 %[n], 0\n"
      "1:\n\t"
      "ds_read_b32 %[v], %[a]\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %[s], %[v]\n\t"
      "s_cmp_ge_u32 %[s], %[t]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_add_u32 %[n], %[n], 1\n\t"
      "s_cmp_gt_u32 %[n], %[lim]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n"
      "2:"
      : [v] "=&v"(v), [s] "=&s"(sv), [n] "=&s"(n)
      : [a] "v"(lds_addr(ctr)), [t] "s"(target), [lim] "s"(kRf2Spin)
      : "memory", "scc");
}

// 16-B LDS-DMA of every lane (LDS byte address base + 16 lane); and of lanes 0..35 only
__device__ __forceinline__ void rf_dma16(const void* g, uint32_t base) {
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(base) : "memory");
}
__device__ __forceinline__ void rf_dma16_lanes36(const void* g, uint32_t base) {
  uint64_t saved;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[mk]\n\t"
      "global_load_lds_dwordx4 %[g], off\n\t"
      "s_mov_b64 exec, %[sv]"
      : [sv] "=&s"(saved)
      : [mk] "s"(0xFFFFFFFFFull), [b] "{m0}"(base), [g] "v"(g)
      : "memory");
}

// per-channel sums of the wave's activated tile: xor 1, xor 2,
// row_ror 8, row_ror 4 is a butterfly (row_ror 4 before 8 is not: lanes 0 and 4 would add
// the quads in different orders), so every lane of a 16-lane row holds the same 16 sums;
// lane fr returns the one of channel 16 (fr >> 2) + 4 fc + (fr & 3) (rf_lane_ch), so the
// fixed-point conversions run once per channel instead of 16 times on lanes fr == 0
__device__ __forceinline__ int rf_lane_ch(int wave, int fr, int fc) {
  return wave * 64 + (fr >> 2) * 16 + fc * 4 + (fr & 3);
}
__device__ __forceinline__ float rf_colsum(const f4v (&acc)[7][4], int fr) {
  float mine = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = 0.f;
#pragma unroll
      for (int i = 0; i < 6; ++i) x += acc[i][t][e];
      if (fr < 4) x += acc[6][t][e];
      x += lane_xor1(x);
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // ^2
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xF, 0xF, true));  // row_ror 8
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x124, 0xF, 0xF, true));  // row_ror 4
      mine = (fr == t * 4 + e) ? x : mine;
    }
  }
  return mine;
}
// the squeeze mean of a sum as trk_enc_se takes it: (float)(llrint(sum * 2^24) * 2^-24) / 100
__device__ __forceinline__ float rf_mean(float sum) {
  return (float)((double)llrintf(sum * kFix) * (1.0 / 16777216.0)) / (float)RF_S;
}
// The workgroup's ROIs roi0, roi0 + stride, ...: ROI it + 1's X DMA and GEMM1 start as soon as
// the blocks they need are free, so half A's GEMM1 of the next ROI runs under half B's epilogue
// of this one instead of behind a workgroup boundary
template <int G, bool PF>
__device__ __forceinline__ void rf2_body(const RfArgs& a, unsigned char* smem, int64_t roi0, int64_t stride,
                                         int64_t roi_end) {
  uint32_t* Y = reinterpret_cast<uint32_t*>(smem);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(smem + RF2_CTR);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = wave >> 2, hw = wave & 3;  // half A = 0, B = 1; wave within the half
  constexpr int NK = 512 / BK;
  const bool prof = a.prof != nullptr;
  if (threadIdx.x < RF2_NCTR) ctr[threadIdx.x] = 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g4_barrier();  // the only full barrier: counters zeroed
  int64_t roi = roi0;
  for (uint32_t it = 0; roi < roi_end; ++it, roi += stride) {
  const uint32_t t4 = 4u * (it + 1), p4 = 4u * it;  // counter targets: this ROI's / the previous one's
  // lane-dependent values re-derived per ROI through an opaque copy: hoisted out of the ROI
  // loop, every address the body derives from them stayed live across it (268 VGPRs spilled)
  int tid_o = threadIdx.x;
  asm volatile("" : "+v"(tid_o));
  const int tid = tid_o, lane = tid & 63;
  const int fr = lane & 15, fc = lane >> 4;
  unsigned long long pst[8];
  unsigned long long rt0 = 0;
  if (prof) {
    pst[0] = eg_stamp();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  const int64_t r0 = roi * RF_S;

  // X -> blocks 0..15, moved by half A only (2 DMA ops per block per wave: pieces
  // 100 hw + lane and 100 hw + 64 + lane < 400, piece p = row p >> 2, slot p & 3)
  const int xp1 = 100 * hw + lane, xp2 = 100 * hw + 64 + lane;
  const uint16_t* xs1 = a.X + (r0 + (xp1 >> 2)) * 512 + (((xp1 & 3) ^ rf_sw(xp1 >> 2)) * 8);
  const uint16_t* xs2 = a.X + (r0 + min(xp2 >> 2, RF_S - 1)) * 512 + (((xp2 & 3) ^ rf_sw(xp2 >> 2)) * 8);
  // the X DMA as asm (M0 and, for the 36-lane second op, exec set explicitly): with the
  // builtin under `if (lane < 36)` the persistent variant's compiler merged the two ops of
  // consecutive blocks across the divergent region and issued a 36-lane op with every lane
  const uint32_t ybase = lds_addr(Y);
  auto issueX = [&](int grp) {
    const uint16_t* p1 = xs1;
    const uint16_t* p2 = xs2;
    asm volatile("" : "+v"(p1), "+v"(p2));  // per group: the block addresses are not all hoisted
#pragma unroll
    for (int kb = 4 * grp; kb < 4 * grp + 4; ++kb) {
      const uint32_t d = __builtin_amdgcn_readfirstlane(ybase + (kb * RF_KBS + 400 * hw) * 4);
      rf_dma16(p1 + kb * BK, d);
      rf_dma16_lanes36(p2 + kb * BK, d + 1024);
    }
  };
  const uint4* b1p = a.W1p + ((size_t)G * NK * 32 + wave * 4) * 64 + lane;
  const uint4* b2p = a.W2p + ((size_t)G * NK * 32 + wave * 4) * 64 + lane;
  u32x4 bq[3][4];
  const int lterm = fr * 4 + (fc ^ rf_sw(fr));
  const uint32_t y_a = lds_addr(Y) + lterm * 16;

  f4v acc[7][4];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};
  u32x4 apre = {0u, 0u, 0u, 0u};  // PF: the next K step's tile-0 fragment (rf_mfma_step_pf)

  // ---- GEMM1 (K = 512 over X blocks 0..15); A: 8 DMA ops per group, B: none.  One
  // loop per half (HALF a template constant): a half test inside the unrolled loop costs
  // spills.  Before the previous ROI's blocks are overwritten (targets 0 on the first ROI),
  // half A's staging reads (X blocks 0..7) and both halves' GEMM2 (blocks 8..15 held Y2(B))
  // are done
  auto gemm1 = [&](auto half_c) {
    constexpr int HALF = decltype(half_c)::value;
    if (HALF == 0) {
      // X groups 0 and 1 (blocks 0..7) go where half A staged the previous ROI's output:
      // free once A's stores read it, while half B may still run that ROI's GEMM2 (over
      // blocks 8..23); groups 2 and 3 wait for both halves' GEMM2 (blocks 8..15 held Y2(B))
      rf2_wait(ctr + RF2_CSD + 0, p4);
      issueX(0);
      issueX(1);
    }
    rf_loadB(b1p, 0, bq[0]);
    rf_loadB(b1p, 1, bq[1]);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      u32x4(&b)[4] = bq[kt % 3];
      if (HALF == 0) {
        // group boundary: vmcnt(0) (an LDS-DMA may retire after younger VGPR loads), count
        // this wave's share of the group, wait for the other three
        if (kt % 4 == 0) {
          // PF: LDS-DMA and loads retire in issue order (MI355X_MICROARCH.md, s_waitcnt vmcnt), so
          // vmcnt(4) retires this group's DMA (issued before B(kt)) and leaves B(kt + 1) in flight;
          // else vmcnt(0)
          rf_vmwait(PF ? 4 : 0, b);
          rf2_signal(ctr + RF2_CX + kt / 4, lane);
          rf2_wait(ctr + RF2_CX + kt / 4, t4);
          if (kt == 4) {
            rf2_wait(ctr + RF2_CG2 + 0, p4);
            rf2_wait(ctr + RF2_CG2 + 1, p4);
          }
          if (kt / 4 + 1 >= 2 && kt / 4 + 1 < 4) issueX(kt / 4 + 1);
        } else {
          // ops issued after B(kt): X group (kt - 1) / 4 + 1 when step kt - 1 issued one, B(kt + 1)
          rf_vmwait(((kt - 1) % 4 == 0 && (kt - 1) / 4 + 1 >= 2 && (kt - 1) / 4 + 1 < 4 ? 8 : 0) +
                        (kt + 1 < NK ? 4 : 0),
                    b);
        }
      } else {
        rf_vmwait(kt + 1 < NK ? 4 : 0, b);
        if (kt % 4 == 0) rf2_wait(ctr + RF2_CX + kt / 4, t4);
      }
      if (kt + 2 < NK) rf_loadB(b1p, kt + 2, bq[(kt + 2) % 3]);
      // PF: the next step's first fragment read ahead, except into a group's first step (its
      // block is waited for there)
      rf_step_pf(PF && kt % 4 != 0, PF && kt + 1 < NK && (kt + 1) % 4 != 0, y_a + kt * RF_KBS * 4, b, acc, apre,
                 y_a + (kt + 1) * RF_KBS * 4);
    }
  };
  __builtin_amdgcn_s_setprio(1);
  if (half == 0) {
    gemm1(std::integral_constant<int, 0>{});
  } else {
    // B starts after A's whole GEMM1: run together, the two halves share every SIMD's
    // matrix pipe and reach their VALU phases together (measured: lag 0 / 8 / 12 K steps tie
    // or lose)
    rf2_wait(ctr + RF2_CG1 + 0, t4);
    gemm1(std::integral_constant<int, 1>{});
  }
  __builtin_amdgcn_s_setprio(0);
  rf2_signal(ctr + RF2_CG1 + half, lane);  // this wave's reads of X are done
  if (prof) {
    asm volatile("" ::"v"(acc[6][3][3]));
    pst[1] = eg_stamp();
  }
  // B's Y1 goes over X blocks 8..15: every wave of both halves must be past GEMM1; A's over
  // blocks 16..23, which held the previous ROI's B staging until B's stores read it
  if (half == 1) {
    rf2_wait(ctr + RF2_CG1 + 0, t4);
    rf2_wait(ctr + RF2_CG1 + 1, t4);
  } else {
    rf2_wait(ctr + RF2_CSD + 1, p4);
  }
  // ---- Y1 -> LDS (the wave's 64 channels of its half's region)
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int px = i * 16 + fr;
    if (px < RF_S) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4v v = acc[i][t];
        *reinterpret_cast<uint2*>(Y + rf2_yaddr(px, wave * 64 + t * 16 + fc * 4)) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  }
  const int cg = wave >> 1;  // the wave's 128 depthwise channels (in its own half)
  dw_pair_t wreg[25];
  {
    const float* wp = a.wdw + G * 512 + cg * 128 + 2 * lane;
#pragma unroll
    for (int k = 0; k < 25; ++k)
      asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(wreg[k]) : "v"(wp + k * 1024) : "memory");
  }
  rf_loadB(b2p, 0, bq[0]);
  rf_loadB(b2p, 1, bq[1]);
  rf2_signal(ctr + RF2_CY1 + half, lane);
  rf2_wait(ctr + RF2_CY1 + half, t4);  // the half's Y1 is in
  if (prof) pst[2] = eg_stamp();
  asm volatile("s_waitcnt vmcnt(8)" : "+v"(wreg[0]), "+v"(wreg[1]), "+v"(wreg[2]), "+v"(wreg[3]), "+v"(wreg[4]),
               "+v"(wreg[5]), "+v"(wreg[6]), "+v"(wreg[7]), "+v"(wreg[8]), "+v"(wreg[9]), "+v"(wreg[10]),
               "+v"(wreg[11]), "+v"(wreg[12])::"memory");
  asm volatile("" : "+v"(wreg[13]), "+v"(wreg[14]), "+v"(wreg[15]), "+v"(wreg[16]), "+v"(wreg[17]), "+v"(wreg[18]),
               "+v"(wreg[19]), "+v"(wreg[20]), "+v"(wreg[21]), "+v"(wreg[22]), "+v"(wreg[23]), "+v"(wreg[24]));
  // L2 prefetch of the workgroup's next ROI's X: one dword of every 128-B line (100 KB, 800
  // lines: 1-2 loads per thread) loaded now, ~40K cycles before that ROI's DMA, so the DMA finds
  // it in L2 (per ROI 60.6K vs 65.1K cycles, GEMM1 13.4K vs 18.4K; pipeline 2.077-2.089 vs
  // 2.050-2.065M ROIs/s in three interleaved pairs).  Younger than GEMM2's first weight loads,
  // so GEMM2's counted waits only get stricter; the destinations stay live until GEMM2's last
  // wait retires them
  uint32_t xpf0 = 0, xpf1 = 0;
  if (roi + stride < roi_end) {
    const uint16_t* nx = a.X + (roi + stride) * RF_S * 512;
    asm volatile("global_load_dword %0, %1, off" : "+v"(xpf0) : "v"(nx + tid * 64) : "memory");
    if (tid < 800 - 512) asm volatile("global_load_dword %0, %1, off" : "+v"(xpf1) : "v"(nx + (tid + 512) * 64) : "memory");
  }

  // ---- depthwise 5x5 in place: waves 2 cg and 2 cg + 1 own the two output halves of the
  // same 128 channels, so the read-before-overwrite hand-off is between those two only
  {
    const int kb0 = rf2_yblk(cg * 4 + (lane >> 4)), c0 = (lane & 15) >> 2, d0 = lane & 3;
    const int yb[4] = {kb0 * RF_KBS + (c0 << 2) + d0, kb0 * RF_KBS + ((c0 ^ 1) << 2) + d0,
                       kb0 * RF_KBS + ((c0 ^ 2) << 2) + d0, kb0 * RF_KBS + ((c0 ^ 3) << 2) + d0};
    uint32_t o0[25], o1[25];
    if ((wave & 1) == 0) {
      rf_dw5q<0, 0>(Y, yb, wreg, o0);
      rf_dw5q<0, 1>(Y, yb, wreg, o1);
      rf2_signal(ctr + RF2_CDW + cg, lane);
      rf2_wait(ctr + RF2_CDW + cg, 2 * (it + 1));
      rf_dw5q_store<0, 0>(Y, yb, o0);
      rf_dw5q_store<0, 1>(Y, yb, o1);
    } else {
      rf_dw5q<1, 0>(Y, yb, wreg, o0);
      rf_dw5q<1, 1>(Y, yb, wreg, o1);
      rf2_signal(ctr + RF2_CDW + cg, lane);
      rf2_wait(ctr + RF2_CDW + cg, 2 * (it + 1));
      rf_dw5q_store<1, 0>(Y, yb, o0);
      rf_dw5q_store<1, 1>(Y, yb, o1);
    }
  }
  rf2_signal(ctr + RF2_CY2 + half, lane);
  if (prof) pst[3] = eg_stamp();

  // ---- GEMM2: K steps 0..7 read Y2(A), 8..15 Y2(B)
  float4 bias4[4];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    u32x4(&b)[4] = bq[kt % 3];
    rf_vmwait(kt + 1 < NK ? 4 : 0, b);
    if (kt == 0) rf2_wait(ctr + RF2_CY2 + 0, t4);
    if (kt == 8) rf2_wait(ctr + RF2_CY2 + 1, t4);
    if (kt + 2 < NK) rf_loadB(b2p, kt + 2, bq[(kt + 2) % 3]);
    if (kt == NK - 3) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bias4[t] = *reinterpret_cast<const float4*>(a.bias + G * 512 + wave * 64 + t * 16 + fc * 4);
    }
    // PF: read ahead except into steps 0 and 8 (waits for the halves' Y2)
    rf_step_pf(PF && kt != 0 && kt != 8, PF && kt + 1 < NK && kt + 1 != 8, y_a + rf2_yblk(kt) * RF_KBS * 4, b, acc,
               apre, y_a + rf2_yblk(kt + 1 < NK ? kt + 1 : kt) * RF_KBS * 4);
  }
  __builtin_amdgcn_s_setprio(0);
  asm volatile("" ::"v"(xpf0), "v"(xpf1));  // (retired by GEMM2's last wait)
  rf2_signal(ctr + RF2_CG2 + half, lane);  // this wave's reads of the Y image are done
  if (prof) {
    asm volatile("" ::"v"(acc[6][3][3]));
    pst[4] = eg_stamp();
  }
  // ---- epilogue: BN-folded bias + activation, ROI column sums (rf_body's)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f2v b01 = {bias4[t].x, bias4[t].y}, b23 = {bias4[t].z, bias4[t].w};
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2v v = f2v{acc[i][t][2 * h], acc[i][t][2 * h + 1]} + (h ? b23 : b01);
        v = G == 1 ? hswish2(v) : silu2(v);
        acc[i][t][2 * h] = v.x;
        acc[i][t][2 * h + 1] = v.y;
      }
  }
  {
    // every lane converts and stores one channel's squeeze mean (the butterfly leaves all 16
    // sums of a row group in every lane of it)
    const float x = rf_colsum(acc, fr);
    (G == 0 ? a.m_r : a.m_n)[roi * 512 + rf_lane_ch(wave, fr, fc)] = rf_mean(x);
  }
  if (prof) pst[5] = eg_stamp();
  // ---- output staging: A over blocks 0..7 (X, dead once B is past GEMM1), B over Y(A)
  // (dead once both halves are past GEMM2); 16-B chunk c of row r at slot c ^ (r & 15)
  if (half == 0) {
    rf2_wait(ctr + RF2_CG1 + 1, t4);
  } else {
    rf2_wait(ctr + RF2_CG2 + 0, t4);
    rf2_wait(ctr + RF2_CG2 + 1, t4);
  }
  uint32_t* stg = Y + (half ? 16 * RF_KBS : 0);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int px = i * 16 + fr;
    if (px < RF_S) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4v v = acc[i][t];
        const int ch = hw * 64 + t * 16 + fc * 4;  // channel within the half
        *reinterpret_cast<uint2*>(stg + px * RF2_SROW + (((ch >> 3) ^ (px & 15)) << 2) + ((ch & 7) >> 1)) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  }
  rf2_signal(ctr + RF2_CST + half, lane);
  rf2_wait(ctr + RF2_CST + half, t4);
  if (prof) pst[6] = eg_stamp();
  {
    // XRN rows through a buffer store with sc1: the line leaves the XCD's L2 with the write
    // (plain stores kept ~2.8 MB of XRN per ROI round in the 4 MB L2, evicting the weight
    // fragments the 28 workgroups re-read every ROI: front FETCH 413 vs 634 MB per launch)
    const uint64_t da = (uint64_t)(a.XRN + r0 * 1024 + G * 512 + half * 256);
    const uint32_t da_lo = __builtin_amdgcn_readfirstlane((uint32_t)da);
    const uint32_t da_hi = __builtin_amdgcn_readfirstlane((uint32_t)(da >> 32));
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)da_hi << 32) | da_lo), 0, RF_S * 2048, 0x00020000);
    const int ht = tid & 255;
#pragma unroll
    for (int j = 0; j < (RF_S * 32 + 255) / 256; ++j) {
      const int q = ht + 256 * j;
      if (q >= RF_S * 32) break;
      const int row = q >> 5, c = q & 31;
      const u32x4 v = *reinterpret_cast<const u32x4*>(stg + row * RF2_SROW + ((c ^ (row & 15)) << 2));
      __builtin_amdgcn_raw_buffer_store_b128(v, drs, (row * 1024 + c * 8) * 2, 0, 16 /* sc1 */);
    }
  }
  rf2_signal(ctr + RF2_CSD + half, lane);  // this wave's staging reads are done (the next ROI may write)
  // the ROI's progress count (the launch's `progress` argument): one relaxed device-scope add per ROI, so a
  // trk_stream_gate on another stream can start its work while this front is in its last round
  if (G == 0 && threadIdx.x == 0 && a.progress)
    __hip_atomic_fetch_add(a.progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pst[7] = eg_stamp();
    if (lane == 0) {  // every wave's phases: [workgroup][wave][8]
      unsigned long long* o = a.prof + ((roi * 2 + G) * 8 + wave) * 8;  // [ROI][group][wave]: 7 phases, start
      for (int q = 0; q < 7; ++q) o[q] = pst[q + 1] - pst[q];
      // the ROI's start on the 100 MHz clock every CU shares (s_memtime counters are not
      // comparable across CUs), with the XCD's id in bits 56..59: pair lag and placement
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
      o[7] = rt0 | ((unsigned long long)xcc << 56);
    }
  }
  }  // ROI loop
}

// The grid is C generations of 16 P workgroups (P pairs per XCD).  Workgroup w of generation c
// sits on XCD w % 8 (the dispatcher's round robin; for speed only, nothing depends on it), runs
// group G = (w / 8) & 1 and the ROIs xcd + 8 (p + P k), p = (w % 16 P) / 16, for k in chunk c of
// the pair's k range -- both groups of a ROI on one XCD, every ROI once.  C = 1: one persistent
// generation; C > 1: workgroups retire between chunks, so kernels of other streams (the tracker's,
// at a higher priority) are dispatched there instead of waiting for the whole launch
template <bool PF>
__global__ void __launch_bounds__(512, 1) rmb_front3_kernel(RfArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t per = 16 * (int64_t)a.pairs;
  const int64_t c = blockIdx.x / per;
  const int w = (int)(blockIdx.x % per), xcd = w & 7, slot = w >> 3;
  const int64_t P = a.pairs;
  const int64_t stride = 8 * P;
  // k range of the pair: ROIs xcd + 8 (p + P k) < R
  const int64_t p = slot >> 1;
  const int64_t nk = (a.R - xcd - 8 * p + stride - 1) / stride;  // ROIs of this pair (0 if none)
  const int64_t kc = (nk + a.chunks - 1) / a.chunks;
  const int64_t k0 = c * kc, k1 = min(nk, k0 + kc);
  if (k0 >= k1) return;
  const int64_t roi0 = xcd + 8 * p + stride * k0, roi_end = xcd + 8 * p + stride * (k1 - 1) + 1;
  if (slot & 1) rf2_body<1, PF>(a, smem, roi0, stride, roi_end);
  else rf2_body<0, PF>(a, smem, roi0, stride, roi_end);
}


// ---------------------------------------------------------------------------
// trans4 (trk_set_tuning("enc_trans", 1)): the transition (K = 1024, x_f = the first 512
// columns scaled by s) on gemm4's 128 x 256 tiles, with the weights read straight into
// VGPRs instead of through LDS.  4 waves as 1 (M) x 4 (N): wave w owns 64 output
// columns for all 128 rows (8 x 4 MFMA 16x16x32 tiles), so no weight element is used by
// two waves of the workgroup and the pre-packed fragments (ops.enc_pack_fragments_k: [k
// step][16-col tile][lane] x 16 B) arrive as one contiguous 4 KiB per wave and K step,
// two steps ahead (asm loads, counted vmcnt, rmb_front's rf_loadB).  LDS carries only the
// activation rows: an 8 KiB stage per K step (3-stage LDS-DMA ring, swizzle and SE scaling
// as gemm4) + the s tile, 32 KiB per workgroup; per K step and CU that is 16 KB of DMA and
// 64 KB of fragment reads against gemm4's 48 + 96.  MFMA operands, K order and the per-
// 64-row-block sums are gemm4's, so T and the ROI sums are bit-identical to it.
constexpr int T4_NK = 32;                       // K = 1024
constexpr int T4_BUF = 512;                     // uint4 per K step: 128 rows x 64 B
// SPS K steps per LDS stage (one barrier per stage), 3 stages: stage j + 2 is issued at the
// start of stage j; B fragments BD steps ahead in BD + 1 register sets.  Issue order:
// A stage 0, B(0), A stage 1, B(1) .. B(BD - 1); step kt: B(kt + BD), then (first step of
// a stage) the A stage two ahead.  t4_vm(kt) = ops issued after the youngest op the end
// of step kt needs (B(kt + 1); at a stage end also the next A stage): its vmcnt.
template <int SPS, int BD>
constexpr int t4_vm(int kt) {
  constexpr int NS = T4_NK / SPS;
  int bend[T4_NK] = {}, aend[T4_NK] = {};
  int pos = 2 * SPS;
  aend[0] = pos;
  pos += 4;
  bend[0] = pos;
  pos += 2 * SPS;
  aend[1] = pos;
  pos += 4;
  bend[1] = pos;
  for (int b = 2; b < BD; ++b) bend[b] = (pos += 4);
  if (kt < 0) return pos - (aend[0] > bend[0] ? aend[0] : bend[0]);
  for (int k = 0; k <= kt; ++k) {
    if (k + BD < T4_NK) bend[k + BD] = (pos += 4);
    if (k % SPS == 0 && k / SPS + 2 < NS) aend[k / SPS + 2] = (pos += 2 * SPS);
  }
  int need = kt + 1 < T4_NK ? bend[kt + 1] : pos;
  if ((kt + 1) % SPS == 0 && kt + 1 < T4_NK && aend[(kt + 1) / SPS] > need) need = aend[(kt + 1) / SPS];
  return pos - need;
}
template <int SPS, int BD>
constexpr bool t4_vm_ok() {
  for (int kt = -1; kt < T4_NK; ++kt)
    if (t4_vm<SPS, BD>(kt) < 0 || t4_vm<SPS, BD>(kt) > 24) return false;
  return true;
}
static_assert(t4_vm<1, 2>(-1) == 6 && t4_vm<1, 2>(0) == 6 && t4_vm<1, 2>(T4_NK - 2) == 0, "trans4 vmcnt: gemm4 order");

// f(integral_constant<int, k>) for k = 0, 1, ...: a loop whose index is a constant expression
template <typename F, int... K>
__device__ __forceinline__ void seq_for(F&& f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, K>{}), ...);
}

// The step's B loads and A DMA are issued between its MFMAs (after row tiles 1 and 3), not
// after them (235.4 vs 244.1 us isolated; measured and dropped: s_setprio(1) over the MFMAs,
// 248.7; the A fragments read by asm with counted waits per row tile, a tie)
template <int SPS, int BD>
__global__ void __launch_bounds__(256, 2) trans4_kernel(EncGemmArgs a, const uint4* Wtp, int64_t ntiles) {
  static_assert(t4_vm_ok<SPS, BD>(), "trans4 vmcnt out of the rf_vmwait range");
  constexpr int NS = T4_NK / SPS, NSLOT = 3 * SPS;
  constexpr size_t RING = (size_t)NSLOT * T4_BUF * 16;
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t lb = xcd_remap(blockIdx.x, ntiles);
  uint4* ring = reinterpret_cast<uint4*>(smem);
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntile_n = a.N / 256;
  const int n0 = (int)(lb % ntile_n) * 256;
  const int64_t m0 = lb / ntile_n * 128;
  const int64_t roi_base = m0 / a.P;
  const int fr = lane & 15, fc = lane >> 4;

  const uint16_t* asrc[2];
  int arow[2], achk[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    arow[q] = r;
    achk[q] = c;
    asrc[q] = a.A + min(m0 + r, (int64_t)a.M - 1) * a.lda + c * 8;
  }
  const uint4* bp = Wtp + (size_t)(n0 / 16 + wave * 4) * 64 + lane;
  u32x4 bq[BD + 1][4];
  auto issueA = [&](int st) {  // the SPS K steps of stage st
#pragma unroll
    for (int u = 0; u < SPS; ++u) {
      const int kt = st * SPS + u;
      uint4* d = ring + (kt % NSLOT) * T4_BUF + wave * 64;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * 256), 16, 0, 0);
    }
  };
  auto loadB = [&](int kt) { rf_loadB(bp, kt, bq[kt % (BD + 1)]); };

  // the s tile (the slots a 128-row tile spans) behind the ring, as gemm4
  float* stile = reinterpret_cast<float*>(smem + RING);
  const float* srow[2];
  {
    const int per = 512 / 4;
    const int64_t nroi = ((int64_t)a.M + a.P - 1) / a.P;
    const int tslots = min(G4_SLOTS, (127 + a.P - 1) / a.P + 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = q * 256 + tid;
      if (p >= tslots * per) continue;
      const int slot = min(p / per, G4_SLOTS - 1);
      const int64_t roi = min(roi_base + slot, nroi - 1);
      __builtin_amdgcn_global_load_lds(GPTR(a.scale + roi * 512 + (p % per) * 4),
                                       LPTR(reinterpret_cast<uint4*>(stile) + q * 256 + wave * 64), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t row = min(m0 + arow[q], (int64_t)a.M - 1);
      srow[q] = stile + (int)(row / a.P - roi_base) * 512 + achk[q] * 8;
    }
  }
  // bf16(x * s) in place on this thread's own two DMA'd chunks of K step kt (x_f steps)
  auto transform = [&](int kt) {
    const uint32_t d = lds_addr(ring + (kt % NSLOT) * T4_BUF + tid);
    u32x4 v[2], s4[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      v[q] = lds_read128(d + q * 256 * 16);
      const uint32_t sa = lds_addr(srow[q] + kt * BK);
      s4[q][0] = lds_read128(sa);
      s4[q][1] = lds_read128(sa + 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(s4[0][0]), "+v"(s4[0][1]), "+v"(s4[1][0]),
                 "+v"(s4[1][1])::"memory");
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
  };
  auto transform_stage = [&](int st) {
#pragma unroll
    for (int u = 0; u < SPS; ++u)
      if ((st * SPS + u) * BK < 512) transform(st * SPS + u);
  };

  const int lterm = fr * 4 + (fc ^ x16(fr));
  f4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};

  unsigned long long pst[8];
  const bool prof = a.prof != nullptr;
  if (prof) pst[0] = eg_stamp();
  issueA(0);
  loadB(0);
  issueA(1);
  loadB(1);
#pragma unroll
  for (int b = 2; b < BD; ++b) loadB(b);
  rf_vmwait(t4_vm<SPS, BD>(-1), bq[0]);  // A stage 0 (own chunks) and B(0); the s tile is older
  g4_barrier();                           // every wave's s-tile DMA landed
  transform_stage(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g4_barrier();
  // the K steps as a compile-time sequence (the counted waits, ring slots and register
  // sets must be immediates; #pragma unroll gave up on the deeper variants)
  auto step = [&](auto ktc) {
    constexpr int kt = decltype(ktc)::value;
    const uint4* buf = ring + (kt % NSLOT) * T4_BUF;
    bf8v afr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) afr[i] = *reinterpret_cast<const bf8v*>(buf + lterm + i * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], __builtin_bit_cast(bf8v, bq[kt % (BD + 1)][t]),
                                                            acc[i][t], 0, 0, 0);
      if (i == 1) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kt + BD < T4_NK) loadB(kt + BD);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (i == 3) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kt % SPS == 0 && kt / SPS + 2 < NS) issueA(kt / SPS + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kt + 1 < T4_NK) {
      rf_vmwait(t4_vm<SPS, BD>(kt), bq[(kt + 1) % (BD + 1)]);
      if constexpr ((kt + 1) % SPS == 0) {
        transform_stage((kt + 1) / SPS);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        g4_barrier();
      }
    }
  };
  seq_for(step, std::make_integer_sequence<int, T4_NK>{});
  if (prof) pst[1] = eg_stamp();

  // ---- SiLU(T + bias), then gemm4's MFMA ROI sums per 64-row half (rows 64 h ..)
  const int colq = wave * 64 + fr;  // + t * 16 (column within the tile)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float bv = a.bias[n0 + colq + t * 16];
    const f2v b2 = {bv, bv};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f2v v = f2v{acc[i][t][2 * hh], acc[i][t][2 * hh + 1]} + b2;
        v = silu2(v);
        acc[i][t][2 * hh] = v.x;
        acc[i][t][2 * hh + 1] = v.y;
      }
  }
  if (prof) pst[2] = eg_stamp();
  float* part = reinterpret_cast<float*>(smem);  // [2 halves][SLOTS][256] (the ring is idle)
  {
    const int P = a.P;
    const int off = (int)(m0 - roi_base * P);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf8v mask[2];
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rl = h * 64 + (2 * p2 + (j >> 2)) * 16 + 4 * fc + (j & 3);
          const int x = off + rl;
          const int slot = (x >= P) + (x >= 2 * P) + (x >= 3 * P);
          mask[p2][j] = (slot == fr && m0 + rl < (int64_t)a.M) ? (__bf16)1.0f : (__bf16)0.0f;
        }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f4v sacc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
          const f4v u = acc[4 * h + 2 * p2][t], v = acc[4 * h + 2 * p2 + 1][t];
          bf8v hi, lo;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hi[e] = (__bf16)u[e];
            hi[4 + e] = (__bf16)v[e];
            lo[e] = (__bf16)(u[e] - (float)hi[e]);
            lo[4 + e] = (__bf16)(v[e] - (float)hi[4 + e]);
          }
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mask[p2], hi, sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mask[p2], lo, sacc, 0, 0, 0);
        }
        if (lane < 16) {
#pragma unroll
          for (int ts = 0; ts < G4_SLOTS; ++ts) part[(h * G4_SLOTS + ts) * 256 + colq + t * 16] = sacc[ts];
        }
      }
    }
  }
  if (prof) pst[3] = eg_stamp();
  __syncthreads();
  {
    const int64_t last_row = min(m0 + 128, (int64_t)a.M) - 1;
    const int nslot = (int)(last_row / a.P - roi_base) + 1;
    for (int q = tid; q < nslot * 256; q += 256) {
      const int slot = q >> 8, c = q & 255;
      const int64_t roi = roi_base + slot;
      const int j = (int)(m0 / kPartRows - roi * a.P / kPartRows);
      a.sums[(roi * kPart + j) * a.ld_sums + n0 + c] =
          llrintf(part[slot * 256 + c] * kFix) + llrintf(part[(G4_SLOTS + slot) * 256 + c] * kFix);
    }
  }
  if (prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pst[4] = eg_stamp();
    if (tid == 0) {
      unsigned long long* o = a.prof + lb * 8;
      for (int q = 0; q < 4; ++q) o[q] = pst[q + 1] - pst[q];
      o[4] = pst[4] - pst[0];
      o[5] = o[6] = o[7] = 0;
    }
  }
}

template <int EPI>
int launch4(const EncGemmArgs& a, hipStream_t st) {
  const int64_t nwg = ((int64_t)a.M + 127) / 128 * (a.N / 256) * a.groups;
  TRK_REQUIRE(nwg < 0x7fffffff, "enc_gemm4: too many workgroups");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm4_kernel<EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G4_LDS);
    attr = true;
  }
  EncGemmArgs b = a;
  b.prof = g_enc_prof.get();
  // dynamic LDS: what the tile uses, not the 80 KiB maximum, so the tracker's and ROI
  // Align's workgroups fit beside two gemm4 workgroups on a CU instead of waiting for one
  // to retire (DSC: ring or staging + partials, 74 KiB; transition: ring + the SE scales
  // of the slots a 128-row tile can span, 78 KiB at P = 100)
  const int tslots = std::min(G4_SLOTS, (127 + a.P - 1) / a.P + 1);
  const size_t lds = EPI == EPI_DSC ? std::max(G4_RING, G4_STAGE + G4_RED)
                                    : std::max(G4_RING + (size_t)tslots * a.kscale * 4, (size_t)G4_RED);
  hipLaunchKernelGGL((gemm4_kernel<EPI>), dim3((unsigned)nwg), dim3(256), lds, st, b, nwg);
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

extern "C" int trk_enc_dsc_gemm(const void* Y2, int64_t M, int64_t P, int64_t Kg, const void* W2,
                                const float* bias, int64_t Ng, void* XRN, long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 43 && P <= 256 && Kg % BK == 0 && Kg > 0 && Ng % 256 == 0 && Ng > 0,
              "enc_dsc_gemm: need 43 <= P <= 256, K %% 32 == 0, N %% 256 == 0");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(Y2 && W2 && bias && XRN && sums && aligned16(Y2) && aligned16(W2) && aligned16(XRN),
              "enc_dsc_gemm: null or unaligned pointer");
  EncGemmArgs a{};
  a.A = (const uint16_t*)Y2; a.lda = 2 * Kg;
  a.B = (const uint16_t*)W2; a.bias = bias;
  a.C = (uint16_t*)XRN; a.ldc = 2 * Ng;
  a.sums = sums; a.ld_sums = (int)(2 * Ng);
  a.M = (int)M; a.N = (int)Ng; a.K = (int)Kg; a.P = (int)P; a.groups = 2; a.kscale = 0;
  return launch4<EPI_DSC>(a, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int trk_enc_transition_gemm(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s,
                                       int64_t kscale, const void* Wt, const float* bias, int64_t N,
                                       long long* sums, void* stream) {
  return trk_enc_transition_gemm2(XRN, M, P, K, s, kscale, Wt, nullptr, bias, N, sums, stream);
}

extern "C" int trk_enc_transition_gemm2(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s,
                                        int64_t kscale, const void* Wt, const void* Wtp, const float* bias,
                                        int64_t N, long long* sums, void* stream) {
  TRK_REQUIRE(M >= 0 && P >= 43 && P <= 256 && K % BK == 0 && K > 0 && N % 256 == 0 && N > 0 &&
                  kscale % BK == 0 && kscale <= K && kscale * G4_SLOTS <= G4_SQ * 256 * 4,
              "enc_transition_gemm: need 43 <= P <= 256, K %% 32 == 0, N %% 256 == 0, kscale %% 32 == 0, "
              "kscale <= 512");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(XRN && s && Wt && bias && sums && aligned16(XRN) && aligned16(Wt) && aligned16(s),
              "enc_transition_gemm: null or unaligned pointer");
  // the packed fragments (ops.enc_pack_fragments_k of Wt [N][K]) are trans4's operand image
  // for exactly K = 1024, N = 512 (rf_loadB steps one K step as 32 column tiles)
  TRK_REQUIRE(!Wtp || (K == 1024 && N == 512 && kscale == 512 && aligned16(Wtp)),
              "enc_transition_gemm: packed Wt needs K = 1024, N = 512, kscale = 512 (16-byte aligned)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EncGemmArgs a{};
  a.A = (const uint16_t*)XRN; a.lda = K;
  a.B = (const uint16_t*)Wt; a.bias = bias;
  a.sums = sums; a.ld_sums = (int)N;
  a.scale = s;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.P = (int)P; a.groups = 1; a.kscale = (int)kscale;
  if (g_enc_trans == 1 && Wtp) {
    const int64_t nwg = ((int64_t)M + 127) / 128 * (N / 256);
    TRK_REQUIRE(nwg < 0x7fffffff, "enc_transition_gemm: too many workgroups");
    a.prof = g_enc_prof.get();
    const size_t slds = (size_t)G4_SLOTS * 512 * 4;
    hipLaunchKernelGGL((trans4_kernel<1, 2>), dim3((unsigned)nwg), dim3(256), 3 * T4_BUF * 16 + slds, st, a,
                       reinterpret_cast<const uint4*>(Wtp), nwg);
    return trk::check_launch("trans4_kernel");
  }
  return launch4<EPI_TRANS>(a, st);
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
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1dw4_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G1Q_LDS);
    attr = true;
  }
  hipLaunchKernelGGL(g1dw4_kernel, dim3((unsigned)nwg), dim3(256), G1Q_LDS, reinterpret_cast<hipStream_t>(stream),
                     (const uint16_t*)X, (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N);
  return trk::check_launch("g1dw4_kernel");
}

extern "C" int trk_enc_rmb_front_means(const void* X, int64_t M, const void* W1p, const float* wdw, const void* W2p,
                                       const float* bias, void* XRN, float* m_r, float* m_n, uint32_t* progress,
                                       void* stream) {
  TRK_REQUIRE(M >= 0 && M % RF_S == 0, "enc_rmb_front_means: 10x10 ROIs (M %% 100 == 0), C = 512, 4h = 1024");
  if (M == 0) return TRK_OK;
  TRK_REQUIRE(X && W1p && wdw && W2p && bias && XRN && m_r && m_n && aligned16(X) && aligned16(W1p) &&
                  aligned16(W2p) && aligned16(XRN) && aligned16(wdw) && aligned16(m_r) && aligned16(m_n),
              "enc_rmb_front_means: null or unaligned pointer");
  TRK_REQUIRE(M / RF_S < 0x7fffffff, "enc_rmb_front_means: too many ROIs");
  // the CU count of the device the launch goes to (queried per call: a process may drive several)
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 16) ncu = 16;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(rmb_front3_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)RF2_LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(rmb_front3_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)RF2_LDS);
    attr = true;
  }
  RfArgs a;
  memset(&a, 0, sizeof a);
  a.X = (const uint16_t*)X;
  a.W1p = (const uint4*)W1p;
  a.wdw = wdw;
  a.W2p = (const uint4*)W2p;
  a.bias = bias;
  a.XRN = (uint16_t*)XRN;
  a.m_r = m_r;
  a.m_n = m_n;
  a.R = M / RF_S;
  a.prof = g_enc_prof.get();
  a.progress = progress;
  // persistent: 16 workgroups per 8 ROIs up to one per CU (a multiple of 16, so both groups of a
  // ROI share an XCD); rf3_groups 0 = two CUs per XCD left free -- the tracker's and the ROI
  // stream's kernels start there instead of waiting for a persistent workgroup to end
  // (2.03-2.05 vs 1.96-1.98M ROIs/s over four interleaved pairs against one ROI per workgroup)
  const int64_t groups =
      std::min<int64_t>((a.R + 7) / 8, g_rf3_groups > 0 ? g_rf3_groups : std::max(1, ncu / 16 - 2));
  // chunks: no more than the ROIs a pair has (an empty generation would only launch and exit)
  const int64_t per_pair = ((a.R + 7) / 8 + groups - 1) / groups;
  const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(g_rf3_chunks, per_pair));
  a.pairs = (int)groups;
  a.chunks = (int)chunks;
  if (g_rf_pf)
    hipLaunchKernelGGL(rmb_front3_kernel<true>, dim3((unsigned)(16 * groups * chunks)), dim3(512), RF2_LDS,
                       reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(rmb_front3_kernel<false>, dim3((unsigned)(16 * groups * chunks)), dim3(512), RF2_LDS,
                       reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("rmb_front3_kernel");
}

// diagnostics: gemm4 per-workgroup phase stamps (8 u64 per workgroup); nullptr
// switches them off
extern "C" int trk_enc_set_prof(unsigned long long* buf) {
  g_enc_prof.set(buf);
  return TRK_OK;
}

namespace {
// one wave: wait until the wrapping count *counter has reached target ((int32_t)(v - target) >= 0,
// so a target within 2^31 of the count is ordered correctly across the wrap; relaxed device-scope
// loads, s_sleep between polls) or
// until max_ticks of the 100 MHz clock have passed, then end: the kernels queued behind it on
// its stream start then.  A performance gate only: it never blocks longer than its bound
__global__ void __launch_bounds__(64) stream_gate_kernel(const uint32_t* counter, uint32_t target,
                                                         unsigned long long max_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int32_t)(__builtin_amdgcn_readfirstlane(v) - target) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(16);
  }
}
}  // namespace

extern "C" int trk_stream_gate(const uint32_t* counter, uint32_t target, int64_t max_us, void* stream) {
  TRK_REQUIRE(counter && max_us >= 0 && max_us <= 1000000, "stream_gate: null counter or max_us outside 0..1e6");
  hipLaunchKernelGGL(stream_gate_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), counter,
                     target, (unsigned long long)max_us * 100);
  return trk::check_launch("stream_gate_kernel");
}
