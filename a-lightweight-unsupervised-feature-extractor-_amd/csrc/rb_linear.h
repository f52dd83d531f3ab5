// Small f32 GEMMs of 16-ROI row tiles on v_mfma_f32_16x16x4_f32, shared by the encoder
// tail kernels (enc_head.hip: enc_se, enc_head) and the persistent front's batched SE
// (enc_gemm.hip: rmb_front3 with the SE folded in) -- one definition, so both produce
// the same bits for the same rows.
//
// The 16 ROI rows are the A operand (from LDS), each wave owns column tiles of 16 outputs
// whose weight rows it streams from L2, pre-packed on the host in fragment order
// (ops.enc_pack_rows: [N/16][K/16][64 lanes][4], lane = 16 g + r holding W[16 t + r][16 kb + 4 g
// .. + 3]), so each load instruction reads 1 KiB contiguous instead of 16 rows' 64-B pieces
// (enc_head 37.1 vs 46.9 us, enc_se 22.3 vs 26.2 us; the same values in the same order).  Within each 16-wide K block, lane group
// g = lane >> 4 takes k = 4g + t at MFMA t (t = 0..3) for BOTH operands, so every lane
// reads 16 contiguous bytes of its A row and of its weight row (the sum's order is
// permuted, not its terms).
#pragma once
#include "trk_common.h"

namespace {

typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int RB = 16;        // ROIs per workgroup
constexpr int MAXC = 1024;    // channel bound (LDS sizing)

// LDS rows of the 16-ROI tiles: ld = C rounded up to 64 floats (a row is a whole number
// of 256-B bank rows) and 16-B chunk q of row r at chunk q ^ (r & 15) (within its aligned
// group of 16 chunks).  The MFMA A reads (lane (r, g) takes chunk kb / 4 + g of row r,
// served in the lane groups of MI355X_MICROARCH.md §LDS) and the callbacks' row writes
// then hit 16 distinct chunks per group: the padded rows (ld = C + 4) were 2-way
// (SQ_LDS_BANK_CONFLICT 3.4 cycles per LDS instruction in enc_se, 2.0 in enc_head)
__host__ __device__ inline int ld_rows(int c) { return (c + 63) & ~63; }
__device__ __forceinline__ int swz_at(int row, int col, int ld) {
  return row * ld + (((col >> 2) ^ (row & 15)) << 2) + (col & 3);
}

// acc[t] (t < NT) += X[16][K] . W[n0 + 16 t .. + 15][K]^T.  K is walked in
// chunks of U blocks of 16; chunk c + 1's weight and activation loads (NT x U + U
// 16-B loads per lane, into the other register buffer) are issued before chunk c's
// MFMAs, so each L2 round trip runs under the previous chunk's MFMAs instead of
// between them.  NT and U are compile-time so loads / MFMAs are straight-line code.
template <int NT, int U>
struct RbBuf {
  float4 a[U], b[U][NT];
};

template <int NT, int U>
__device__ __forceinline__ void rb_load(const float* xp, int xq, const float* const (&wp)[NT], int kb0,
                                        RbBuf<NT, U>& d) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      d.b[u][t] = *reinterpret_cast<const float4*>(wp[t] + (kb0 / 16 + u) * 256);
  // A: chunk (kb / 4 + g) ^ (r & 15) of row r = the chunk group kb / 64 plus ((kb / 4) & 15) ^ xq
  // (kb / 4 is a multiple of 4 and g < 4, so kb / 4 + g = kb / 4 ^ g; xq = g ^ (r & 15))
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = (kb0 + 16 * u) >> 2;
    d.a[u] = *reinterpret_cast<const float4*>(xp + (((q & ~15) | ((q & 15) ^ xq)) << 2));
  }
}

template <int NT, int U>
__device__ __forceinline__ void rb_mfma(const RbBuf<NT, U>& d, f4_t (&acc)[NT]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(d.a[u].x, d.b[u][t].x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(d.a[u].y, d.b[u][t].y, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(d.a[u].z, d.b[u][t].z, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(d.a[u].w, d.b[u][t].w, acc[t], 0, 0, 0);
    }
}

template <int NT, int U>
__device__ __forceinline__ void rb_gemm(const float* __restrict__ Xs, int ldx, const float* __restrict__ W,
                                        int64_t ldw, int n0, int K, f4_t (&acc)[NT]) {
  constexpr int KC = 16 * U;
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const float* wp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    wp[t] = W + ((int64_t)(n0 / 16 + t) * (ldw / 16) * 64 + lane) * 4;
  const float* xp = Xs + r * ldx;  // swizzled row (swz_at)
  const int xq = g ^ (r & 15);
  const int nch = K / KC;
  if (nch > 0) {
    RbBuf<NT, U> b0, b1;
    rb_load<NT, U>(xp, xq, wp, 0, b0);
    int c = 0;
    for (;;) {
      if (c + 1 < nch) rb_load<NT, U>(xp, xq, wp, (c + 1) * KC, b1);
      __builtin_amdgcn_sched_barrier(0);
      rb_mfma<NT, U>(b0, acc);
      if (++c == nch) break;
      if (c + 1 < nch) rb_load<NT, U>(xp, xq, wp, (c + 1) * KC, b0);
      __builtin_amdgcn_sched_barrier(0);
      rb_mfma<NT, U>(b1, acc);
      if (++c == nch) break;
    }
  }
  for (int kb = nch * KC; kb < K; kb += 16) {
    RbBuf<NT, 1> t1;
    rb_load<NT, 1>(xp, xq, wp, kb, t1);
    rb_mfma<NT, 1>(t1, acc);
  }
}

// Y[16][N] = epi(col, X[16][K] . W[N][K]^T + bias) -> per-element store
// callback, column tiles of 16 spread over the 8 waves (runs of 4, then singles).
template <int NT, int U, class Store>
__device__ __forceinline__ void rb_tiles(const float* Xs, int ldx, const float* W, const float* bias, int K,
                                         int t0, Store store) {
  const int lane = threadIdx.x & 63;
  f4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_t{0.f, 0.f, 0.f, 0.f};
  rb_gemm<NT, U>(Xs, ldx, W, K, t0 * 16, K, acc);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = (t0 + t) * 16 + (lane & 15);
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) store(4 * (lane >> 4) + i, col, acc[t][i] + bv);
  }
}

// column tiles spread over the NW waves: runs of 4 (8-wave workgroups) or 2 (16-wave
// workgroups, 128 VGPRs), then singles; U = K blocks per double-buffered chunk
template <int NW, class Store>
__device__ __forceinline__ void rb_linear(const float* Xs, int ldx, const float* W, const float* bias, int N,
                                          int K, Store store) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntile = N / 16;
  const int per = (ntile + NW - 1) / NW;
  const int t_begin = wave * per, t_end = min(ntile, t_begin + per);
  int t0 = t_begin;
  if constexpr (NW <= 8) {
    for (; t0 + 4 <= t_end; t0 += 4) rb_tiles<4, 4>(Xs, ldx, W, bias, K, t0, store);
    for (; t0 < t_end; ++t0) rb_tiles<1, 8>(Xs, ldx, W, bias, K, t0, store);
  } else {
    for (; t0 + 2 <= t_end; t0 += 2) rb_tiles<2, 2>(Xs, ldx, W, bias, K, t0, store);
    for (; t0 < t_end; ++t0) rb_tiles<1, 4>(Xs, ldx, W, bias, K, t0, store);
  }
}

}  // namespace
