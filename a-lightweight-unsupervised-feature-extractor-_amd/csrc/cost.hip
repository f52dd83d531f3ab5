// Fused association-cost kernel for gfx950 (MI355X), batched over frames.
//
// One launch replaces, per frame (video stream):
//   Tracking.build_C_app_topk      reference model/mainTracking.py:141-211
//   costCard.bbox_cost / conf_cost model/utils/costTool/costCard.py:109-203
//   costCard.cal_cost C_total      costCard.py:264-268
//   Tracking.apply_kalman_gating   mainTracking.py:306-338 +
//   gating_distance_maha           model/utils/costTool/KalmanFilter.py:105-116
// Restated in SURVEY.md A.3/A.4 and oracle/trk_oracle.c:ora_cost_build.
//
// Work decomposition:
//   workgroup = (frame f, 32-detection tile, block of 16 track rows); 4 waves,
//   each wave owns 4 track rows.  The 32x128 detection tile is normalised once
//   and held in registers as the B operand of v_mfma_f32_32x32x2_f32 (exact
//   f32, 64 k-steps; lane half h supplies k = s + 64h).  Per track the <=30x128
//   memory bank is read straight into the A operand (16-B loads, L1-resident),
//   the next track's bank is prefetched during the MFMA chain.  The 32x32
//   accumulator holds sim[t][j] with the column on the lane, so the per-column
//   top-k over t is a register sort of 16 values per lane + one __shfl_xor(32)
//   merge.  bbox / conf / Mahalanobis terms are fused into the epilogue.
// Built with -ffp-contract=off: scalar f32 ops round as torch's separate ops do;
// the one FMA torch's CPU norm performs is written as an explicit fmaf.
#include "trk_common.h"

int g_cost_v2 = 0;  // trk_set_tuning("cost_v2"): 1 = bank-resident cost2_kernel on trk_build_cost (Nmax <= 272;
                    // its 147 KiB LDS workgroups stall behind the encoder in the pipeline: 1.23M vs 1.51M ROIs/s),
                    // and cost_kernel instead of cost3 on trk_build_cost_dev (A/B); 0 = default

trk::DiagBuf g_cost_prof;  // trk_cost_set_prof (diagnostics)
int g_cost_split = 1;  // trk_set_tuning("cost_split"): 1 (default) = cost3's similarities from f16 hi / lo splits on
                       // the f16 MFMA (3 products, within 1.1e-6 of exact f32); 0 = exact f32 MFMA
                       // (bit-identical to cost_kernel)

namespace {

constexpr int D = 128;           // embedding dim (mainTracking.py:109-110,267-268)
constexpr int kMaxFrames = 64;   // frames per launch (kernarg-resident shapes)
constexpr int kMaxTopk = 8;
constexpr int kRowsPerWave = 4;
constexpr int kWavesPerWG = 4;
constexpr int kRowsPerWG = kRowsPerWave * kWavesPerWG;
constexpr int kCost3Rows = 256;  // cost3 rows per frame in one pass of its grid (one wave each)

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct CostArgs {
  int F, Mmax, Nmax, Tmax;
  int rs_ld;                // row_slot row stride
  const int32_t* dev_M;     // per-frame sizes in device memory (trk_build_cost_dev), else M / N below
  const int32_t* dev_N;
  const int32_t* row_slot;
  const float* bank;
  const int32_t* bank_len;
  const float* pbox;
  const float* conf_prev;
  const double* gmean;
  const double* gsinv;
  const int32_t* gate_on;
  const float* det_emb;
  const float* dbox;
  const float* conf_cur;
  float* C_total;
  float* C_app;
  float* C_center;
  float* C_scale;
  float* C_conf;
  trk_cost_params p;
  int M[kMaxFrames];
  int N[kMaxFrames];
};

__device__ __forceinline__ void load_a_frag(const float* __restrict__ rowp, bool ok, float (&a)[64]) {
  // lane (t, h): elements 64h + 0..63 of bank row t (16 x 16-B loads)
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    float4 v = ok ? *reinterpret_cast<const float4*>(rowp + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    a[4 * q + 0] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
  }
}

// insert x into a descending list of length K (K <= kMaxTopk, compile-time bound)
__device__ __forceinline__ void topk_insert(float (&v)[kMaxTopk], float x) {
#pragma unroll
  for (int q = 0; q < kMaxTopk; ++q) {
    float hi = fmaxf(v[q], x);
    x = fminf(v[q], x);
    v[q] = hi;
  }
}
// the same network on the first KT slots only: slot q depends on slots <= q and x,
// so the first KT slots equal topk_insert's (cost3 with topk <= 5: 10 ops instead of 16)
template <int KT>
__device__ __forceinline__ void topk_insert_k(float (&v)[kMaxTopk], float x) {
#pragma unroll
  for (int q = 0; q < KT; ++q) {
    float hi = fmaxf(v[q], x);
    x = fminf(v[q], x);
    v[q] = hi;
  }
}

// topk_insert on a list of any compile-time length
template <int K>
__device__ __forceinline__ void topk_insert_n(float (&v)[K], float x) {
#pragma unroll
  for (int q = 0; q < K; ++q) {
    float hi = fmaxf(v[q], x);
    x = fminf(v[q], x);
    v[q] = hi;
  }
}
// compare-exchange: a = max, b = min (descending order)
__device__ __forceinline__ void topk_ce(float& a, float& b) {
  const float hi = fmaxf(a, b);
  b = fminf(a, b);
  a = hi;
}
// 5-input sorting network (9 compare-exchanges), descending
__device__ __forceinline__ void sort5_desc(float (&c)[5]) {
  topk_ce(c[0], c[1]); topk_ce(c[3], c[4]); topk_ce(c[2], c[4]);
  topk_ce(c[2], c[3]); topk_ce(c[0], c[3]); topk_ce(c[0], c[2]);
  topk_ce(c[1], c[4]); topk_ce(c[1], c[3]); topk_ce(c[1], c[2]);
}
// the top 5 of the union of two descending 5-lists, descending: max(a_i, b_{4-i}) is that set
// (a bitonic sequence), then sorted
__device__ __forceinline__ void top5_merge(const float (&a)[5], const float (&b)[5], float (&o)[5]) {
#pragma unroll
  for (int i = 0; i < 5; ++i) o[i] = fmaxf(a[i], b[4 - i]);
  sort5_desc(o);
}
// the top 5 of 16 values, descending: four sorted quads, two Batcher odd-even merges (4 + 4, the
// compare-exchange that only orders slots 5 and 6 dropped), the two top-5 lists merged.  95 max /
// min against 16 insertions' 160; the same multiset in the same order as the insertion network, so
// every top-k sum is bit-identical to it (tools: a 0/1 exhaustive check of the network)
__device__ __forceinline__ void top5_of16(float (&x)[16], float (&o)[5]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float* q = x + 4 * g;
    topk_ce(q[0], q[1]); topk_ce(q[2], q[3]); topk_ce(q[0], q[2]); topk_ce(q[1], q[3]); topk_ce(q[1], q[2]);
  }
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    float* v = x + 8 * hh;
    topk_ce(v[0], v[4]); topk_ce(v[1], v[5]); topk_ce(v[2], v[6]); topk_ce(v[3], v[7]);
    topk_ce(v[2], v[4]); topk_ce(v[3], v[5]);
    topk_ce(v[1], v[2]); topk_ce(v[3], v[4]);
  }
  const float p[5] = {x[0], x[1], x[2], x[3], x[4]}, q[5] = {x[8], x[9], x[10], x[11], x[12]};
  top5_merge(p, q, o);
}

// torch's clamp(min=lo): a NaN stays NaN (fmaxf would return lo), so a NaN box or
// confidence reaches C_total and the solver raises as scipy does
__device__ __forceinline__ float clamp_lo(float x, float lo) { return x < lo ? lo : x; }

// torch.topk treats NaN as the largest value, so a NaN similarity (a NaN embedding)
// is always among the top k and makes the mean NaN; the max / min network drops
// NaNs, so the kernels carry a per-column NaN flag beside it.  nan: this lane's
// flag; the column's two lane halves (col, col + 32) are merged here.
__device__ __forceinline__ float app_nan(float app, bool nan, int col) {
  const unsigned long long b = __ballot(nan);
  return ((b >> col) & 1ull) | ((b >> (col + 32)) & 1ull) ? __builtin_nanf("") : app;
}

// costCard.bbox_cost / conf_cost / cal_cost C_total (costCard.py:141-168,
// :196-201, :264-268) + the Mahalanobis gate (mainTracking.py:327-336) for one
// (track, detection) pair.  Track-side inputs are wave-uniform.
__device__ __forceinline__ float combine(const trk_cost_params& p, float app, const float* bp,
                                         float conf_prev, float ccx, float ccy, float Ac, float ccv,
                                         bool gate, const double* gm, const double* S, double z0,
                                         double z1, double z2, double z3, float& cen, float& scl,
                                         float& cf) {
  const float px1 = bp[0], py1 = bp[1], px2 = bp[2], py2 = bp[3];
  const float cpx = 0.5f * (px1 + px2), cpy = 0.5f * (py1 + py2);
  const float wp = clamp_lo(px2 - px1, 1.0f), hp = clamp_lo(py2 - py1, 1.0f);
  const float sp = clamp_lo(sqrtf(wp * wp + hp * hp), 1.0f);
  const float Ap = wp * hp;
  const float cpv = clamp_lo(conf_prev, 1e-6f);
  const float dx = cpx - ccx, dy = cpy - ccy;
  const float dist = sqrtf(fmaf(dy, dy, dx * dx));  // torch.norm CPU rounding
  cen = dist / sp;
  scl = fabsf(logf(clamp_lo(Ac / Ap, 1e-6f)));
  cf = fabsf(logf(ccv / cpv));
  const float bbox = p.alpha * cen + p.beta * scl;
  float tot = p.w_app * app + p.w_bbox * bbox;
  tot = tot + p.w_conf * cf;
  if (gate) {
    const double y[4] = {z0 - gm[0], z1 - gm[1], z2 - gm[2], z3 - gm[3]};
    double d2 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) t += S[r * 4 + c] * y[c];
      d2 += y[r] * t;
    }
    if (d2 > p.maha_thr) tot = p.inf_cost;
  }
  return tot;
}

// detection-side terms: centre, area, clamped conf and KF measurement z
// (bbox_xyxy_to_z, KalmanFilter.py:5-16: double arithmetic, float32 result)
__device__ __forceinline__ void det_terms(const float* bc, float conf, float& ccx, float& ccy,
                                          float& Ac, float& ccv, double& z0, double& z1,
                                          double& z2, double& z3) {
  const float x1 = bc[0], y1 = bc[1], x2 = bc[2], y2 = bc[3];
  ccx = 0.5f * (x1 + x2);
  ccy = 0.5f * (y1 + y2);
  const float wc = clamp_lo(x2 - x1, 1.0f), hc = clamp_lo(y2 - y1, 1.0f);
  Ac = wc * hc;
  ccv = clamp_lo(conf, 1e-6f);
  const double dx1 = x1, dy1 = y1, dx2 = x2, dy2 = y2;
  const double w = fmax(dx2 - dx1, 1.0), hh = fmax(dy2 - dy1, 1.0);
  z0 = (float)(dx1 + 0.5 * w);
  z1 = (float)(dy1 + 0.5 * hh);
  z2 = (float)(w / hh);
  z3 = (float)hh;
}

__global__ void __launch_bounds__(256)
cost_kernel(const CostArgs A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = blockIdx.z;
  const int j0 = blockIdx.x * 32;
  const int i0 = blockIdx.y * kRowsPerWG + wave * kRowsPerWave;
  const int M = A.dev_M ? min(A.dev_M[f], A.Mmax) : A.M[f];
  const int N = A.dev_N ? min(A.dev_N[f], A.Nmax) : A.N[f];
  if (j0 >= N || blockIdx.y * kRowsPerWG >= M) return;
  const int col = lane & 31, h = lane >> 5;
  const int j = j0 + col;
  const bool jok = j < N;

  // ---- detection tile: B operand, renormalised (build_C_app_topk :167-169)
  float b[64];
  {
    const float* dp = A.det_emb + ((int64_t)f * A.Nmax + (jok ? j : 0)) * D + 64 * h;
    load_a_frag(dp, jok, b);
    double ss = 0.0;
#pragma unroll
    for (int s = 0; s < 64; ++s) ss += (double)b[s] * (double)b[s];
    ss += __shfl_xor(ss, 32);
    const float nrm = (float)sqrt(ss) + 1e-12f;
#pragma unroll
    for (int s = 0; s < 64; ++s) b[s] = b[s] / nrm;
  }
  // ---- detection-side box / conf terms for column j
  float ccx = 0.f, ccy = 0.f, Ac = 1.f, ccv = 1.f;
  double z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  if (jok)
    det_terms(A.dbox + ((int64_t)f * A.Nmax + j) * 4, A.conf_cur[(int64_t)f * A.Nmax + j], ccx, ccy,
              Ac, ccv, z0, z1, z2, z3);

  const int Tmax = A.Tmax;
  const int topk = A.p.topk;
  auto slot_of = [&](int i) -> int64_t {
    return A.row_slot ? (int64_t)A.row_slot[(int64_t)f * A.rs_ld + i] : (int64_t)f * A.Mmax + i;
  };

  float a[64];
  int iend = min(i0 + kRowsPerWave, M);
  const bool chunked = Tmax > 32;  // hist_max > 32: the bank in 32-row MFMA chunks
  if (i0 < iend && !chunked) {
    const int64_t s0 = slot_of(i0);
    const int T0 = min(A.bank_len[s0], Tmax);
    load_a_frag(A.bank + (s0 * Tmax + col) * D + 64 * h, col < T0, a);
  }
  for (int i = i0; i < iend; ++i) {
    const int64_t slot = slot_of(i);
    const int T = min(A.bank_len[slot], Tmax);
    // ---- top-k over t for column j (torch.topk(dim=0) + mean, :201-203): each lane keeps
    // the largest of its rows' sims; the selection is order-free, so 32-row chunks give
    // exactly the single-pass result
    float tk[kMaxTopk];
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) tk[q] = -INFINITY;
    bool nan = false;
    for (int t0 = 0; t0 < (chunked ? T : 1); t0 += 32) {
      if (chunked) load_a_frag(A.bank + (slot * Tmax + t0 + col) * D + 64 * h, t0 + col < T, a);
      f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 64; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
      // prefetch the next row's bank while the MFMA chain drains
      if (!chunked && i + 1 < iend) {
        const int64_t sn = slot_of(i + 1);
        const int Tn = min(A.bank_len[sn], Tmax);
        load_a_frag(A.bank + (sn * Tmax + col) * D + 64 * h, col < Tn, a);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float x = t < T ? acc[r] : -INFINITY;
        nan |= __builtin_isnan(x);
        topk_insert(tk, x);
      }
    }
    float other[kMaxTopk];
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) other[q] = __shfl_xor(tk[q], 32);
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) topk_insert(tk, other[q]);
    const int k = min(topk, T);
    float app;
    if (k <= 0) {
      app = 1.0f;  // empty bank, no EMA fallback (:180-186 / :197-199)
    } else {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < kMaxTopk; ++q)
        if (q < k) sum = sum + tk[q];
      app = 1.0f - sum / (float)k;
    }
    app = app_nan(app, nan && k > 0, col);
    if (h != 0 || !jok) continue;

    float cen, scl, cf;
    const float tot = combine(A.p, app, A.pbox + slot * 4, A.conf_prev[slot], ccx, ccy, Ac, ccv,
                              A.p.gate && A.gate_on[slot], A.gmean + slot * 4, A.gsinv + slot * 16,
                              z0, z1, z2, z3, cen, scl, cf);
    const int64_t o = ((int64_t)f * A.Mmax + i) * A.Nmax + j;
    if (A.C_total) A.C_total[o] = tot;
    if (A.C_app) A.C_app[o] = app;
    if (A.C_center) A.C_center[o] = cen;
    if (A.C_scale) A.C_scale[o] = scl;
    if (A.C_conf) A.C_conf[o] = cf;
  }
}

// ---------------------------------------------------------------------------
// cost2_kernel (default): the track's bank is the resident operand, the
// detections stream.  Workgroup = (4 tracks, frame), one wave per track.  The
// prologue renormalises the frame's detections once into LDS (the same double
// sum-of-squares / f32 divide as cost_kernel, so every B fragment is bit-identical)
// and precomputes their box / conf / KF-measurement terms; each wave then loads
// its track's <=30x128 bank into registers ONCE (cost_kernel re-read it for every
// 32-detection tile: 178 MB of HBM reads per 8 x 256 x 256 launch against 33 MB of
// algorithmic bytes) and walks the detection tiles with the B fragments read from
// LDS (row stride 132 floats: the 16-lane groups of a ds_read_b128 hit distinct
// banks).  MFMA chain, top-k and epilogue are cost_kernel's: identical outputs.
constexpr int C2_LD = D + 4;
struct DetTerms {
  float ccx, ccy, Ac, ccv;
  double z0, z1, z2, z3;
};
constexpr size_t c2_lds_bytes(int nmax) { return (size_t)nmax * C2_LD * 4 + (size_t)nmax * sizeof(DetTerms); }

__global__ void __launch_bounds__(256) cost2_kernel(const CostArgs A) {
  extern __shared__ __align__(16) float dl[];
  const int f = blockIdx.y;
  const int M = A.dev_M ? min(A.dev_M[f], A.Mmax) : A.M[f];
  const int N = A.dev_N ? min(A.dev_N[f], A.Nmax) : A.N[f];
  if ((int)blockIdx.x * 4 >= M || N == 0) return;  // whole workgroup: before any barrier
  DetTerms* dt_lds = reinterpret_cast<DetTerms*>(dl + (size_t)A.Nmax * C2_LD);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // ---- prologue: renormalised detections (thread pair 2j, 2j + 1 = halves of row j)
  for (int q = threadIdx.x; q < 2 * N; q += 256) {
    const int j = q >> 1, h = q & 1;
    float b[64];
    load_a_frag(A.det_emb + ((int64_t)f * A.Nmax + j) * D + 64 * h, true, b);
    double ss = 0.0;
#pragma unroll
    for (int s = 0; s < 64; ++s) ss += (double)b[s] * (double)b[s];
    ss += __shfl_xor(ss, 1);
    const float nrm = (float)sqrt(ss) + 1e-12f;
    float* o = dl + j * C2_LD + 64 * h;
#pragma unroll
    for (int s = 0; s < 64; s += 4)
      *reinterpret_cast<float4*>(o + s) = make_float4(b[s] / nrm, b[s + 1] / nrm, b[s + 2] / nrm, b[s + 3] / nrm);
  }
  for (int j = threadIdx.x; j < N; j += 256) {
    DetTerms t;
    det_terms(A.dbox + ((int64_t)f * A.Nmax + j) * 4, A.conf_cur[(int64_t)f * A.Nmax + j], t.ccx, t.ccy, t.Ac,
              t.ccv, t.z0, t.z1, t.z2, t.z3);
    dt_lds[j] = t;
  }
  __syncthreads();

  const int i = blockIdx.x * 4 + wave;
  if (i >= M) return;
  const int col = lane & 31, h = lane >> 5;
  const int64_t slot = A.row_slot ? (int64_t)A.row_slot[(int64_t)f * A.rs_ld + i] : (int64_t)f * A.Mmax + i;
  const int T = min(A.bank_len[slot], A.Tmax);
  float a[64];
  load_a_frag(A.bank + (slot * A.Tmax + col) * D + 64 * h, col < T, a);
  const int topk = A.p.topk;
  const bool gate = A.p.gate && A.gate_on[slot];
  for (int j0 = 0; j0 < N; j0 += 32) {
    const int j = j0 + col;
    const bool jok = j < N;
    float b[64];
    {
      const float* bp = dl + (jok ? j : 0) * C2_LD + 64 * h;
#pragma unroll
      for (int s = 0; s < 64; s += 4) {
        const float4 v = jok ? *reinterpret_cast<const float4*>(bp + s) : make_float4(0.f, 0.f, 0.f, 0.f);
        b[s] = v.x; b[s + 1] = v.y; b[s + 2] = v.z; b[s + 3] = v.w;
      }
    }
    f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 64; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    float tk[kMaxTopk];
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) tk[q] = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float x = t < T ? acc[r] : -INFINITY;
      nan |= __builtin_isnan(x);
      topk_insert(tk, x);
    }
    float other[kMaxTopk];
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) other[q] = __shfl_xor(tk[q], 32);
#pragma unroll
    for (int q = 0; q < kMaxTopk; ++q) topk_insert(tk, other[q]);
    const int k = min(topk, T);
    float app;
    if (k <= 0) {
      app = 1.0f;
    } else {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < kMaxTopk; ++q)
        if (q < k) sum = sum + tk[q];
      app = 1.0f - sum / (float)k;
    }
    app = app_nan(app, nan && k > 0, col);
    if (h != 0 || !jok) continue;
    const DetTerms t = dt_lds[j];
    float cen, scl, cf;
    const float tot = combine(A.p, app, A.pbox + slot * 4, A.conf_prev[slot], t.ccx, t.ccy, t.Ac, t.ccv, gate,
                              A.gmean + slot * 4, A.gsinv + slot * 16, t.z0, t.z1, t.z2, t.z3, cen, scl, cf);
    const int64_t o = ((int64_t)f * A.Mmax + i) * A.Nmax + j;
    if (A.C_total) A.C_total[o] = tot;
    if (A.C_app) A.C_app[o] = app;
    if (A.C_center) A.C_center[o] = cen;
    if (A.C_scale) A.C_scale[o] = scl;
    if (A.C_conf) A.C_conf[o] = cf;
  }
}

// ---------------------------------------------------------------------------
// cost3 (trk_build_cost_dev with a workspace): the track's bank is the resident
// MFMA A operand, the detections stream -- with no LDS, so its workgroups are
// placed beside the encoder's (cost2's 147 KiB LDS image of the frame's
// detections made them wait for a CU of their own).
//   det_prep_kernel  once per frame: the renormalised detection rows (thread pair
//                    2j, 2j + 1 = the halves of row j; the same double
//                    sum-of-squares and f32 divide as cost_kernel, so every B
//                    fragment is bit-identical) and their box / conf / KF terms,
//                    into the workspace
//   cost3_kernel     one wave per track row: its <=30x128 bank is read from HBM
//                    once into registers; the 32-detection tiles' B fragments come
//                    from the workspace (L2-resident), the next tile's prefetched
//                    while the MFMA chain runs.  MFMA chain, top-k and epilogue are
//                    cost_kernel's: identical outputs.
// HBM bytes per launch: the live banks (M x T x 512 B) + the detections twice
// (N x 512 B) + the cost rows, against cost_kernel's bank read per 32-column tile.
// The similarity on the f16 MFMA (cost_split 1): each f32 x of a unit row as x ~ hi + 2^-11 lo with
// hi = f16(x) (f16 subnormals flushed to zero here, so the MFMA multiplies exactly the hi the
// residual was taken from) and lo = f16((x - hi) * 2^11) (scaled into f16's normal range).  Then
// a.b = sum hi_a hi_b + 2^-11 sum (hi_a lo_b + lo_a hi_b) + e, three products of exact f16 pairs
// with f32 accumulation (v_mfma_f32_32x32x16_f16: 32 cycles per 32x32x16, against the exact f32
// 32x32x2's 64 cycles per 32x32x2: 768 vs 4,096 cycles per 32-detection tile); |e| <= 3 * 2^-22
// sum |a_k b_k| + 128 * 2^-25 <= 1.1e-6 for unit rows (the dropped lo*lo term, the two f16
// roundings of lo, lo's subnormal floor), typically ~1e-8
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
struct Split16 {
  _Float16 hi, lo;
};
__device__ __forceinline__ Split16 split16(float x) {
  _Float16 hh = (_Float16)x;
  if (__builtin_fabsf((float)hh) < 6.103515625e-05f) hh = (_Float16)0.f;  // below 2^-14: subnormal
  return {hh, (_Float16)((x - (float)hh) * 2048.f)};
}

struct Cost3Work {
  float* dn;       // [F][Nmax][D] renormalised detections
  DetTerms* dt;    // [F][Nmax]
  unsigned long long* prof;  // trk_cost_set_prof (diagnostics): per wave [start, bank, chain+top-k, epilogue]
};
__device__ __forceinline__ unsigned long long c3_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
// detection rows padded to whole 32-detection tiles per frame
__host__ __device__ inline int64_t cost3_np(int64_t Nmax) { return (Nmax + 31) / 32 * 32; }
inline Cost3Work cost3_work(void* work, int64_t F, int64_t Nmax) {
  Cost3Work w;
  w.dn = reinterpret_cast<float*>(work);
  w.dt = reinterpret_cast<DetTerms*>(reinterpret_cast<unsigned char*>(work) + (size_t)F * cost3_np(Nmax) * D * 4);
  w.prof = nullptr;
  return w;
}

// The renormalised rows in MFMA fragment order: per frame, per 32-detection tile, 16 chunks of
// 1 KiB, chunk q = [lane 0..63][16 B] with lane = 32 h + (j & 31) (the B-operand lane of
// detection j's column, K half h).  Chunk q of the f32 rows holds elements 64 h + 4 q .. + 3;
// with SPLIT (f16 hi / lo pairs, split16) chunk 2 st holds the hi and chunk 2 st + 1 the lo of
// elements 64 h + 8 st .. + 7.  So each of a wave's 16 fragment loads per tile is one
// contiguous 1 KiB (the row-major image had every lane of a load on its own 512-B row: 64
// cache lines per load instruction, which bound cost3 at the L1's line rate)
__device__ __forceinline__ int64_t c3_chunk(int j, int q) {  // in floats, from the frame's base
  return ((int64_t)(j >> 5) * 16 + q) * 256;
}
template <bool SPLIT>
__global__ void __launch_bounds__(256) det_prep_kernel(const CostArgs A, Cost3Work w) {
  const int f = blockIdx.y;
  const int N = A.dev_N ? min(A.dev_N[f], A.Nmax) : A.N[f];
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int j = q >> 1, h = q & 1;
  if (j >= N) return;  // both threads of a pair leave together (N is per frame)
  float b[64];
  load_a_frag(A.det_emb + ((int64_t)f * A.Nmax + j) * D + 64 * h, true, b);
  double ss = 0.0;
#pragma unroll
  for (int s = 0; s < 64; ++s) ss += (double)b[s] * (double)b[s];
  ss += __shfl_xor(ss, 1);
  const float nrm = (float)sqrt(ss) + 1e-12f;
  float* o = w.dn + (int64_t)f * cost3_np(A.Nmax) * D + (32 * h + (j & 31)) * 4;
  if (SPLIT) {
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      h8v hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const Split16 v = split16(b[8 * st + e] / nrm);
        hi[e] = v.hi;
        lo[e] = v.lo;
      }
      *reinterpret_cast<h8v*>(o + c3_chunk(j, 2 * st)) = hi;
      *reinterpret_cast<h8v*>(o + c3_chunk(j, 2 * st + 1)) = lo;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q)
      *reinterpret_cast<float4*>(o + c3_chunk(j, q)) =
          make_float4(b[4 * q] / nrm, b[4 * q + 1] / nrm, b[4 * q + 2] / nrm, b[4 * q + 3] / nrm);
  }
  if (h == 0) {
    DetTerms t;
    det_terms(A.dbox + ((int64_t)f * A.Nmax + j) * 4, A.conf_cur[(int64_t)f * A.Nmax + j], t.ccx, t.ccy, t.Ac, t.ccv,
              t.z0, t.z1, t.z2, t.z3);
    w.dt[(int64_t)f * A.Nmax + j] = t;
  }
}

// B fragments of the 32-detection tile holding detection j, for this lane (fragment order above;
// a tile past the frame's last reads the last: the sims of columns past N are never stored, and an
// unconditional load keeps the compiler's vmcnt counting exact so the next tile's loads stay in
// flight across the current MFMA chain; columns past N in the last tile read rows det_prep did not
// write, for the same unstored sims)
// (tile: wave-uniform, so the tile base is a scalar address and the lane's offset one VGPR)
// (buffer loads on the frame's fragment image: the tile's and 4-KiB group's offset a scalar, the
// lane's byte offset one VGPR plus an immediate -- with plain pointers the compiler kept a 64-bit
// address per load live across the loop and spilled them)
typedef unsigned c3u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ c3u4 c3_frag(__amdgpu_buffer_rsrc_t rs, int tile, int q, int loff) {
  const int so = __builtin_amdgcn_readfirstlane(tile) * 16384 + (q >> 2) * 4096;
  return __builtin_amdgcn_raw_buffer_load_b128(rs, loff + (q & 3) * 1024, so, 0);
}
__device__ __forceinline__ void load_b_tile(__amdgpu_buffer_rsrc_t rs, int tile, int lane, float (&b)[64]) {
  const int loff = lane * 16;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 v = __builtin_bit_cast(float4, c3_frag(rs, tile, q, loff));
    b[4 * q + 0] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
  }
}

// the f16 split B fragments (lane half h, K step st: elements 64 h + 8 st .. + 7, hi in bh, lo in bl)
__device__ __forceinline__ void load_b_split(__amdgpu_buffer_rsrc_t rs, int tile, int lane, h8v (&bh)[8], h8v (&bl)[8]) {
  const int loff = lane * 16;
#pragma unroll
  for (int st = 0; st < 8; ++st) {
    bh[st] = __builtin_bit_cast(h8v, c3_frag(rs, tile, 2 * st, loff));
    bl[st] = __builtin_bit_cast(h8v, c3_frag(rs, tile, 2 * st + 1, loff));
  }
}

// KT: top-k network length (5 when the requested topk <= 5 -- the YAML's 5 -- else kMaxTopk).
// SPLIT: the similarities from f16 hi / lo splits (split16) on the f16 MFMA, else exact f32 MFMA
template <int KT, bool SPLIT>
__global__ void __launch_bounds__(256, 2) cost3_kernel(const CostArgs A, const Cost3Work w) {
  const int f = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // track terms below: scalar loads
  const int M = A.dev_M ? min(A.dev_M[f], A.Mmax) : A.M[f];
  const int N = A.dev_N ? min(A.dev_N[f], A.Nmax) : A.N[f];
  if (N == 0) return;  // no barriers below
  // grid-stride over the frame's rows: the grid is sized for the usual count (kCost3Rows),
  // not the launch's bound (live tracks + detections in flight), so a bound 4x the live
  // count costs no idle waves; a frame with more rows than the grid loops
  for (int i = blockIdx.x * 4 + wave; i < M; i += gridDim.x * 4) {
    const int col = lane & 31, h = lane >> 5;
    const int64_t slot = A.row_slot ? (int64_t)A.row_slot[(int64_t)f * A.rs_ld + i] : (int64_t)f * A.Mmax + i;
    const int T = min(A.bank_len[slot], A.Tmax);
    unsigned long long p0 = 0, p1 = 0, pc = 0, pe = 0, pt = 0;
    if (w.prof) p0 = c3_stamp();
    float a[64];
    load_a_frag(A.bank + (slot * A.Tmax + col) * D + 64 * h, col < T, a);
    if (w.prof) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      p1 = pt = c3_stamp();
    }
    const int topk = A.p.topk;
    const bool gate = A.p.gate && A.gate_on[slot];
    // the track's box / conf / gate terms, hoisted out of the tile loop into scalar
    // registers (wave-uniform; readfirstlane tells the compiler so)
    auto uni_f = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    auto uni_d = [](double v) {
      const unsigned long long u = (unsigned long long)__double_as_longlong(v);
      const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
      const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
      return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    };
    float tb[4];
  #pragma unroll
    for (int q = 0; q < 4; ++q) tb[q] = uni_f(A.pbox[slot * 4 + q]);
    const float tconf = uni_f(A.conf_prev[slot]);
    double tg[4] = {0.0, 0.0, 0.0, 0.0}, tS[16];
  #pragma unroll
    for (int q = 0; q < 16; ++q) tS[q] = 0.0;
    if (gate) {
  #pragma unroll
      for (int q = 0; q < 4; ++q) tg[q] = uni_d(A.gmean[slot * 4 + q]);
  #pragma unroll
      for (int q = 0; q < 16; ++q) tS[q] = uni_d(A.gsinv[slot * 16 + q]);
    }
    // the frame's fragment image as one buffer (descriptor inputs readfirstlane'd: uniform)
    // (each half through uint32_t: readfirstlane returns int, whose sign extension would set the
    // address's upper half to all ones when bit 31 of the lower is set)
    const uint64_t da = reinterpret_cast<uint64_t>(w.dn + (int64_t)f * cost3_np(A.Nmax) * D);
    const uint32_t da_lo = __builtin_amdgcn_readfirstlane((uint32_t)da);
    const uint32_t da_hi = __builtin_amdgcn_readfirstlane((uint32_t)(da >> 32));
    const __amdgpu_buffer_rsrc_t dnf = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)da_hi << 32) | (uint64_t)da_lo), 0,
        __builtin_amdgcn_readfirstlane((int)(cost3_np(A.Nmax) * D * 4)), 0x00020000);
    const DetTerms* dtf = w.dt + (int64_t)f * A.Nmax;
    float* Ct = A.C_total ? A.C_total + ((int64_t)f * A.Mmax + i) * A.Nmax : nullptr;
    float* Ca = A.C_app ? A.C_app + ((int64_t)f * A.Mmax + i) * A.Nmax : nullptr;
    // two 32-detection tiles (A = j0.., B = j0 + 32..): each lane reduces its 16 bank rows of both
    // to partial top-k lists, then lane half h finishes tile h's column (the halves swap the
    // partial list the other one needs), so the merge, the epilogue and the stores run once per
    // column instead of once per lane half.  `sims` runs the MFMA chain of one tile (prefetching
    // the next tile's B fragments) and leaves the 32 x 32 similarities in the f32x16 layout
    auto pair = [&](int j0, auto&& simsA, auto&& simsB, bool hasB) {
      const int j = j0 + 32 * h + col;
      float tk[2][KT];
      unsigned long long nanb[2];
      auto partial = [&](const f32x16& acc, float (&o)[KT]) {
        bool nan = false;
        float x[16];
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tr = (r & 3) + 8 * (r >> 2) + 4 * h;
          x[r] = tr < T ? acc[r] : -INFINITY;
          nan |= __builtin_isnan(x[r]);
        }
        if constexpr (KT == 5) {
          float o5[5];
          top5_of16(x, o5);
  #pragma unroll
          for (int q = 0; q < 5; ++q) o[q] = o5[q];
        } else {
  #pragma unroll
          for (int q = 0; q < KT; ++q) o[q] = -INFINITY;
  #pragma unroll
          for (int r = 0; r < 16; ++r) topk_insert_n(o, x[r]);
        }
        return __ballot(nan);
      };
      nanb[0] = partial(simsA(j0), tk[0]);
      // this lane's column's box / conf terms, loaded under tile B's chain (its gate terms after it:
      // registers)
      const DetTerms* tp = dtf + min(j, N - 1);
      const float4 tf = *reinterpret_cast<const float4*>(tp);
      if (hasB) {
        nanb[1] = partial(simsB(j0 + 32), tk[1]);
      } else {
        nanb[1] = 0;
  #pragma unroll
        for (int q = 0; q < KT; ++q) tk[1][q] = -INFINITY;
      }
      const double2 tz01 = *reinterpret_cast<const double2*>(&tp->z0);  // (DetTerms: 16-B aligned halves)
      const double2 tz23 = *reinterpret_cast<const double2*>(&tp->z2);
      float mine[KT], other[KT], fin[KT];
  #pragma unroll
      for (int q = 0; q < KT; ++q) {
        mine[q] = h ? tk[1][q] : tk[0][q];
        other[q] = __shfl_xor(h ? tk[0][q] : tk[1][q], 32);
      }
      if constexpr (KT == 5) {
        float o5[5];
        top5_merge(mine, other, o5);
  #pragma unroll
        for (int q = 0; q < 5; ++q) fin[q] = o5[q];
      } else {
  #pragma unroll
        for (int q = 0; q < KT; ++q) fin[q] = mine[q];
  #pragma unroll
        for (int q = 0; q < KT; ++q) topk_insert_n(fin, other[q]);
      }
      const int k = min(topk, T);
      float sum = 0.f;
  #pragma unroll
      for (int q = 0; q < KT; ++q)
        if (q < k) sum = sum + fin[q];
      const unsigned long long nb = h ? nanb[1] : nanb[0];
      const bool nan = (((nb >> col) | (nb >> (col + 32))) & 1ull) && k > 0;
      const float app = nan ? __builtin_nanf("") : (k <= 0 ? 1.0f : 1.0f - sum / (float)k);
      if (w.prof) {
        asm volatile("" ::"v"(app));
        const unsigned long long t1 = c3_stamp();
        pc += t1 - pt;
        pt = t1;
      }
      float cen, scl, cf;
      const float tot = combine(A.p, app, tb, tconf, tf.x, tf.y, tf.z, tf.w, gate, tg, tS, tz01.x, tz01.y, tz23.x, tz23.y,
                                cen, scl, cf);
      if (j < N) {
        if (Ct) Ct[j] = tot;
        if (Ca) Ca[j] = app;
      }
    };
    if constexpr (SPLIT) {
      h8v ah[8], al[8];
  #pragma unroll
      for (int st = 0; st < 8; ++st)
  #pragma unroll
        for (int e = 0; e < 8; ++e) {
          const Split16 v = split16(a[8 * st + e]);
          ah[st][e] = v.hi;
          al[st][e] = v.lo;
        }
      auto chain = [&](const h8v (&bh)[8], const h8v (&bl)[8], h8v (&nh)[8], h8v (&nl)[8]) {
        return [&](int jt) {  // jt: the tile's first detection (the next tile is prefetched)
          load_b_split(dnf, min((jt >> 5) + 1, (N - 1) >> 5), lane, nh, nl);
          __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the chain
          // one accumulator (a second one spilled the kernel): the 2^11-scaled cross terms
          // first, scaled back exactly, then the hi x hi products on top
          f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int st = 0; st < 8; ++st) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[st], bl[st], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[st], bh[st], acc, 0, 0, 0);
          }
  #pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = acc[r] * (1.0f / 2048.0f);
  #pragma unroll
          for (int st = 0; st < 8; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[st], bh[st], acc, 0, 0, 0);
          return acc;
        };
      };
      h8v h0[8], l0[8], h1[8], l1[8];
      load_b_split(dnf, 0, lane, h0, l0);
      for (int j0 = 0; j0 < N; j0 += 64) pair(j0, chain(h0, l0, h1, l1), chain(h1, l1, h0, l0), j0 + 32 < N);
    } else {
      auto chain = [&](const float (&b)[64], float (&bn)[64]) {
        return [&](int jt) {
          load_b_tile(dnf, min((jt >> 5) + 1, (N - 1) >> 5), lane, bn);
          __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the chain
          f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int s = 0; s < 64; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
          return acc;
        };
      };
      float b0[64], b1[64];
      load_b_tile(dnf, 0, lane, b0);
      for (int j0 = 0; j0 < N; j0 += 64) pair(j0, chain(b0, b1), chain(b1, b0), j0 + 32 < N);
    }
    if (w.prof) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long t1 = c3_stamp();
      pe = t1 - p1 - pc;
      if (lane == 0) {
        unsigned long long* o = w.prof + ((int64_t)(f * gridDim.x + blockIdx.x) * 4 + wave) * 4;
        o[0] = p0; o[1] = p1 - p0; o[2] = pc; o[3] = pe;
      }
    }
  }
}

// C_app given (costCard.cal_cost API): elementwise combine over [M, N].
__global__ void __launch_bounds__(256)
combine_kernel(int M, int N, const float* __restrict__ C_app, const float* __restrict__ pbox,
               const float* __restrict__ conf_prev, const float* __restrict__ dbox,
               const float* __restrict__ conf_cur, const double* __restrict__ gmean,
               const double* __restrict__ gsinv, const int32_t* __restrict__ gate_on,
               trk_cost_params p, float* C_total, float* C_center, float* C_scale, float* C_conf) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)M * N) return;
  const int i = (int)(q / N), j = (int)(q % N);
  float ccx, ccy, Ac, ccv;
  double z0, z1, z2, z3;
  det_terms(dbox + (int64_t)j * 4, conf_cur[j], ccx, ccy, Ac, ccv, z0, z1, z2, z3);
  const bool g = p.gate && gate_on[i];
  float cen, scl, cf;
  const float tot = combine(p, C_app[q], pbox + (int64_t)i * 4, conf_prev[i], ccx, ccy, Ac, ccv, g,
                            g ? gmean + (int64_t)i * 4 : nullptr, g ? gsinv + (int64_t)i * 16 : nullptr,
                            z0, z1, z2, z3, cen, scl, cf);
  if (C_total) C_total[q] = tot;
  if (C_center) C_center[q] = cen;
  if (C_scale) C_scale[q] = scl;
  if (C_conf) C_conf[q] = cf;
}

}  // namespace

extern "C" int trk_cost_combine(int64_t M, int64_t N, const float* C_app, const float* pbox,
                                const float* conf_prev, const float* dbox, const float* conf_cur,
                                const double* gmean, const double* gsinv, const int32_t* gate_on,
                                const trk_cost_params* host_params, float* C_total,
                                float* C_center, float* C_scale, float* C_conf, void* stream) {
  TRK_REQUIRE(M >= 0 && N >= 0 && M * N < ((int64_t)1 << 31), "cost_combine: bad shape");
  TRK_REQUIRE(host_params, "cost_combine: null params");
  if (M == 0 || N == 0) return TRK_OK;
  TRK_REQUIRE(C_app && pbox && conf_prev && dbox && conf_cur, "cost_combine: null input pointer");
  TRK_REQUIRE(!host_params->gate || (gmean && gsinv && gate_on),
              "cost_combine: gating needs gmean/gsinv/gate_on");
  const int64_t n = M * N;
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (int)M, (int)N, C_app, pbox, conf_prev,
                     dbox, conf_cur, gmean, gsinv, gate_on, *host_params, C_total, C_center, C_scale,
                     C_conf);
  return trk::check_launch("combine_kernel");
}

extern "C" int trk_build_cost(int64_t F, int64_t Mmax, int64_t Nmax, const int32_t* host_M,
                              const int32_t* host_N, const int32_t* row_slot, int64_t Tmax,
                              const float* bank, const int32_t* bank_len, const float* pbox,
                              const float* conf_prev, const double* gmean, const double* gsinv,
                              const int32_t* gate_on, const float* det_emb, const float* dbox,
                              const float* conf_cur, const trk_cost_params* host_params,
                              float* C_total, float* C_app, float* C_center, float* C_scale,
                              float* C_conf, void* stream) {
  TRK_REQUIRE(F >= 0 && Mmax >= 0 && Nmax >= 0, "build_cost: negative shape");
  TRK_REQUIRE(host_params, "build_cost: null params");
  TRK_REQUIRE(Tmax >= 1 && Tmax <= 1024, "build_cost: Tmax (hist_max) must be in [1, 1024], got %lld",
              (long long)Tmax);
  TRK_REQUIRE(host_params->topk >= 0 && host_params->topk <= kMaxTopk,
              "build_cost: topk must be in [0, %d]", kMaxTopk);
  TRK_REQUIRE(Mmax < (1 << 30) && Nmax < (1 << 30), "build_cost: shape too large");
  if (F == 0 || Mmax == 0 || Nmax == 0) return TRK_OK;
  TRK_REQUIRE(host_M && host_N, "build_cost: null shape arrays");
  TRK_REQUIRE(bank && bank_len && pbox && conf_prev && det_emb && dbox && conf_cur,
              "build_cost: null input pointer");
  TRK_REQUIRE(!host_params->gate || (gmean && gsinv && gate_on), "build_cost: gating needs gmean/gsinv/gate_on");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t f0 = 0; f0 < F; f0 += kMaxFrames) {
    const int nf = (int)std::min<int64_t>(kMaxFrames, F - f0);
    CostArgs a;
    memset(&a, 0, sizeof a);
    int mmax = 0, nmax = 0;
    for (int q = 0; q < nf; ++q) {
      TRK_REQUIRE(host_M[f0 + q] >= 0 && host_M[f0 + q] <= Mmax && host_N[f0 + q] >= 0 &&
                      host_N[f0 + q] <= Nmax,
                  "build_cost: frame %lld M/N outside [0, Mmax/Nmax]", (long long)(f0 + q));
      a.M[q] = host_M[f0 + q];
      a.N[q] = host_N[f0 + q];
      mmax = std::max(mmax, a.M[q]);
      nmax = std::max(nmax, a.N[q]);
    }
    if (mmax == 0 || nmax == 0) continue;
    const int64_t fr = f0;
    a.F = nf; a.Mmax = (int)Mmax; a.Nmax = (int)Nmax; a.Tmax = (int)Tmax; a.rs_ld = (int)Mmax;
    a.row_slot = row_slot ? row_slot + fr * Mmax : nullptr;
    // without row_slot, slot = f*Mmax + i indexes the per-frame-packed arrays
    const int64_t so = row_slot ? 0 : fr * Mmax;
    a.bank = bank + so * Tmax * D;
    a.bank_len = bank_len + so;
    a.pbox = pbox + so * 4;
    a.conf_prev = conf_prev + so;
    a.gmean = gmean ? gmean + so * 4 : nullptr;
    a.gsinv = gsinv ? gsinv + so * 16 : nullptr;
    a.gate_on = gate_on ? gate_on + so : nullptr;
    a.det_emb = det_emb + fr * Nmax * D;
    a.dbox = dbox + fr * Nmax * 4;
    a.conf_cur = conf_cur + fr * Nmax;
    const int64_t co = fr * Mmax * Nmax;
    a.C_total = C_total ? C_total + co : nullptr;
    a.C_app = C_app ? C_app + co : nullptr;
    a.C_center = C_center ? C_center + co : nullptr;
    a.C_scale = C_scale ? C_scale + co : nullptr;
    a.C_conf = C_conf ? C_conf + co : nullptr;
    a.p = *host_params;
    const size_t lds2 = c2_lds_bytes((int)Nmax);
    if (g_cost_v2 && lds2 <= 160 * 1024 && Tmax <= 32) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(cost2_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      dim3 grid((unsigned)((mmax + 3) / 4), (unsigned)nf);
      hipLaunchKernelGGL(cost2_kernel, grid, dim3(256), lds2, st, a);
      if (int e = trk::check_launch("cost2_kernel")) return e;
      continue;
    }
    dim3 grid((unsigned)((nmax + 31) / 32), (unsigned)((mmax + kRowsPerWG - 1) / kRowsPerWG), (unsigned)nf);
    hipLaunchKernelGGL(cost_kernel, grid, dim3(256), 0, st, a);
    if (int e = trk::check_launch("cost_kernel")) return e;
  }
  return TRK_OK;
}

extern "C" int64_t trk_cost_work_bytes(int64_t F, int64_t Nmax) {
  if (F <= 0 || Nmax <= 0) return 0;
  return F * (cost3_np(Nmax) * D * 4 + Nmax * (int64_t)sizeof(DetTerms));
}

extern "C" int trk_build_cost_dev(int64_t F, int64_t Mmax, int64_t Nmax, const int32_t* dev_M, const int32_t* dev_N,
                                  const int32_t* row_slot, int64_t rs_ld, int64_t Tmax, const float* bank,
                                  const int32_t* bank_len, const float* pbox, const float* conf_prev,
                                  const double* gmean, const double* gsinv, const int32_t* gate_on,
                                  const float* det_emb, const float* dbox, const float* conf_cur,
                                  const trk_cost_params* host_params, float* C_total, float* C_app, void* work,
                                  void* stream) {
  TRK_REQUIRE(F >= 0 && Mmax >= 0 && Nmax >= 0, "build_cost_dev: negative shape");
  TRK_REQUIRE(host_params, "build_cost_dev: null params");
  TRK_REQUIRE(Tmax >= 1 && Tmax <= 1024, "build_cost_dev: Tmax (hist_max) must be in [1, 1024], got %lld",
              (long long)Tmax);
  TRK_REQUIRE(host_params->topk >= 0 && host_params->topk <= kMaxTopk, "build_cost_dev: topk must be in [0, %d]",
              kMaxTopk);
  TRK_REQUIRE(Mmax < (1 << 30) && Nmax < (1 << 30) && rs_ld >= 0 && rs_ld < (1 << 30), "build_cost_dev: shape too large");
  if (F == 0 || Mmax == 0 || Nmax == 0) return TRK_OK;
  TRK_REQUIRE(dev_M && dev_N && row_slot, "build_cost_dev: null size / row_slot arrays");
  TRK_REQUIRE(bank && bank_len && pbox && conf_prev && det_emb && dbox && conf_cur, "build_cost_dev: null input");
  TRK_REQUIRE(!host_params->gate || (gmean && gsinv && gate_on), "build_cost_dev: gating needs gmean/gsinv/gate_on");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t f0 = 0; f0 < F; f0 += kMaxFrames) {
    const int nf = (int)std::min<int64_t>(kMaxFrames, F - f0);
    CostArgs a;
    memset(&a, 0, sizeof a);
    a.F = nf; a.Mmax = (int)Mmax; a.Nmax = (int)Nmax; a.Tmax = (int)Tmax; a.rs_ld = (int)rs_ld;
    a.dev_M = dev_M + f0;
    a.dev_N = dev_N + f0;
    a.row_slot = row_slot + f0 * rs_ld;
    a.bank = bank; a.bank_len = bank_len; a.pbox = pbox; a.conf_prev = conf_prev;
    a.gmean = gmean; a.gsinv = gsinv; a.gate_on = gate_on;
    a.det_emb = det_emb + f0 * Nmax * D;
    a.dbox = dbox + f0 * Nmax * 4;
    a.conf_cur = conf_cur + f0 * Nmax;
    const int64_t co = f0 * Mmax * Nmax;
    a.C_total = C_total ? C_total + co : nullptr;
    a.C_app = C_app ? C_app + co : nullptr;
    a.p = *host_params;
    if (work && !g_cost_v2 && Tmax <= 32) {
      // the workspace holds all F frames; this chunk's rows start at frame f0
      Cost3Work w = cost3_work(work, F, Nmax);
      w.prof = g_cost_prof.get() ? g_cost_prof.get() + f0 * ((Mmax + 3) / 4) * 16 : nullptr;
      w.dn += f0 * cost3_np(Nmax) * D;
      w.dt += f0 * Nmax;
      const dim3 pgrid((unsigned)((2 * Nmax + 255) / 256), (unsigned)nf);
      if (g_cost_split)
        hipLaunchKernelGGL(det_prep_kernel<true>, pgrid, dim3(256), 0, st, a, w);
      else
        hipLaunchKernelGGL(det_prep_kernel<false>, pgrid, dim3(256), 0, st, a, w);
      if (int e = trk::check_launch("det_prep_kernel")) return e;
      const dim3 cgrid((unsigned)std::min<int64_t>((Mmax + 3) / 4, kCost3Rows / 4), (unsigned)nf);
      if (host_params->topk <= 5) {
        if (g_cost_split)
          hipLaunchKernelGGL((cost3_kernel<5, true>), cgrid, dim3(256), 0, st, a, w);
        else
          hipLaunchKernelGGL((cost3_kernel<5, false>), cgrid, dim3(256), 0, st, a, w);
      } else {
        if (g_cost_split)
          hipLaunchKernelGGL((cost3_kernel<kMaxTopk, true>), cgrid, dim3(256), 0, st, a, w);
        else
          hipLaunchKernelGGL((cost3_kernel<kMaxTopk, false>), cgrid, dim3(256), 0, st, a, w);
      }
      if (int e = trk::check_launch("cost3_kernel")) return e;
      continue;
    }
    dim3 grid((unsigned)((Nmax + 31) / 32), (unsigned)((Mmax + kRowsPerWG - 1) / kRowsPerWG), (unsigned)nf);
    hipLaunchKernelGGL(cost_kernel, grid, dim3(256), 0, st, a);
    if (int e = trk::check_launch("cost_kernel")) return e;
  }
  return TRK_OK;
}

// diagnostics: cost3 per-wave s_memtime breakdown [start, bank load, MFMA chain +
// top-k, epilogue] (u64 x 4 per wave, 4 waves per (frame, row block)); NULL = off
extern "C" int trk_cost_set_prof(unsigned long long* buf) {
  g_cost_prof.set(buf);
  return TRK_OK;
}
