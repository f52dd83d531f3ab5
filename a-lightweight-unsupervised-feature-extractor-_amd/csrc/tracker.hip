// Device-resident track state for the tracker hot path (gfx950 / MI355X).
//
// The reference keeps one filterpy KalmanFilter + Python lists per track and
// walks them in Python every frame.  Here the state of every track of every
// stream lives in HBM slot arrays and each per-frame operation is one launch:
//   trk_kf_predict   Tracking.predict_all           reference model/mainTracking.py:340-345
//                    + x_to_bbox_xyxy               model/utils/costTool/KalmanFilter.py:19-33
//                    + the gate inputs of gating_distance_maha (KalmanFilter.py:105-116)
//   trk_track_update Tracking.update_matched        mainTracking.py:375-448
//                    (filterpy update, Joseph form; last_* fields; appearance
//                    gates conf / cost / post-update Mahalanobis; EMA feature;
//                    bank push with hist_max)
//   trk_track_init   Tracking.create_new_tracks / creat_item / init_kf_from_bbox
//                    mainTracking.py:99-140,362-373, KalmanFilter.py:36-101
// KF constants are init_kf_from_bbox's defaults: dt = 1, Q = diag(1,1,1,1,100,
// 100,100,100), R = I4, P0 = diag(10,10,10,10,1000,1000,1000,1000).  State is
// kept in float64 throughout (filterpy drifts from float32 to float64 after the
// first update -- SURVEY.md A.4 / §7 "Kalman state dtype drift").
//
// Slot layout (S slots): x [S][8] f64, P [S][64] f64, pbox [S][4] f32,
// last_conf [S] f32, gmean [S][4] f64, gsinv [S][16] f64, enc [S][128] f32
// (EMA feature, normalised), bank [S][T][128] f32 (unit rows, renormalised the
// way build_C_app_topk renormalises them at use, mainTracking.py:188-189),
// bank_len [S] i32, bank_head [S] i32.
#include "trk_common.h"

namespace {

constexpr int D = 128;

// 4x4 inverse, Gauss-Jordan with partial pivoting (f64).  Fully unrolled with the
// row swap as selects over static indices: a swap through a runtime row index put
// m[][] in scratch memory (272 B per lane; step_apply wrote 66 MB per launch of it).
// Same pivot choice (first row with the strictly largest |m[r][c]|) and operation
// order as the indexed form, so the results are bit-identical.
__device__ inline void inv4(const double* A, double* out) {
  double m[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m[r][c] = A[r * 4 + c];
      m[r][c + 4] = r == c ? 1.0 : 0.0;
    }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int p = c;
    double best = fabs(m[c][c]);
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const double v = fabs(m[r][c]);
      if (v > best) { best = v; p = r; }
    }
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const bool sw = p == r;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double a = m[c][k], b = m[r][k];
        m[c][k] = sw ? b : a;
        m[r][k] = sw ? a : b;
      }
    }
    const double d = m[c][c];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[c][k] /= d;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double fct = m[r][c];
#pragma unroll
      for (int k = 0; k < 8; ++k) m[r][k] -= fct * m[c][k];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) out[r * 4 + c] = m[r][c + 4];
}

// bbox_xyxy_to_z (KalmanFilter.py:5-16): double arithmetic, float32 values
__device__ inline void box_to_z(const float* b, double* z) {
  const double x1 = b[0], y1 = b[1], x2 = b[2], y2 = b[3];
  const double w = fmax(1.0, x2 - x1), h = fmax(1.0, y2 - y1);
  z[0] = (float)(x1 + 0.5 * w);
  z[1] = (float)(y1 + 0.5 * h);
  z[2] = (float)(w / h);
  z[3] = (float)h;
}

// gate inputs: H x and (H P H^T + R + 1e-9 I)^-1 (gating_distance_maha)
__device__ inline void gate_params(const double* x, const double* P, double* gm, double* gs) {
  double S[16];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) S[r * 4 + c] = P[r * 8 + c] + (r == c ? 1.0 + 1e-9 : 0.0);
  inv4(S, gs);
  for (int r = 0; r < 4; ++r) gm[r] = x[r];
}

__device__ inline double maha(const double* z, const double* gm, const double* gs) {
  double y[4], d2 = 0.0;
  for (int a = 0; a < 4; ++a) y[a] = z[a] - gm[a];
  for (int a = 0; a < 4; ++a) {
    double t = 0.0;
    for (int c = 0; c < 4; ++c) t += gs[a * 4 + c] * y[c];
    d2 += y[a] * t;
  }
  return d2;
}

// Tracking.predict_all for one slot: x = F x, P = F P F^T + Q, predicted box
// (x_to_bbox_xyxy) and the gate inputs
__device__ inline void kf_predict_slot(int64_t s, double* __restrict__ X, double* __restrict__ PP,
                                       float* __restrict__ pbox, double* __restrict__ gmean,
                                       double* __restrict__ gsinv) {
  double* x = X + s * 8;
  double* P = PP + s * 64;
  // x = F x
  for (int i = 0; i < 4; ++i) x[i] = x[i] + x[i + 4];
  // P = F P F^T + Q   (F = I + E(i, i+4))
  double FP[64];
  for (int r = 0; r < 8; ++r)
    for (int c = 0; c < 8; ++c) FP[r * 8 + c] = P[r * 8 + c] + (r < 4 ? P[(r + 4) * 8 + c] : 0.0);
  for (int r = 0; r < 8; ++r)
    for (int c = 0; c < 8; ++c) {
      double v = FP[r * 8 + c] + (c < 4 ? FP[r * 8 + c + 4] : 0.0);
      if (r == c) v += r < 4 ? 1.0 : 100.0;
      P[r * 8 + c] = v;
    }
  // predicted box (x_to_bbox_xyxy), handed to the cost as float32
  const double cx = x[0], cy = x[1];
  const double h = fmax(x[3], 1.0), a = fmax(x[2], 1e-3);
  const double w = fmax(a * h, 1.0);
  float* b = pbox + s * 4;
  b[0] = (float)(cx - 0.5 * w);
  b[1] = (float)(cy - 0.5 * h);
  b[2] = (float)(cx + 0.5 * w);
  b[3] = (float)(cy + 0.5 * h);
  gate_params(x, P, gmean + s * 4, gsinv + s * 16);
}

__global__ void __launch_bounds__(64)
kf_predict_kernel(int n, const int32_t* __restrict__ slots, double* __restrict__ X,
                  double* __restrict__ PP, float* __restrict__ pbox, double* __restrict__ gmean,
                  double* __restrict__ gsinv) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  kf_predict_slot(slots[t], X, PP, pbox, gmean, gsinv);
}

struct UpdArgs {
  int n;
  const int32_t* slots;     // [n]
  const int32_t* dets;      // [n] global detection rows
  const int64_t* cost_idx;  // [n] index into cost (matched C value), or null
  const float* cost;
  const float* dbox;        // [*][4]
  const float* dconf;       // [*]
  const float* demb;        // [*][128]
  double* X;
  double* P;
  float* pbox;
  float* last_conf;
  float* enc;
  float* bank;
  int32_t* bank_len;
  int32_t* bank_head;
  int T;
  float ema_alpha, conf_update_min, cost_update_max;
  double maha_thr;
};

// update_matched for one (slot s, detection d) pair, one wavefront (all 64
// lanes active; the workgroup is that one wave): the 8-D filter runs with one
// lane per element of the 8x8 products (LDS-shared operands, each element
// accumulated in the serial order, so the results equal a one-lane filter bit
// for bit), then the wave does the 128-D appearance update (2 dims per lane).
// conf: the detection's confidence as the caller's float (the appearance gate
// compares it in double, :416); has_cost / costv: the matched cost entry (:418).
__device__ void track_update_wave(const UpdArgs& A, int64_t s, int64_t d, double conf, bool has_cost,
                                  float costv, double conf_update_min, double cost_update_max,
                                  double maha_thr) {
  __shared__ double sP[64], sK[32], sIKH[64], sT1[64], sX[8];
  const int lane = threadIdx.x & 63;
  const int r = lane >> 3, c = lane & 7;
  double* x = A.X + s * 8;
  double* P = A.P + s * 64;
  sP[lane] = P[lane];
  if (lane < 8) sX[lane] = x[lane];
  double z[4];
  box_to_z(A.dbox + d * 4, z);
  __syncthreads();
  // filterpy KalmanFilter.update (R = I, H = [I4 | 0]): y, S = H P H^T + R, S^-1 (every lane)
  double y[4], S[16], SI[16];
  for (int q = 0; q < 4; ++q) y[q] = z[q] - sX[q];
  for (int q = 0; q < 4; ++q)
    for (int k = 0; k < 4; ++k) S[q * 4 + k] = sP[q * 8 + k] + (q == k ? 1.0 : 0.0);
  inv4(S, SI);
  if (lane < 32) {  // K = P H^T S^-1, element (lane / 4, lane % 4)
    const int kr = lane >> 2, kc = lane & 3;
    double v = 0.0;
    for (int k = 0; k < 4; ++k) v += sP[kr * 8 + k] * SI[k * 4 + kc];
    sK[lane] = v;
  }
  __syncthreads();
  double xn = 0.0;
  if (lane < 8) {  // x = x + K y
    double v = 0.0;
    for (int k = 0; k < 4; ++k) v += sK[lane * 4 + k] * y[k];
    xn = sX[lane] + v;
    x[lane] = xn;
  }
  // P = (I - K H) P (I - K H)^T + K R K^T, element (r, c) per lane
  sIKH[lane] = (r == c ? 1.0 : 0.0) - (c < 4 ? sK[r * 4 + c] : 0.0);
  __syncthreads();
  {
    double v = 0.0;
    for (int k = 0; k < 8; ++k) v += sIKH[r * 8 + k] * sP[k * 8 + c];
    sT1[lane] = v;
  }
  __syncthreads();
  double pn;
  {
    double v = 0.0;
    for (int k = 0; k < 8; ++k) v += sT1[r * 8 + k] * sIKH[c * 8 + k];
    double kk = 0.0;
    for (int k = 0; k < 4; ++k) kk += sK[r * 4 + k] * sK[c * 4 + k];
    pn = v + kk;
  }
  P[lane] = pn;
  __syncthreads();  // every read of the old P is done
  sP[lane] = pn;
  if (lane < 8) sX[lane] = xn;
  __syncthreads();
  int push = 0;
  if (lane == 0) {
    // last_* fields (update_matched :402-405)
    const float* b = A.dbox + d * 4;
    float* pb = A.pbox + s * 4;
    for (int k = 0; k < 4; ++k) pb[k] = b[k];
    A.last_conf[s] = (float)conf;
    // appearance-update gates (:417-426): conf, matched cost, post-update d2
    push = 1;
    if (conf < conf_update_min) push = 0;
    if (push && has_cost && (double)costv > cost_update_max) push = 0;
    if (push) {
      double gm[4], gs[16];
      gate_params(sX, sP, gm, gs);
      if (maha(z, gm, gs) > maha_thr) push = 0;
    }
  }
  push = __builtin_amdgcn_readfirstlane(push);  // lane 0's decision, wave-uniform
  if (!push) return;
  // det_emb_norm = emb / (||emb|| + 1e-12) (:429-431)
  const float* e = A.demb + d * D;
  const float e0 = e[lane], e1 = e[lane + 64];
  double ss = (double)e0 * e0 + (double)e1 * e1;
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
  const float nrm = (float)sqrt(ss) + 1e-12f;
  const float n0 = e0 / nrm, n1 = e1 / nrm;
  // EMA feature (:436-438): float32(0.9 * f + (1 - 0.9) * e), renormalised
  float* f = A.enc + s * D;
  const float ca = A.ema_alpha, cb = (float)(1.0 - (double)A.ema_alpha);
  const float f0 = ca * f[lane] + cb * n0, f1 = ca * f[lane + 64] + cb * n1;
  double fs = (double)f0 * f0 + (double)f1 * f1;
  for (int o = 32; o >= 1; o >>= 1) fs += __shfl_xor(fs, o);
  const float fn = (float)sqrt(fs) + 1e-12f;
  f[lane] = f0 / fn;
  f[lane + 64] = f1 / fn;
  // bank push (hist_max ring); stored renormalised as build_C_app_topk uses it
  double bs = (double)n0 * n0 + (double)n1 * n1;
  for (int o = 32; o >= 1; o >>= 1) bs += __shfl_xor(bs, o);
  const float bn = (float)sqrt(bs) + 1e-12f;
  const int head = A.bank_head[s];
  float* row = A.bank + (s * A.T + head % A.T) * D;
  row[lane] = n0 / bn;
  row[lane + 64] = n1 / bn;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    A.bank_head[s] = (head + 1) % A.T;
    A.bank_len[s] = min(A.bank_len[s] + 1, A.T);
  }
}

// new track from one detection (creat_item + init_kf_from_bbox), one wavefront
__device__ void track_init_wave(const UpdArgs& A, int64_t s, int64_t d, float conf) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    double* x = A.X + s * 8;
    double* P = A.P + s * 64;
    double z[4];
    box_to_z(A.dbox + d * 4, z);
    for (int k = 0; k < 8; ++k) x[k] = k < 4 ? z[k] : 0.0;
    for (int k = 0; k < 64; ++k) P[k] = 0.0;
    for (int k = 0; k < 8; ++k) P[k * 9] = k < 4 ? 10.0 : 1000.0;
    const float* b = A.dbox + d * 4;
    for (int k = 0; k < 4; ++k) A.pbox[s * 4 + k] = b[k];
    A.last_conf[s] = conf;
    A.bank_len[s] = 1;
    A.bank_head[s] = 1 % A.T;
  }
  const float* e = A.demb + d * D;
  const float e0 = e[lane], e1 = e[lane + 64];
  double ss = (double)e0 * e0 + (double)e1 * e1;
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
  const float nrm = (float)sqrt(ss) + 1e-12f;
  const float n0 = e0 / nrm, n1 = e1 / nrm;  // creat_item :112-114
  A.enc[s * D + lane] = n0;
  A.enc[s * D + lane + 64] = n1;
  double bs = (double)n0 * n0 + (double)n1 * n1;
  for (int o = 32; o >= 1; o >>= 1) bs += __shfl_xor(bs, o);
  const float bn = (float)sqrt(bs) + 1e-12f;
  float* row = A.bank + (s * A.T) * D;
  row[lane] = n0 / bn;
  row[lane + 64] = n1 / bn;
}

__global__ void __launch_bounds__(64)
track_update_kernel(const UpdArgs A) {
  const int t = blockIdx.x;
  if (t >= A.n) return;
  const int64_t d = A.dets[t];
  const bool hc = A.cost != nullptr;
  track_update_wave(A, A.slots[t], d, (double)A.dconf[d], hc, hc ? A.cost[A.cost_idx[t]] : 0.f,
                    (double)A.conf_update_min, (double)A.cost_update_max, A.maha_thr);
}

__global__ void __launch_bounds__(64)
track_init_kernel(const UpdArgs A) {
  const int t = blockIdx.x;
  if (t >= A.n) return;
  const int64_t d = A.dets[t];
  track_init_wave(A, A.slots[t], d, A.dconf[d]);
}

// ---------------------------------------------------------------------------
// Device-resident tracker step (trk_step_*): one workgroup per stream for the
// bookkeeping kernels, every list built with order-preserving block scans so
// the outputs come in the reference's list order.
constexpr int kStepThreads = 256;
constexpr int kStepMaxStreams = 64;   // streams per launch (kernarg-resident counts)
constexpr int kStepMaxDets = 4096;    // Nmax bound (LDS flags)
constexpr int kResHdr = 8;

struct StepArgs {
  trk_step_state st;
  trk_step_config cfg;
  int s0;
  int Mb;
  const float* C;         // stage cost matrix [S][Mb][Nmax]
  const int32_t* assign;  // [S][Mb]
  const float* det_emb;
  const float* dbox;
  const float* dconf;
  const double* dconf64;
  int ndet[kStepMaxStreams];
  int64_t frame[kStepMaxStreams];
};

// Order-preserving rank among the flagged threads of the block, offset by
// `base` (uniform; advanced by the block's flagged count).  Every thread of
// the block must call it (it synchronises).
__device__ int block_rank(bool flag, int* s_cnt, int& base) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t b = __ballot(flag);
  const int r = __popcll(b & ((1ull << lane) - 1));
  __syncthreads();  // s_cnt free (previous call's readers are done)
  if (lane == 0) s_cnt[w] = __popcll(b);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < kStepThreads / 64; ++q) {
    const int c = s_cnt[q];
    off += q < w ? c : 0;
    tot += c;
  }
  const int pos = base + off + r;
  base += tot;
  return pos;
}

__device__ __forceinline__ int64_t* res_of(const StepArgs& A, int s) {
  return A.st.result + (int64_t)s * (kResHdr + 3 * A.cfg.Nmax + A.cfg.cap);
}

// predict_all + row split (or the frame-without-detections path)
__global__ void __launch_bounds__(kStepThreads) step_begin_kernel(const StepArgs A) {
  __shared__ int s_cnt[kStepThreads / 64];
  const trk_step_state& S = A.st;
  const int s = A.s0 + blockIdx.x;
  const int N = A.ndet[blockIdx.x];
  const int64_t fr = A.frame[blockIdx.x];
  const int64_t cap = A.cfg.cap, base = (int64_t)s * cap;
  const int32_t* ord = S.order + base;
  const int n = S.n_live[s];
  int64_t* res = res_of(A, s);
  int64_t* ut = res + kResHdr + 2 * A.cfg.Nmax;
  const int t = threadIdx.x;
  if (t == 0) {
    S.ndet[s] = N;
    S.frame_id[s] = fr;
    S.ap_n[s] = 0;
    S.n2[s] = 0;
    S.m1[s] = 0;
    S.m2[s] = 0;
    S.lsap_status[s] = 0;
    S.lsap_status[A.cfg.S + s] = 0;
    for (int k = 0; k < kResHdr; ++k) res[k] = 0;
  }
  if (N == 0) {  // :467-471: every live track missed (no predict), purge in step_end
    for (int k = t; k < n; k += kStepThreads) {
      const int64_t g = base + ord[k];
      ut[k] = S.tid[g];
      S.miss[g] += 1;
    }
    if (t == 0) {
      S.flags[s] = 1;
      res[1] = n;
    }
    return;
  }
  if (t == 0) S.flags[s] = 0;
  const bool over = n > A.Mb;  // the host's row bound was wrong: refuse the frame
  if (over) {
    if (t == 0) { S.flags[s] = 2; res[4] = -4; }
    return;
  }
  for (int k = t; k < n; k += kStepThreads)
    kf_predict_slot(base + ord[k], S.x, S.P, S.pbox, S.gmean, S.gsinv);
  // rows_main / rows_reid in ascending track id (:478-487)
  int n1 = 0, n2 = 0;
  for (int k0 = 0; k0 < n; k0 += kStepThreads) {
    const int k = k0 + t;
    const bool v = k < n;
    const int64_t g = v ? base + ord[k] : 0;
    const bool main_row = v && S.miss[g] <= A.cfg.lost_reid_after;
    const int p1 = block_rank(main_row, s_cnt, n1);
    const int p2 = block_rank(v && !main_row, s_cnt, n2);
    if (main_row) S.row1[base + p1] = (int32_t)g;
    else if (v) S.row2[base + p2] = (int32_t)g;
  }
  if (t == 0) {
    S.m1[s] = n1;
    S.m2[s] = n2;
    res[6] = n1;
    res[7] = n2;
  }
}

// stage-1 outcome (:520-541) + unmatched detections + stage-2 inputs (:548-552)
__global__ void __launch_bounds__(kStepThreads) step_mid_kernel(const StepArgs A) {
  __shared__ int s_cnt[kStepThreads / 64];
  __shared__ uint8_t taken[kStepMaxDets];
  const trk_step_state& S = A.st;
  const int s = A.s0 + blockIdx.x;
  if (S.flags[s]) return;
  const int t = threadIdx.x;
  const int64_t cap = A.cfg.cap, base = (int64_t)s * cap, Nmax = A.cfg.Nmax;
  const int N = S.ndet[s], M1 = S.m1[s], M2 = S.m2[s];
  const int64_t fr = S.frame_id[s];
  int64_t* res = res_of(A, s);
  int64_t* mt = res + kResHdr;
  int64_t* md = mt + Nmax;
  int64_t* ut = md + Nmax;
  if (M1 > 0) {
    const int st1 = S.lsap_status[s];
    if (st1 != 0) {  // hungarian_assign raises (:519): the frame's result is the error
      if (t == 0) { S.flags[s] = 2; res[4] = st1; }
      return;
    }
  }
  for (int j = t; j < N; j += kStepThreads) taken[j] = 0;
  int nm = 0, nu = 0;
  for (int i0 = 0; i0 < M1; i0 += kStepThreads) {
    const int i = i0 + t;
    const bool v = i < M1;
    const int a = v ? A.assign[(int64_t)s * A.Mb + i] : -1;
    const int64_t g = v ? S.row1[base + i] : 0;
    const bool m = v && a >= 0;
    const int pm = block_rank(m, s_cnt, nm);
    const int pu = block_rank(v && !m, s_cnt, nu);
    if (m) {
      const int64_t e = (int64_t)s * Nmax + pm;
      S.ap_slot[e] = (int32_t)g;
      S.ap_det[e] = a;
      S.ap_kind[e] = 0;
      S.ap_cost[e] = A.C[((int64_t)s * A.Mb + i) * Nmax + a];
      S.miss[g] = 0;
      S.age[g] += 1;
      S.last_frame[g] = fr;
      mt[pm] = S.tid[g];
      md[pm] = a;
      taken[a] = 1;
    } else if (v) {
      ut[pu] = S.tid[g];
      S.miss[g] += 1;
    }
  }
  __syncthreads();
  int nud = 0;
  for (int j0 = 0; j0 < N; j0 += kStepThreads) {
    const int j = j0 + t;
    const bool f = j < N && !taken[j];
    const int p = block_rank(f, s_cnt, nud);
    if (f) S.ud[(int64_t)s * Nmax + p] = j;
  }
  __syncthreads();
  if (M2 > 0 && nud > 0) {
    // gather the unmatched detections as stage 2's detection arrays
    const int32_t* ud = S.ud + (int64_t)s * Nmax;
    for (int q = t; q < nud * 32; q += kStepThreads) {
      const int k = q >> 5, c = q & 31;
      const int64_t src = (int64_t)s * Nmax + ud[k], dst = (int64_t)s * Nmax + k;
      reinterpret_cast<float4*>(S.e2 + dst * D)[c] = reinterpret_cast<const float4*>(A.det_emb + src * D)[c];
      if (c == 0) {
        reinterpret_cast<float4*>(S.b2)[dst] = reinterpret_cast<const float4*>(A.dbox)[src];
        S.c2[dst] = A.dconf[src];
      }
    }
  } else if (M2 > 0) {  // long-lost rows with no unmatched detection: all missed (:596-598)
    for (int k = t; k < M2; k += kStepThreads) {
      const int64_t g = S.row2[base + k];
      ut[nu + k] = S.tid[g];
      S.miss[g] += 1;
    }
    nu += M2;
  }
  if (t == 0) {
    S.n2[s] = nud;
    S.m2[s] = nud > 0 ? M2 : 0;  // rows of the stage-2 problem
    S.ap_n[s] = nm;
    res[0] = nm;
    res[1] = nu;
  }
}

// stage-2 outcome (:568-595), create_new_tracks (:601), purge_dead (:604), results
__global__ void __launch_bounds__(kStepThreads) step_end_kernel(const StepArgs A) {
  __shared__ int s_cnt[kStepThreads / 64];
  __shared__ uint8_t taken[kStepMaxDets];
  const trk_step_state& S = A.st;
  const int s = A.s0 + blockIdx.x;
  const int flags = S.flags[s];
  const int t = threadIdx.x;
  // a failed frame (refused row bound, or a stage-1 solver error) leaves the live list
  // and the id counter as they were: the results block says so, so the host's live
  // count stays exact and the stream keeps running after the error
  if (flags & 2) {
    if (t == 0) {
      int64_t* res = res_of(A, s);
      res[3] = S.n_live[s];
      res[5] = S.next_id[s];
    }
    return;
  }
  const int64_t cap = A.cfg.cap, base = (int64_t)s * cap, Nmax = A.cfg.Nmax;
  int64_t* res = res_of(A, s);
  int64_t* mt = res + kResHdr;
  int64_t* md = mt + Nmax;
  int64_t* ut = md + Nmax;
  int64_t* udr = ut + cap;
  int32_t* ord = S.order + base;
  int32_t* ud = S.ud + (int64_t)s * Nmax;
  int nl = S.n_live[s];
  const int64_t next0 = S.next_id[s];
  int nb = 0, nfree = 0, nud = 0;
  if (!(flags & 1)) {
    const int M2 = S.m2[s];
    const int64_t fr = S.frame_id[s];
    int nm = (int)res[0], nu = (int)res[1];
    nud = S.n2[s];
    if (M2 > 0) {
      const int st2 = S.lsap_status[A.cfg.S + s];
      if (st2 != 0) {  // stage 1's outcome stands (the reference raises after it, :561)
        if (t == 0) { S.flags[s] = 2; res[4] = st2; res[3] = nl; res[5] = next0; }
        return;
      }
      for (int j = t; j < nud; j += kStepThreads) taken[j] = 0;
      __syncthreads();
      const int nm0 = nm;
      for (int i0 = 0; i0 < M2; i0 += kStepThreads) {
        const int i = i0 + t;
        const bool v = i < M2;
        const int a = v ? A.assign[(int64_t)s * A.Mb + i] : -1;
        const int64_t g = v ? S.row2[base + i] : 0;
        const bool m = v && a >= 0;
        const int pm = block_rank(m, s_cnt, nm);
        const int pu = block_rank(v && !m, s_cnt, nu);
        if (m) {
          const int det = ud[a];
          const int64_t e = (int64_t)s * Nmax + pm;
          S.ap_slot[e] = (int32_t)g;
          S.ap_det[e] = det;
          S.ap_kind[e] = 1;
          S.ap_cost[e] = A.C[((int64_t)s * A.Mb + i) * Nmax + a];
          S.miss[g] = 0;
          S.age[g] += 1;
          S.last_frame[g] = fr;
          mt[pm] = S.tid[g];
          md[pm] = det;
          taken[a] = 1;
        } else if (v) {
          ut[pu] = S.tid[g];
          S.miss[g] += 1;
        }
      }
      (void)nm0;
      __syncthreads();
      // unmatched_dets = [unmatched_dets[du] for du in unmatched_dets_u] (in place, stable)
      int n = 0;
      for (int k0 = 0; k0 < nud; k0 += kStepThreads) {
        const int k = k0 + t;
        const bool f = k < nud && !taken[k];
        const int j = f ? ud[k] : 0;
        const int p = block_rank(f, s_cnt, n);  // synchronises: reads above precede writes below
        if (f) ud[p] = j;
      }
      nud = n;
      __syncthreads();
    }
    if (t == 0) { res[0] = nm; res[1] = nu; }
    for (int k = t; k < nud; k += kStepThreads) udr[k] = ud[k];
    // create_new_tracks: unmatched dets with conf >= init_conf_min take the lowest free slots
    for (int q0 = 0; q0 < cap; q0 += kStepThreads) {
      const int q = q0 + t;
      const bool f = q < cap && !S.alive[base + q];
      const int p = block_rank(f, s_cnt, nfree);
      if (f) S.freelist[base + p] = q;
    }
    __syncthreads();
    for (int k0 = 0; k0 < nud; k0 += kStepThreads) {
      const int k = k0 + t;
      const bool v = k < nud;
      const int j = v ? ud[k] : 0;
      const int64_t dj = (int64_t)s * Nmax + j;
      const double conf = v ? (A.dconf64 ? A.dconf64[dj] : (double)A.dconf[dj]) : 0.0;
      const bool el = v && conf >= A.cfg.init_conf_min;
      const int p = block_rank(el, s_cnt, nb);
      if (el && p < nfree) {
        const int q = S.freelist[base + p];
        const int64_t g = base + q;
        S.alive[g] = 1;
        S.tid[g] = next0 + p;
        S.miss[g] = 0;
        S.age[g] = 1;
        S.last_frame[g] = fr;
        ord[nl + p] = q;
        const int64_t e = (int64_t)s * Nmax + nm + p;
        S.ap_slot[e] = (int32_t)g;
        S.ap_det[e] = j;
        S.ap_kind[e] = 2;
        S.ap_cost[e] = 0.f;
      }
    }
    if (t == 0) S.ap_n[s] = nm + min(nb, nfree);
    nl += min(nb, nfree);
    __syncthreads();
  }
  // purge_dead (:357-360): stable compaction of the live list
  int keep_n = 0;
  for (int k0 = 0; k0 < nl; k0 += kStepThreads) {
    const int k = k0 + t;
    const bool v = k < nl;
    const int q = v ? ord[k] : 0;
    const int64_t g = base + q;
    const bool keep = v && S.miss[g] <= A.cfg.max_age;
    const int p = block_rank(keep, s_cnt, keep_n);
    if (keep) ord[p] = q;
    else if (v) { S.alive[g] = 0; S.tid[g] = -1; }
  }
  if (t == 0) {
    S.n_live[s] = keep_n;
    S.next_id[s] = next0 + min(nb, nfree);
    res[2] = nud;
    res[3] = keep_n;
    res[5] = next0 + min(nb, nfree);
    if (nb > nfree) res[4] = -5;
  }
}

// update_matched (both stages) + new tracks: one wavefront per apply entry
__global__ void __launch_bounds__(64) step_apply_kernel(const StepArgs A) {
  const trk_step_state& S = A.st;
  const int64_t Nmax = A.cfg.Nmax;
  const int s = A.s0 + blockIdx.x / (int)Nmax;
  const int k = blockIdx.x % (int)Nmax;
  if (k >= S.ap_n[s]) return;
  const int64_t e = (int64_t)s * Nmax + k;
  const int64_t g = S.ap_slot[e];
  const int64_t d = (int64_t)s * Nmax + S.ap_det[e];
  const int kind = S.ap_kind[e];
  UpdArgs u{0, nullptr, nullptr, nullptr, nullptr, A.dbox, A.dconf, A.det_emb, S.x, S.P, S.pbox,
            S.last_conf, S.enc, S.bank, S.bank_len, S.bank_head, (int)A.cfg.T, A.cfg.ema_alpha,
            0.f, 0.f, 0.0};
  const double conf = A.dconf64 ? A.dconf64[d] : (double)A.dconf[d];
  if (kind == 2) {
    track_init_wave(u, g, d, A.dconf[d]);
  } else if (kind == 0) {  // stage 1: cost_update_max, motion gate
    track_update_wave(u, g, d, conf, true, S.ap_cost[e], A.cfg.conf_update_min, A.cfg.cost_update_max,
                      A.cfg.maha_thr);
  } else {                 // stage 2: reid_only_cost_max, no motion gate (:578-580)
    track_update_wave(u, g, d, conf, true, S.ap_cost[e], A.cfg.conf_update_min, A.cfg.reid_only_cost_max,
                      1e18);
  }
}

}  // namespace

extern "C" int trk_kf_predict(int64_t n, const int32_t* slots, double* x, double* P, float* pbox,
                              double* gmean, double* gsinv, void* stream) {
  TRK_REQUIRE(n >= 0 && n < (1 << 30), "kf_predict: bad count");
  if (n == 0) return TRK_OK;
  TRK_REQUIRE(slots && x && P && pbox && gmean && gsinv, "kf_predict: null pointer");
  hipLaunchKernelGGL(kf_predict_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), (int)n, slots, x, P, pbox, gmean, gsinv);
  return trk::check_launch("kf_predict_kernel");
}

extern "C" int trk_track_update(int64_t n, const int32_t* slots, const int32_t* dets,
                                const int64_t* cost_idx, const float* cost, const float* dbox,
                                const float* dconf, const float* demb, double* x, double* P,
                                float* pbox, float* last_conf, float* enc, float* bank,
                                int32_t* bank_len, int32_t* bank_head, int64_t T, float ema_alpha,
                                float conf_update_min, float cost_update_max, double maha_thr,
                                void* stream) {
  TRK_REQUIRE(n >= 0 && n < (1 << 30), "track_update: bad count");
  TRK_REQUIRE(T >= 1 && T <= 1024, "track_update: bad hist_max");
  if (n == 0) return TRK_OK;
  TRK_REQUIRE(slots && dets && dbox && dconf && demb && x && P && pbox && last_conf && enc && bank &&
                  bank_len && bank_head,
              "track_update: null pointer");
  TRK_REQUIRE(!cost || cost_idx, "track_update: cost without cost_idx");
  UpdArgs a{(int)n, slots, dets, cost_idx, cost, dbox, dconf, demb, x, P, pbox, last_conf, enc, bank,
            bank_len, bank_head, (int)T, ema_alpha, conf_update_min, cost_update_max, maha_thr};
  hipLaunchKernelGGL(track_update_kernel, dim3((unsigned)n), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("track_update_kernel");
}

extern "C" int trk_track_init(int64_t n, const int32_t* slots, const int32_t* dets, const float* dbox,
                              const float* dconf, const float* demb, double* x, double* P, float* pbox,
                              float* last_conf, float* enc, float* bank, int32_t* bank_len,
                              int32_t* bank_head, int64_t T, void* stream) {
  TRK_REQUIRE(n >= 0 && n < (1 << 30), "track_init: bad count");
  TRK_REQUIRE(T >= 1 && T <= 1024, "track_init: bad hist_max");
  if (n == 0) return TRK_OK;
  TRK_REQUIRE(slots && dets && dbox && dconf && demb && x && P && pbox && last_conf && enc && bank &&
                  bank_len && bank_head,
              "track_init: null pointer");
  UpdArgs a{(int)n, slots, dets, nullptr, nullptr, dbox, dconf, demb, x, P, pbox, last_conf, enc, bank,
            bank_len, bank_head, (int)T, 0.f, 0.f, 0.f, 0.0};
  hipLaunchKernelGGL(track_init_kernel, dim3((unsigned)n), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return trk::check_launch("track_init_kernel");
}

// ------------------------------------------------------------ tracker step --
namespace {

int step_check(const trk_step_state* st, const trk_step_config* cfg) {
  TRK_REQUIRE(st && cfg, "step: null state / config");
  TRK_REQUIRE(cfg->S >= 1 && cfg->cap >= 1 && cfg->cap < (1 << 24), "step: bad S / cap");
  TRK_REQUIRE(cfg->Nmax >= 1 && cfg->Nmax <= kStepMaxDets, "step: Nmax must be in [1, %d]", kStepMaxDets);
  TRK_REQUIRE(cfg->T >= 1 && cfg->T <= 1024, "step: bad hist_max");
  TRK_REQUIRE(cfg->S * cfg->cap < ((int64_t)1 << 31), "step: too many slots");
  const void* ptrs[] = {st->x, st->P, st->pbox, st->last_conf, st->gmean, st->gsinv, st->enc, st->bank,
                        st->bank_len, st->bank_head, st->alive, st->tid, st->miss, st->age, st->last_frame,
                        st->order, st->n_live, st->next_id, st->ndet, st->frame_id, st->flags, st->m1, st->row1,
                        st->m2, st->row2, st->n2, st->ud, st->freelist, st->e2, st->b2, st->c2, st->ap_n,
                        st->ap_slot, st->ap_det, st->ap_kind, st->ap_cost, st->lsap_status, st->result};
  for (const void* p : ptrs) TRK_REQUIRE(p, "step: null state pointer");
  return TRK_OK;
}

StepArgs step_args(const trk_step_state* st, const trk_step_config* cfg) {
  StepArgs a;
  memset(&a, 0, sizeof a);
  a.st = *st;
  a.cfg = *cfg;
  return a;
}

template <typename K>
int step_launch(K kernel, StepArgs a, int threads, int per_stream, hipStream_t stream, const char* what) {
  for (int64_t s0 = 0; s0 < a.cfg.S; s0 += kStepMaxStreams) {
    const int ns = (int)std::min<int64_t>(kStepMaxStreams, a.cfg.S - s0);
    a.s0 = (int)s0;
    hipLaunchKernelGGL(kernel, dim3((unsigned)(ns * per_stream)), dim3(threads), 0, stream, a);
    if (int e = trk::check_launch(what)) return e;
  }
  return TRK_OK;
}

}  // namespace

extern "C" int64_t trk_step_result_stride(int64_t cap, int64_t Nmax) { return kResHdr + 3 * Nmax + cap; }

extern "C" int trk_step_begin(const trk_step_state* st, const trk_step_config* cfg, const int32_t* host_ndet,
                              const int64_t* host_frame_id, int64_t Mb, void* stream) {
  if (int e = step_check(st, cfg)) return e;
  TRK_REQUIRE(host_ndet && host_frame_id, "step_begin: null host arrays");
  TRK_REQUIRE(Mb >= 0 && Mb <= cfg->cap, "step_begin: row bound %lld outside [0, cap]", (long long)Mb);
  StepArgs a = step_args(st, cfg);
  a.Mb = (int)Mb;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  for (int64_t s0 = 0; s0 < cfg->S; s0 += kStepMaxStreams) {
    const int ns = (int)std::min<int64_t>(kStepMaxStreams, cfg->S - s0);
    for (int q = 0; q < ns; ++q) {
      TRK_REQUIRE(host_ndet[s0 + q] >= 0 && host_ndet[s0 + q] <= cfg->Nmax,
                  "step_begin: stream %lld has %d detections (Nmax %lld)", (long long)(s0 + q),
                  host_ndet[s0 + q], (long long)cfg->Nmax);
      a.ndet[q] = host_ndet[s0 + q];
      a.frame[q] = host_frame_id[s0 + q];
    }
    a.s0 = (int)s0;
    hipLaunchKernelGGL(step_begin_kernel, dim3((unsigned)ns), dim3(kStepThreads), 0, hs, a);
    if (int e = trk::check_launch("step_begin_kernel")) return e;
  }
  return TRK_OK;
}

extern "C" int trk_step_mid(const trk_step_state* st, const trk_step_config* cfg, int64_t Mb, const float* C1,
                            const int32_t* assign1, const float* det_emb, const float* dbox, const float* dconf,
                            void* stream) {
  if (int e = step_check(st, cfg)) return e;
  TRK_REQUIRE(Mb >= 0 && Mb <= cfg->cap, "step_mid: bad row bound");
  TRK_REQUIRE(C1 && assign1 && det_emb && dbox && dconf, "step_mid: null pointer");
  StepArgs a = step_args(st, cfg);
  a.Mb = (int)Mb;
  a.C = C1;
  a.assign = assign1;
  a.det_emb = det_emb;
  a.dbox = dbox;
  a.dconf = dconf;
  return step_launch(step_mid_kernel, a, kStepThreads, 1, reinterpret_cast<hipStream_t>(stream), "step_mid_kernel");
}

extern "C" int trk_step_end(const trk_step_state* st, const trk_step_config* cfg, int64_t Mb, const float* C2,
                            const int32_t* assign2, const double* dconf64, const float* dconf, void* stream) {
  if (int e = step_check(st, cfg)) return e;
  TRK_REQUIRE(Mb >= 0 && Mb <= cfg->cap, "step_end: bad row bound");
  TRK_REQUIRE(C2 && assign2 && dconf, "step_end: null pointer");
  StepArgs a = step_args(st, cfg);
  a.Mb = (int)Mb;
  a.C = C2;
  a.assign = assign2;
  a.dconf = dconf;
  a.dconf64 = dconf64;
  return step_launch(step_end_kernel, a, kStepThreads, 1, reinterpret_cast<hipStream_t>(stream), "step_end_kernel");
}

extern "C" int trk_step_apply(const trk_step_state* st, const trk_step_config* cfg, const float* det_emb,
                              const float* dbox, const float* dconf, const double* dconf64, void* stream) {
  if (int e = step_check(st, cfg)) return e;
  TRK_REQUIRE(det_emb && dbox && dconf, "step_apply: null pointer");
  StepArgs a = step_args(st, cfg);
  a.det_emb = det_emb;
  a.dbox = dbox;
  a.dconf = dconf;
  a.dconf64 = dconf64;
  return step_launch(step_apply_kernel, a, 64, (int)cfg->Nmax, reinterpret_cast<hipStream_t>(stream),
                     "step_apply_kernel");
}
