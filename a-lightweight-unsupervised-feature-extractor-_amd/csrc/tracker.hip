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

// 4x4 inverse, Gauss-Jordan with partial pivoting (f64)
__device__ inline void inv4(const double* A, double* out) {
  double m[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      m[r][c] = A[r * 4 + c];
      m[r][c + 4] = r == c ? 1.0 : 0.0;
    }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r)
      if (fabs(m[r][c]) > fabs(m[p][c])) p = r;
    if (p != c)
      for (int k = 0; k < 8; ++k) { double t = m[c][k]; m[c][k] = m[p][k]; m[p][k] = t; }
    const double d = m[c][c];
    for (int k = 0; k < 8; ++k) m[c][k] /= d;
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double fct = m[r][c];
      for (int k = 0; k < 8; ++k) m[r][k] -= fct * m[c][k];
    }
  }
  for (int r = 0; r < 4; ++r)
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

__global__ void __launch_bounds__(64)
kf_predict_kernel(int n, const int32_t* __restrict__ slots, double* __restrict__ X,
                  double* __restrict__ PP, float* __restrict__ pbox, double* __restrict__ gmean,
                  double* __restrict__ gsinv) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t s = slots[t];
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

// one wavefront per matched pair: lane 0 runs the 8-D filter, the wave does
// the 128-D appearance update (2 dims per lane)
__global__ void __launch_bounds__(64)
track_update_kernel(const UpdArgs A) {
  const int t = blockIdx.x;
  const int lane = threadIdx.x;
  if (t >= A.n) return;
  const int64_t s = A.slots[t], d = A.dets[t];
  __shared__ int s_push;
  if (lane == 0) {
    double* x = A.X + s * 8;
    double* P = A.P + s * 64;
    double z[4];
    box_to_z(A.dbox + d * 4, z);
    // filterpy KalmanFilter.update (R = I, H = [I4 | 0]):
    double y[4], S[16], SI[16], K[32];
    for (int r = 0; r < 4; ++r) y[r] = z[r] - x[r];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) S[r * 4 + c] = P[r * 8 + c] + (r == c ? 1.0 : 0.0);
    inv4(S, SI);
    for (int r = 0; r < 8; ++r)  // K = P H^T S^-1
      for (int c = 0; c < 4; ++c) {
        double v = 0.0;
        for (int k = 0; k < 4; ++k) v += P[r * 8 + k] * SI[k * 4 + c];
        K[r * 4 + c] = v;
      }
    for (int r = 0; r < 8; ++r) {
      double v = 0.0;
      for (int k = 0; k < 4; ++k) v += K[r * 4 + k] * y[k];
      x[r] = x[r] + v;
    }
    // P = (I - K H) P (I - K H)^T + K R K^T
    double IKH[64], T1[64];
    for (int r = 0; r < 8; ++r)
      for (int c = 0; c < 8; ++c) IKH[r * 8 + c] = (r == c ? 1.0 : 0.0) - (c < 4 ? K[r * 4 + c] : 0.0);
    for (int r = 0; r < 8; ++r)
      for (int c = 0; c < 8; ++c) {
        double v = 0.0;
        for (int k = 0; k < 8; ++k) v += IKH[r * 8 + k] * P[k * 8 + c];
        T1[r * 8 + c] = v;
      }
    for (int r = 0; r < 8; ++r)
      for (int c = 0; c < 8; ++c) {
        double v = 0.0;
        for (int k = 0; k < 8; ++k) v += T1[r * 8 + k] * IKH[c * 8 + k];
        double kk = 0.0;
        for (int k = 0; k < 4; ++k) kk += K[r * 4 + k] * K[c * 4 + k];
        P[r * 8 + c] = v + kk;
      }
    // last_* fields (update_matched :402-405)
    const float* b = A.dbox + d * 4;
    float* pb = A.pbox + s * 4;
    for (int k = 0; k < 4; ++k) pb[k] = b[k];
    const float conf = A.dconf[d];
    A.last_conf[s] = conf;
    // appearance-update gates (:417-426): conf, matched cost, post-update d2
    int push = 1;
    if (conf < A.conf_update_min) push = 0;
    if (push && A.cost && (double)A.cost[A.cost_idx[t]] > (double)A.cost_update_max) push = 0;
    if (push) {
      double gm[4], gs[16];
      gate_params(x, P, gm, gs);
      if (maha(z, gm, gs) > A.maha_thr) push = 0;
    }
    s_push = push;
  }
  __syncthreads();
  if (!s_push) return;
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
  __syncthreads();
  if (lane == 0) {
    A.bank_head[s] = (head + 1) % A.T;
    A.bank_len[s] = min(A.bank_len[s] + 1, A.T);
  }
}

// new track from one detection (creat_item + init_kf_from_bbox)
__global__ void __launch_bounds__(64)
track_init_kernel(UpdArgs A) {
  const int t = blockIdx.x;
  const int lane = threadIdx.x;
  if (t >= A.n) return;
  const int64_t s = A.slots[t], d = A.dets[t];
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
    A.last_conf[s] = A.dconf[d];
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
