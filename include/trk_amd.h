/*
 * trk_amd.h -- C ABI of the MI355X (gfx950) tracker hot-path library
 * (libtrk_amd.so, built from a-lightweight-unsupervised-feature-extractor-_amd/csrc).
 *
 * The reference has no FFI layer; its boundary is a set of
 * Python call signatures.  Each entry point below replaces the third-party
 * native call the reference makes at that signature, and is bound from Python
 * with ctypes (INTEGRATION.md shows the stub).  Conventions:
 *   - all pointers are DEVICE pointers unless the name says host_;
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous on
 *     it and never synchronises the device (no malloc/free inside: callers pass
 *     workspaces, so calls are hipGraph-capturable);
 *   - return 0 on success; a negative TRK_E* code otherwise, with a message in
 *     trk_last_error() (thread-local).  Argument errors are detected on the host
 *     before any launch.
 */
#ifndef TRK_AMD_H
#define TRK_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRK_ABI_VERSION 2

enum {
  TRK_OK = 0,
  TRK_EINVAL = -1,     /* bad argument (shape, dtype, null pointer)        */
  TRK_ELAUNCH = -2,    /* HIP launch / runtime error                        */
  TRK_EUNSUPPORTED = -3/* shape outside what the kernel implements          */
};

enum { TRK_F32 = 0, TRK_BF16 = 1, TRK_F64 = 2 };
enum { TRK_NCHW = 0, TRK_NHWC = 1 };

int trk_abi_version(void);
const char* trk_last_error(void);
/* Performance knobs (process-global; results are bit-identical for every value
 * unless noted; the defaults are the fastest measured in the pipelined bench):
 *   "roi_window_kb"  LDS budget (KiB) for staging a ROI's source window; 0 = never stage
 *   "roi_vec"        channels per lane in roi_align (0 = auto, 1, 2, 4)
 *   "roi_sweep"      1 (default): NHWC output through the row-sweep kernel (256 channels per
 *                    wave); 2: 512 channels per wave; 0: per-sample taps
 *   "roi_wlds"       1 (default): row sweep reads its sample weights from LDS; 0: readlanes
 *   "roi_asm"        row sweep: the bilinear sample as one asm block (same operations, same
 *                    order, bit-identical)
 *   "roi_fma"        row sweep, bf16 output only: the sample's additions fused into its
 *                    products (NOT bit-identical: within a few f32 roundings before the
 *                    bf16 rounding; f32 output is always the exact torchvision arithmetic)
 *   "dw_fast"        1 (default): 7x7/10x10 depthwise fast path; 0: generic depthwise kernel
 *   "enc_trans"      1 (default): trk_enc_transition_gemm2 with packed weights runs trans4
 *                    (weights straight into VGPRs); 0: gemm4 (weights through LDS), same sums
 *   "rf3_groups"     0 (default: CUs / 16 - 2): trk_enc_rmb_front_means workgroup pairs per XCD
 *                    (1..64; all bit-identical)
 *   "rf3_chunks"     1 (default): trk_enc_rmb_front_means as one persistent generation of
 *                    workgroups; n: n generations, each pair's ROIs in n chunks (bit-identical)
 *   "se_waves", "head_waves"  8 or 16 (default) waves per SE / head workgroup
 *   "cost_v2"        0 (default): the bank-in-registers cost3 kernel where a workspace is
 *                    given (the device tracker), else the detection-tile kernel; 1: the
 *                    LDS bank-resident cost2 kernel (all bit-identical)
 *   "cost_split"     1 (default): cost3 (trk_build_cost_dev with a workspace) computes the
 *                    bank x detection similarities from f16 hi / lo splits on the f16 MFMA
 *                    (NOT bit-identical: within 1.1e-6 of the exact f32 products for unit
 *                    rows); 0: exact f32 MFMA, bit-identical to the detection-tile kernel
 *   "lsap_dev_lds_kb" LDS budget of trk_lsap_dev workgroups (default 24: they fit beside the
 *                    encoder's workgroups instead of waiting for a whole CU) */
int trk_set_tuning(const char* key, int value);

/* ------------------------------------------------------------------------
 * ROI Align forward.  Replaces torchvision.ops.roi_align as called by
 *   MainInfer.roi_align_from_input_boxes   reference tracking.py:193-221
 *   MainInfer._roi_align_from_input_boxes  reference model/utils/inferScr/infer.py:143-170
 *   PreProcess._preprocess_roi             reference model/utils/trainingScr/trainingCard.py:24-79
 * Semantics: torchvision 0.20.1 CPU kernel, bit-exact in f32.
 *   input  [B,C,H,W] f32, layout TRK_NCHW (torchvision contract) or TRK_NHWC
 *   rois   [K,5] f32 (batch_index, x1, y1, x2, y2) in input coordinates
 *   out    [K,C,PH,PW] (TRK_NCHW, torchvision contract) or [K,PH,PW,C]
 *          (TRK_NHWC, the encoder's GEMM layout); dtype TRK_F32 or TRK_BF16
 *   workspace: >= trk_roi_align_workspace_bytes(...) bytes when the input is
 *          NCHW (the map is transposed once to NHWC so the 4-tap gathers read
 *          whole channel vectors); may be NULL for NHWC input.
 * ---------------------------------------------------------------------- */
size_t trk_roi_align_workspace_bytes(int64_t B, int64_t C, int64_t H, int64_t W, int in_layout);
/* The NCHW -> NHWC map copy that trk_roi_align_fwd makes for an NCHW input, as
 * its own call: in [B,C,H,W] f32 -> out [B,H,W,C] f32 (out may then be passed to
 * trk_roi_align_fwd as TRK_NHWC).  Lets a caller convert a frame's map ahead of
 * its ROI Align, e.g. on another stream beside the previous frame's encoder. */
int trk_nchw_to_nhwc(const float* in, int64_t B, int64_t C, int64_t H, int64_t W, float* out, void* stream);
int trk_roi_align_fwd(const float* input, int64_t B, int64_t C, int64_t H, int64_t W, int in_layout,
                      const float* rois, int64_t K, float spatial_scale,
                      int PH, int PW, int sampling_ratio, int aligned,
                      void* out, int out_dtype, int out_layout,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Association cost, batched over F frames (one frame per video stream).
 * Replaces, fused into one launch:
 *   Tracking.build_C_app_topk     reference model/mainTracking.py:141-211
 *   costCard.cal_cost/bbox_cost/conf_cost  model/utils/costTool/costCard.py:109-268
 *   Tracking.apply_kalman_gating  model/mainTracking.py:306-338 with
 *   gating_distance_maha          model/utils/costTool/KalmanFilter.py:105-116
 * Per frame f (rows i < host_M[f], dets j < host_N[f]; leading dims Mmax, Nmax;
 * host_M / host_N are HOST arrays):
 *   track data is addressed through slot = row_slot[f*Mmax+i] (or f*Mmax+i
 *   when row_slot == NULL):
 *     bank      [slot][Tmax][128] f32 unit rows (already renormalised)
 *     bank_len  [slot] int32 (<= Tmax <= 32); 0 -> C_app row of ones
 *     pbox      [slot][4] f32 KF-predicted xyxy box (mainTracking.py:340-345)
 *     conf_prev [slot] f32 last matched det conf
 *     gmean     [slot][4] f64 H x_pred;  gsinv [slot][16] f64 (H P H^T + R + 1e-9 I)^-1
 *     gate_on   [slot] int32, nonzero = apply the Mahalanobis gate to this row
 *   dets:  det_emb [f][Nmax][128] f32, dbox [f][Nmax][4] f32, conf_cur [f][Nmax] f32
 *   outputs [f][Mmax][Nmax] f32 (any may be NULL): C_total (gated), C_app,
 *     C_center, C_scale, C_conf.
 * ---------------------------------------------------------------------- */
typedef struct {
  float w_app, w_bbox, w_conf, alpha, beta; /* conf.yaml:8-12              */
  double maha_thr;                          /* conf.yaml:21 (9.49)          */
  float inf_cost;                           /* mainTracking.py:511 (1e9)    */
  int topk;                                 /* conf.yaml:4 (emb_top_k = 5)  */
  int gate;                                 /* 0 = no gating at all         */
} trk_cost_params;

int trk_build_cost(int64_t F, int64_t Mmax, int64_t Nmax, const int32_t* host_M, const int32_t* host_N,
                   const int32_t* row_slot, int64_t Tmax,
                   const float* bank, const int32_t* bank_len, const float* pbox,
                   const float* conf_prev, const double* gmean, const double* gsinv,
                   const int32_t* gate_on,
                   const float* det_emb, const float* dbox, const float* conf_cur,
                   const trk_cost_params* host_params,
                   float* C_total, float* C_app, float* C_center, float* C_scale, float* C_conf,
                   void* stream);

/* Combine-only variant for the costCard.cal_cost API (reference
 * model/utils/costTool/costCard.py:206-300), where C_app [M,N] is given:
 * C_total = w_app*C_app + w_bbox*(alpha*C_center + beta*C_scale) + w_conf*C_conf,
 * optionally Mahalanobis-gated per row (gate_on [M]).  Track arrays are [M,...],
 * detection arrays [N,...]; outputs [M,N] f32 (any may be NULL). */
int trk_cost_combine(int64_t M, int64_t N, const float* C_app, const float* pbox,
                     const float* conf_prev, const float* dbox, const float* conf_cur,
                     const double* gmean, const double* gsinv, const int32_t* gate_on,
                     const trk_cost_params* host_params, float* C_total,
                     float* C_center, float* C_scale, float* C_conf, void* stream);

/* ------------------------------------------------------------------------
 * Rectangular linear sum assignment, batched over F independent matrices.
 * Replaces scipy.optimize.linear_sum_assignment at reference
 *   model/utils/costTool/hung.py:28 (hungarian_assign, hung.py:5-45),
 * index-for-index identical (Crouse SAP, float64 duals, scipy tie rule).
 *   C       [f][ld * nr[f]] f32 or f64 (TRK_F32 / TRK_F64), row-major, row
 *           stride ld >= nc[f]; matrix f starts at C + f*batch_stride elements.
 *   rows,cols [f][kmax] int64 (kmax >= min(nr,nc)); count [f] int32 = min(nr,nc)
 *   status  [f] int32: 0 ok, -1 invalid numeric entries (NaN / -inf),
 *           -2 infeasible, -3 internal stall (a bounded wait expired: not a
 *           property of the matrix), -4 (trk_lsap_dev) shape above the launch bound
 *   If assign != NULL: assign[f][nr_max] int32 = column of row i if matched and
 *           C[i,col] <= cost_max, else -1 (hung.py:35-40's cost gate).
 *   nr, nc are HOST arrays (shapes are decided on the host).
 * One 64-lane wavefront per matrix; nc and nr up to TRK_LSAP_MAX_DIM.
 * ---------------------------------------------------------------------- */
#define TRK_LSAP_MAX_DIM 2048
int trk_lsap(int64_t F, const void* C, int dtype, int64_t ld, int64_t batch_stride,
             const int32_t* host_nr, const int32_t* host_nc, int64_t kmax,
             int64_t* rows, int64_t* cols, int32_t* count, int32_t* status,
             int32_t* assign, int64_t nr_max, double cost_max, void* stream);

/* Diagnostics: later trk_lsap / trk_lsap_dev launches write a per-matrix solver
 * cycle breakdown into buf [F][16] u64 (shader clocks: waiting for rows, scans +
 * argmin, dual updates, augmentation; iterations, total, nr, nc; then the workgroup's
 * shortcut pass, loaders + solver, outputs, total).  NULL = off. */
int trk_lsap_set_prof(unsigned long long* buf);  /* (bound to the device current at the call, like every *_set_prof) */
/* diagnostics: per-workgroup (gemm4, trans4: 8 u64 each) or per-wave (rmb_front3: [ROI][group]
 * [wave][8] u64) phase timestamps of the encoder GEMMs; NULL = off */
int trk_enc_set_prof(unsigned long long* buf);
/* trk_stream_gate enqueues on `stream` a one-wave kernel that returns once the wrapping u32
 * count *counter has reached target -- (int32_t)(*counter - target) >= 0, so targets must lie
 * within 2^31 of the count when the gate runs -- or after max_us microseconds (0..1e6) whatever
 * the count: work queued behind it on that stream starts when a front on another stream
 * (trk_enc_rmb_front_means with that counter as its `progress`) has finished `target` ROIs.  A
 * scheduling hint only (the bound makes it one); order that correctness needs still takes
 * events.  The counter lives on the device the gate is launched on. */
int trk_stream_gate(const uint32_t* counter, uint32_t target, int64_t max_us, void* stream);
/* diagnostics: per-wave timestamps of the bank-resident cost kernel; NULL = off */
int trk_cost_set_prof(unsigned long long* buf);
/* diagnostics: per-wave phase timestamps of enc_head; NULL = off */
int trk_head_set_prof(unsigned long long* buf);

/* ------------------------------------------------------------------------
 * Encoder helpers (the non-GEMM parts of encoderAndHead.Model's eval graph,
 * reference model/utils/modules/card.py:48-148, encoderAndHead.py:26-31).
 * Activations are NHWC rows [N, P = S*S, C], dtype TRK_F32 or TRK_BF16.
 * ---------------------------------------------------------------------- */
/* depthwise 5x5, stride 1, zero pad 2 (card.py:28-29,38-39 DSC depth.1/point.1):
 * in/out [N,H,W,C] (must not alias), weight tap-major [25][C] f32.  W <= 32. */
int trk_dwconv5_nhwc(const void* in, const float* weight, void* out, int64_t N, int64_t H,
                     int64_t W, int64_t C, int dtype, void* stream);
/* y = act(x) (act 0 none, 1 SiLU, 2 Hardswish), written to out (may equal x,
 * may be NULL); mean [N, C] f32 = mean over the P pixels of y.  x / out are
 * [N*P] rows of C channels with row stride ld (>= C; a column block of a wider
 * row-major buffer when ld > C). */
int trk_act_mean(const void* x, void* out, float* mean, int64_t N, int64_t P, int64_t C, int64_t ld,
                 int act, int dtype, void* stream);
/* x[n, p, c] *= s[n, c] in place (SE excitation, card.py:78). */
int trk_scale_rows(void* x, const float* s, int64_t N, int64_t P, int64_t C, int dtype, void* stream);
/* x[n,p,c] = act(x[n,p,c]) * s[n,c] in place (act as trk_act_mean): the SE
 * excitation applied to the activated DSC output without a separate
 * activation write-back (card.py:53-56 + :78). */
int trk_act_scale_rows(void* x, const float* s, int64_t N, int64_t P, int64_t C, int64_t ld, int act,
                       int dtype, void* stream);

/* ------------------------------------------------------------------------
 * Fused bf16 encoder GEMMs (RMB of reference card.py:48-148).  A rows are
 * bf16 [M, *] with M = ROIs x P pixels; weights bf16 [N][K] (conv [out, in]).
 * Per-ROI column sums are int64 fixed point (value x 2^24) PARTIALS
 * [ROIs][TRK_ENC_PARTS][ld]: entry j holds the sum over the rows of the ROI's
 * j-th 128-row M tile (j < 1 + (roi*P + P - 1)/128 - roi*P/128); entries past
 * that count are not written.  The total of a ROI is the integer sum of its
 * partials (trk_enc_sums_reduce, or inside trk_enc_se / trk_enc_head), so it
 * does not depend on tile order.  Requires 43 <= P <= 256, K % 32 == 0,
 * N % 256 == 0, 16-B aligned operands.
 *
 * trk_enc_dsc_gemm: both DSC 1x1 GEMMs (card.py:53-56, depth.2 + point.2 with
 *   eval-BN folded): Y2 [M, 2*Kg] (reinforce half | normal half), W2
 *   [2][Ng][Kg], bias [2*Ng] -> XRN [M, 2*Ng] = [SiLU(x_r) | Hardswish(x_n)],
 *   sums [ROIs][TRK_ENC_PARTS][2*Ng] = per-ROI partial sums of SiLU(x_r) (SE
 *   squeeze, card.py:75) and Hardswish(x_n) (GAP).
 * trk_enc_transition_gemm: T = [x_f * s | x_n] . Wt^T + bias (card.py:78 +
 *   :138-139) with XRN = [x_f | x_n], the SE scale s[roi] applied to the first
 *   kscale columns while staging; only the per-ROI sums of SiLU(T) are
 *   produced (partials [ROIs][TRK_ENC_PARTS][N]); T is never stored.
 * ---------------------------------------------------------------------- */
#define TRK_ENC_PARTS 3
/* out[roi][c] = (float)(sum_j part[roi][j][c] * 2^-24) for the partial sums above. */
int trk_enc_sums_reduce(const long long* part, int64_t R, int64_t P, int64_t ld, float* out, void* stream);
/* trk_enc_g1_dwconv: the four first 1x1 convs of the RMB as one GEMM (card.py:28,38;
 *   X [M][512] . W1^T, W1 [N][512]) followed by the 1024-channel depthwise 5x5
 *   (card.py:29,39) in one kernel for 10x10 ROIs (M = ROIs x 100):
 *   Y2 = dwconv5(bf16(X . W1^T)) with weights tap-major [25][N] f32; Y1 never
 *   reaches HBM. */
int trk_enc_g1_dwconv(const void* X, int64_t M, const void* W1, int64_t N, const float* wdw, void* Y2,
                      void* stream);
int trk_enc_dsc_gemm(const void* Y2, int64_t M, int64_t P, int64_t Kg, const void* W2, const float* bias,
                     int64_t Ng, void* XRN, long long* sums, void* stream);
/* trk_enc_rmb_front_means: trk_enc_g1_dwconv followed by trk_enc_dsc_gemm in ONE kernel
 *   for 10x10 ROIs of C = 512 channels (M = ROIs x 100, 4h = 1024, Ng = Kg = 512;
 *   card.py:28-57), writing the SE squeeze means instead of the int64 sums: a persistent
 *   grid whose workgroups each run one DSC (reinforce or normal) of their ROIs with Y1 and
 *   Y2 kept in LDS, so Y2 never reaches HBM.  Weights in MFMA fragment order: W1p = W1
 *   [1024][512] and W2p = W2 [2][512][512] each as [2 groups][16 k steps][32 col tiles]
 *   [64 lanes][8] bf16, element (g, s, n, l, j) = W[g*512 + 16n + (l % 16)][32 s + 8 (l / 16)
 *   + j] (trk.ops.enc_pack_fragments); wdw [25][1024] f32, bias [1024] f32 (BN-folded).
 *   XRN [M][1024] is bit-identical to the two-kernel path; m_r = mean SiLU(x_r), m_n = mean
 *   Hardswish(x_n) [R][512] f32 as trk_enc_se computes them from int64 sums, of the kernel's
 *   own f32 column sums.  Pair with trk_enc_se_means.
 *   progress (may be NULL): one u32 in device memory on the launch's device, owned by the
 *   caller; the launch adds 1 to it (relaxed, device scope) for every ROI it finishes, so a
 *   trk_stream_gate on another stream can start work before the whole front is done.  The
 *   count wraps at 2^32; the library keeps no pointer after the call. */
int trk_enc_rmb_front_means(const void* X, int64_t M, const void* W1p, const float* wdw, const void* W2p,
                            const float* bias, void* XRN, float* m_r, float* m_n, uint32_t* progress,
                            void* stream);
int trk_enc_transition_gemm(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s, int64_t kscale,
                            const void* Wt, const float* bias, int64_t N, long long* sums, void* stream);
/* trk_enc_transition_gemm2: the same, also given Wtp = Wt [512][1024] in MFMA fragment order
 *   ([32 k steps][32 col tiles][64 lanes][8] bf16, trk.ops.enc_pack_fragments_k; may be NULL).
 *   Wtp requires K = 1024, N = 512, kscale = 512 (else TRK_EINVAL); with it and
 *   trk_set_tuning("enc_trans", 1) the weights are read straight into registers (trans4
 *   kernel) instead of through LDS; the sums are bit-identical either way. */
int trk_enc_transition_gemm2(const void* XRN, int64_t M, int64_t P, int64_t K, const float* s, int64_t kscale,
                             const void* Wt, const void* Wtp, const float* bias, int64_t N, long long* sums,
                             void* stream);
/* Per-ROI tail of the encoder (f32, 16 ROIs per workgroup, f32-input MFMA).
 * trk_enc_se: squeeze means and SE excitation (card.py:59-78) from the partial
 *   sums of trk_enc_dsc_gemm ([R][TRK_ENC_PARTS][ld_sums], ld_sums >= 2C: C sums
 *   of SiLU(x_r), then C of Hardswish(x_n)): m_r, m_n [R][C] = (float)(sum *
 *   2^-24) / P;
 *   s [R][C] = hardsigmoid(w2 . relu(w1 . m_r + b1) + b2), w1 [H][C], w2 [C][H].
 * trk_enc_head: g = 0.5 m_cat + 0.5 (alpha (s m_r) + (1 - alpha) m_n) (Shake2
 *   eval + GAP, card.py:83-96, :128-148; m_cat from the trk_enc_transition_gemm
 *   partials [R][TRK_ENC_PARTS][C]) -> ProjectionHead (card.py:151-169): out [R][D] =
 *   normalize(w4 . silu(LayerNorm(w0 . g; ln_w, ln_b, ln_eps)) + b4), w0 [C][C],
 *   w4 [D][C].  Replaces ~25 small torch launches between and after the GEMMs.
 * Weight layout (w1, w2, w0, w4; also trk_enc_se_means): an [N][K] f32 weight is passed in
 *   fragment order, [N/16][K/16][64][4] with element [t][kb][16 g + r][e] = W[16 t + r][16 kb +
 *   4 g + e] (ops.enc_pack_rows), so each load reads 1 KiB contiguous; the bias vectors are
 *   plain.  (Row-major weights are not detected: they give wrong results.)
 * C, H, D multiples of 16, <= 1024; P <= 256. */
int trk_enc_se(const long long* sums, int64_t R, int64_t ld_sums, int64_t P, int64_t C, const float* w1,
               const float* b1, int64_t H, const float* w2, const float* b2, float* m_r, float* m_n, float* s,
               void* stream);

/* trk_enc_se's excitation from given squeeze means: s = hardsigmoid(W2 relu(W1 m_r + b1) + b2)
 * [R][C] f32, bit-identical to trk_enc_se's s for the same m_r (card.py:59-78). */
int trk_enc_se_means(const float* m_r, int64_t R, int64_t C, const float* w1, const float* b1, int64_t H,
                     const float* w2, const float* b2, float* s, void* stream);
int trk_enc_head(const long long* tsums, int64_t R, int64_t P, int64_t C, const float* s, const float* m_r,
                 const float* m_n, double alpha, const float* w0, const float* ln_w, const float* ln_b,
                 float ln_eps, const float* w4, const float* b4, int64_t D, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Device-resident track state.  Track slots of all
 * streams share one set of slot arrays:
 *   x [S][8] f64, P [S][64] f64           Kalman state (float64 throughout)
 *   pbox [S][4] f32, last_conf [S] f32     mem.last_bbox / mem.last_conf
 *   gmean [S][4] f64, gsinv [S][16] f64    gate inputs (see trk_build_cost)
 *   enc [S][128] f32                       mem.encoder_feat (EMA, unit)
 *   bank [S][T][128] f32, bank_len [S], bank_head [S]   mem.feat_historical ring
 * Detection arrays are indexed by a global detection row d: dbox [d][4],
 * dconf [d], demb [d][128].
 * ---------------------------------------------------------------------- */
/* Tracking.predict_all (reference model/mainTracking.py:340-345): x = F x,
 * P = F P F^T + Q for each listed slot; pbox = x_to_bbox_xyxy(x)
 * (KalmanFilter.py:19-33); gmean/gsinv for the Mahalanobis gate. */
int trk_kf_predict(int64_t n, const int32_t* slots, double* x, double* P, float* pbox,
                   double* gmean, double* gsinv, void* stream);
/* Tracking.update_matched (mainTracking.py:375-448) for n matched (slot, det)
 * pairs: filterpy update (Joseph form), last_bbox/last_conf, then -- if
 * conf >= conf_update_min, cost[cost_idx] <= cost_update_max (cost may be NULL)
 * and the post-update Mahalanobis d2 <= maha_thr -- the EMA feature update and
 * the bank push (ring of T = hist_max). */
int trk_track_update(int64_t n, const int32_t* slots, const int32_t* dets,
                     const int64_t* cost_idx, const float* cost, const float* dbox,
                     const float* dconf, const float* demb, double* x, double* P,
                     float* pbox, float* last_conf, float* enc, float* bank,
                     int32_t* bank_len, int32_t* bank_head, int64_t T, float ema_alpha,
                     float conf_update_min, float cost_update_max, double maha_thr,
                     void* stream);
/* Tracking.create_new_tracks / creat_item / init_kf_from_bbox
 * (mainTracking.py:99-140,362-373, KalmanFilter.py:36-101) for n (slot, det). */
int trk_track_init(int64_t n, const int32_t* slots, const int32_t* dets, const float* dbox,
                   const float* dconf, const float* demb, double* x, double* P, float* pbox,
                   float* last_conf, float* enc, float* bank, int32_t* bank_len,
                   int32_t* bank_head, int64_t T, void* stream);

/* ------------------------------------------------------------------------
 * Device-resident tracker step (Tracking.update, reference
 * model/mainTracking.py:450-610, for S streams at once) with NO host
 * round trip inside a frame: the per-track bookkeeping the reference keeps in
 * Python dicts (ids, miss counts, ages, the main / ReID-only row split, the
 * cost_max gate outcome, births with fresh ids, purge) lives in HBM next to
 * the Kalman state and memory bank, and every decision is made by a kernel.
 * A frame is this launch sequence on one stream (sizes are read from device
 * memory, so the host never waits on a frame):
 *   trk_step_begin   N == 0 frames (:467-471); predict_all (:474-475); row split (:478-487)
 *   trk_build_cost_dev + trk_lsap_dev     stage 1 (gated C_total, cost_max)  (:493-523)
 *   trk_step_mid     stage-1 matches / misses (:525-541); unmatched dets; stage-2 inputs (:548-552)
 *   trk_build_cost_dev + trk_lsap_dev     stage 2 (C_app, reid_only_cost_max) (:555-566)
 *   trk_step_end     stage-2 matches / misses (:568-595); create_new_tracks (:601, :362-373);
 *                    purge_dead (:604, :357-360); the frame's results
 *   trk_step_apply   update_matched's KF update / EMA / bank push (:375-448) for both stages
 *                    and the new tracks' init (creat_item, init_kf_from_bbox), one wave each
 * Results per stream s: result[s * trk_step_result_stride(cap, Nmax) + ...] int64:
 *   [0] n_match [1] n_unmatched_tracks [2] n_unmatched_dets [3] n_live [4] status
 *   (0 ok, -1 invalid cost entries, -2 infeasible, -3 solver stall, -4 launch bound
 *   exceeded, -5 track capacity exhausted) [5] next_id [6] stage-1 rows [7] stage-2 rows,
 *   then match_tid[Nmax], match_det[Nmax], unmatched_tid[cap], unmatched_det[Nmax],
 *   each in the reference's return order.
 * Slot g of stream s is s * cap + local slot.  Row bound Mb (host): an upper bound
 * of every stream's live-track count this frame (<= cap), the row stride of the
 * stage cost matrices [S][Mb][Nmax] and of the assignment arrays [S][Mb].
 * ---------------------------------------------------------------------- */
typedef struct {
  /* Kalman state and memory (the trk_track_update arrays), [S * cap] slots */
  double* x; double* P; float* pbox; float* last_conf; double* gmean; double* gsinv;
  float* enc; float* bank; int32_t* bank_len; int32_t* bank_head;
  /* bookkeeping, [S * cap] */
  int32_t* alive; int64_t* tid; int32_t* miss; int32_t* age; int64_t* last_frame;
  /* per stream: live local slots in ascending track id [S][cap], counts [S] */
  int32_t* order; int32_t* n_live; int64_t* next_id;
  /* per-frame scratch */
  int32_t* ndet;      /* [S] detections this frame                          */
  int64_t* frame_id;  /* [S]                                                 */
  int32_t* flags;     /* [S] bit 0: frame without detections, bit 1: failed  */
  int32_t* m1; int32_t* row1;   /* [S], [S][cap] stage-1 rows (global slots)   */
  int32_t* m2; int32_t* row2;   /* [S], [S][cap] stage-2 rows                  */
  int32_t* n2; int32_t* ud;     /* [S], [S][Nmax] unmatched dets after stage 1 */
  int32_t* freelist;            /* [S][cap]                                    */
  float* e2; float* b2; float* c2;  /* [S][Nmax][128] / [4] / [1] stage-2 detections */
  int32_t* ap_n; int32_t* ap_slot; int32_t* ap_det; int32_t* ap_kind; float* ap_cost; /* [S], [S][Nmax] */
  int32_t* lsap_status;         /* [2][S] status of the two LSAP launches       */
  int64_t* result;              /* [S][trk_step_result_stride]                 */
} trk_step_state;

typedef struct {
  int64_t S, cap, Nmax, T;      /* streams, slots per stream, detection stride, hist_max */
  int lost_reid_after, max_age; /* conf.yaml tracker section                   */
  double init_conf_min, conf_update_min, cost_update_max, reid_only_cost_max, maha_thr;
  float ema_alpha;              /* compared / mixed as the reference's Python floats */
} trk_step_config;

int64_t trk_step_result_stride(int64_t cap, int64_t Nmax);
/* host_ndet [S], host_frame_id [S]: this frame's detection counts and ids (HOST
 * arrays, copied into the launch); Mb: the row bound of this frame. */
int trk_step_begin(const trk_step_state* st, const trk_step_config* cfg, const int32_t* host_ndet,
                   const int64_t* host_frame_id, int64_t Mb, void* stream);
/* C1 [S][Mb][Nmax] gated C_total of stage 1, assign1 [S][Mb] (trk_lsap_dev with
 * cost_max); det arrays [S][Nmax][...] of the frame. */
int trk_step_mid(const trk_step_state* st, const trk_step_config* cfg, int64_t Mb, const float* C1,
                 const int32_t* assign1, const float* det_emb, const float* dbox, const float* dconf,
                 void* stream);
/* C2 [S][Mb][Nmax] stage-2 C_app, assign2 [S][Mb]; dconf64 [S][Nmax] f64 (the
 * detections' confidences as the caller's floats, for the creation / appearance
 * gates; NULL: dconf widened). */
int trk_step_end(const trk_step_state* st, const trk_step_config* cfg, int64_t Mb, const float* C2,
                 const int32_t* assign2, const double* dconf64, const float* dconf, void* stream);
int trk_step_apply(const trk_step_state* st, const trk_step_config* cfg, const float* det_emb,
                   const float* dbox, const float* dconf, const double* dconf64, void* stream);
/* trk_build_cost / trk_lsap with the per-frame sizes read from DEVICE arrays
 * (dev_M / dev_N, dev_nr / dev_nc); Mmax / nr_bound / nc_bound are host upper
 * bounds that size the launch (a larger device size is an error: status -4 for
 * the solver, rows past Mmax are not computed by the cost).  row_slot has row
 * stride rs_ld.  work: device scratch of trk_cost_work_bytes(F, Nmax) bytes, 16-B
 * aligned (the renormalised detections in MFMA fragment order, whole 32-detection
 * tiles per frame, and their box / conf / KF terms; the bank then is read once per
 * launch instead of once per 32-detection tile), or NULL.  Its contents are private
 * to the call (only its size is part of the interface). */
int64_t trk_cost_work_bytes(int64_t F, int64_t Nmax);
int trk_build_cost_dev(int64_t F, int64_t Mmax, int64_t Nmax, const int32_t* dev_M, const int32_t* dev_N,
                       const int32_t* row_slot, int64_t rs_ld, int64_t Tmax, const float* bank,
                       const int32_t* bank_len, const float* pbox, const float* conf_prev, const double* gmean,
                       const double* gsinv, const int32_t* gate_on, const float* det_emb, const float* dbox,
                       const float* conf_cur, const trk_cost_params* host_params, float* C_total, float* C_app,
                       void* work, void* stream);
int trk_lsap_dev(int64_t F, const void* C, int dtype, int64_t ld, int64_t batch_stride, const int32_t* dev_nr,
                 const int32_t* dev_nc, int64_t nr_bound, int64_t nc_bound, int64_t kmax, int64_t* rows,
                 int64_t* cols, int32_t* count, int32_t* status, int32_t* assign, int64_t nr_max, double cost_max,
                 void* stream);

/* ------------------------------------------------------------------------
 * Detector-side boundary.
 *
 * YOLOv7 post-processing as YoloDetects.run_with_tensor applies it
 * (reference model/yolov7/yoloDetects2.py:111-160) to the raw head output
 * pred [B][A][no] f32 (no = 5 + nc: cx, cy, w, h, obj, cls...):
 *   cand_count[b] = #(obj > conf_thres)              yoloDetects2.py:124-125
 *   if cand_count < cand_gate: no detections          :127-129
 *   else non_max_suppression(pred, conf_thres, iou_thres)  general.py:608-700
 *        (defaults: best class only, class-offset batched NMS with
 *        max_wh 4096 unless agnostic, torchvision nms, first max_det kept)
 *   det[b][k] = (x1, y1, x2, y2, conf, cls) in input (letterbox) pixels,
 *   k < det_count[b], in keep order (descending conf).
 *   xywh (optional, may be NULL): scale_coords(img1, det, img0).round() then
 *   xyxy2xywh (general.py:320-341, :255-262), with host_scale = {gain, pad_w,
 *   pad_h, img0_w, img0_h} (the Python doubles of scale_coords; HOST array).
 * workspace: >= trk_det_workspace_bytes(B, A), 16-B aligned; B <= 32.
 * Numerics: the reference CPU path (torch CPU kernels; torchvision 0.20.1 CPU
 * nms with its stable descending score sort), bit-exact.
 * ---------------------------------------------------------------------- */
size_t trk_det_workspace_bytes(int64_t B, int64_t A);
int trk_det_nms(const float* pred, int64_t B, int64_t A, int64_t no, float conf_thres, double iou_thres,
                int max_det, int max_nms, int agnostic, int cand_gate, float* det, int32_t* det_count,
                int32_t* cand_count, const float* host_scale, float* xywh, void* workspace,
                size_t workspace_bytes, void* stream);
/* PreProcess._preprocess_roi box preparation (reference
 * model/utils/trainingScr/trainingCard.py:24-79): boxes [N][4] image xyxy ->
 * rois [N][5] = (0, x1, y1, x2, y2) in feature pixels (sorted corners, scale
 * Wf/img_w and Hf/img_h, clamp to [0, W-1], minimum size enforce_min_size if
 * > 0), for trk_roi_align_fwd with spatial_scale = 1. */
int trk_train_rois(const float* boxes, int64_t N, int64_t Hf, int64_t Wf, double img_h, double img_w,
                   float enforce_min_size, float* rois, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TRK_AMD_H */
