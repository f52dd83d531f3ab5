// The detector-side boundary of the ROI path on gfx950:
//
//   trk_det_nms     YOLOv7 post-processing as YoloDetects.run_with_tensor uses it
//                   (reference model/yolov7/yoloDetects2.py:111-160): the cand_gate
//                   count (:124-127), non_max_suppression with its defaults
//                   (model/yolov7/utils/general.py:608-700: single best class,
//                   class-offset batched NMS, max_det 300, max_nms 30000), and
//                   scale_coords (:320-341) + xyxy2xywh (:255-262) for the boxes the
//                   tracker reports in original-frame pixels.
//   trk_train_rois  the training-side ROI boxes of PreProcess._preprocess_roi
//                   (model/utils/trainingScr/trainingCard.py:24-79): sorted corners,
//                   per-axis image->feature scale, clamp to [0, W-1], minimum size;
//                   followed by trk_roi_align_fwd with spatial_scale 1.
//
// Float semantics follow the reference's CPU path (torch CPU kernels, torchvision
// 0.20.1's CPU nms): scalar operands are rounded to f32 first, comparisons
// against Python floats are made in the tensor dtype, except torchvision's
// `ovr > iou_threshold`, whose threshold is a C++ double.  Built with
// -ffp-contract=off and correctly rounded division (Makefile).
//
// NMS on the GPU, per image:
//   det_filter_kernel  one thread per anchor: objectness gate (+ the cand_gate
//                      count as one atomic per wave), best class of obj * cls,
//                      xywh -> xyxy, conf gate; a survivor writes its row at its
//                      anchor slot and a sort key (~conf bits, anchor) to a
//                      compacted list.  Slot order is nondeterministic; the key is
//                      not, and it orders exactly as torchvision's stable
//                      descending sort of the anchor-ordered candidates.
//   det_nms_kernel     one workgroup: bitonic sort of the keys (LDS up to 8192
//                      candidates, the workspace above), then greedy NMS by one
//                      wave in chunks of 64 candidates: each lane tests its
//                      candidate against the kept list in LDS, then the chunk's
//                      survivors are resolved in score order with ballots.  Kept
//                      boxes are final (a later box can never remove an earlier
//                      one), so the scan stops at max_det kept boxes -- the
//                      reference truncates to max_det after NMS.
#include "trk_common.h"

namespace {

constexpr int kMaxWh = 4096;           // general.py:622 (class offset of batched NMS)
constexpr int kSortLds = 8192;         // candidates sorted in LDS (64 KiB of keys)
constexpr int kNmsThreads = 1024;
constexpr int kMaxDetCap = 1024;       // kept-list capacity in LDS

// torch / std semantics of the scalar helpers the reference's kernels use
__device__ __forceinline__ float std_max(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float std_min(float a, float b) { return (b < a) ? b : a; }
// torch.minimum / maximum / clamp propagate NaN
__device__ __forceinline__ float t_minimum(float a, float b) { return (a != a || b != b) ? __int_as_float(0x7fc00000) : (a < b ? a : b); }
__device__ __forceinline__ float t_maximum(float a, float b) { return (a != a || b != b) ? __int_as_float(0x7fc00000) : (a > b ? a : b); }
__device__ __forceinline__ float t_clamp(float x, float lo, float hi) { return x != x ? x : (x < lo ? lo : (x > hi ? hi : x)); }

struct DetArgs {
  const float* pred;      // [B][A][no]
  int64_t A;
  int no, nc;
  float conf_thres;       // f32, as the tensor comparisons round it
  double iou_thres;       // double, as torchvision's nms compares
  int max_det, max_nms, agnostic, cand_gate;
  int apad;               // keys per image (power of two >= A)
  int* cnt;               // [B][2]: survivors, candidates (obj > conf)
  unsigned long long* keys;   // [B][apad]
  float* rows;            // [B][A][6]  x1 y1 x2 y2 conf cls, at the anchor's slot
  float* det;             // [B][max_det][6]
  int32_t* det_count;     // [B]
  int32_t* cand_count;    // [B] (may be null)
  // scale_coords + xyxy2xywh (xywh == nullptr: skipped)
  float gain, pad_w, pad_h, clip_w, clip_h;
  float* xywh;            // [B][max_det][4]
};

__global__ void __launch_bounds__(256) det_filter_kernel(DetArgs a) {
  const int b = blockIdx.y;
  const int64_t an = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool cand = false;
  if (an < a.A) {
    const float* row = a.pred + ((int64_t)b * a.A + an) * a.no;
    const float obj = row[4];
    cand = obj > a.conf_thres;                                   // general.py:617
    if (cand) {
      // x[:, 5:] = x[:, 4:5] (nc == 1) or x[:, 5:] *= x[:, 4:5]; then .max(1): first maximum,
      // NaN wins (and then fails the conf gate)
      float best = a.nc == 1 ? obj : row[5] * obj;
      int bj = 0;
      bool nan = best != best;
      for (int c = 1; c < a.nc; ++c) {
        const float v = row[5 + c] * obj;
        if (v != v) nan = true;
        else if (v > best) { best = v; bj = c; }
      }
      if (!nan && best > a.conf_thres) {                          // general.py:657
        const float cx = row[0], cy = row[1], w = row[2], h = row[3];
        float* o = a.rows + ((int64_t)b * a.A + an) * 6;
        o[0] = cx - w / 2.0f;                                      // xywh2xyxy, general.py:265-272
        o[1] = cy - h / 2.0f;
        o[2] = cx + w / 2.0f;
        o[3] = cy + h / 2.0f;
        o[4] = best;
        o[5] = (float)bj;
        const int slot = atomicAdd(&a.cnt[2 * b], 1);
        // ascending key == descending conf (positive floats order as their bits), ties by anchor
        a.keys[(int64_t)b * a.apad + slot] =
            ((unsigned long long)(0xffffffffu - __float_as_uint(best)) << 32) | (unsigned long long)an;
      }
    }
  }
  const unsigned long long bal = __ballot(cand);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(&a.cnt[2 * b + 1], (int)__popcll(bal));
}

// bitonic sort of n (power of two) keys at p, by the whole workgroup
__device__ void bitonic(unsigned long long* p, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long x = p[i], y = p[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { p[i] = y; p[l] = x; }
        }
      }
      __syncthreads();
    }
  }
}

// torchvision CPU nms overlap test (nms_kernel.cpp): i is the earlier (kept) box
__device__ __forceinline__ bool suppresses(const float4 bi, float ai, const float4 bj, float aj, double thr) {
  const float xx1 = std_max(bi.x, bj.x), yy1 = std_max(bi.y, bj.y);
  const float xx2 = std_min(bi.z, bj.z), yy2 = std_min(bi.w, bj.w);
  const float w = std_max(0.0f, xx2 - xx1), h = std_max(0.0f, yy2 - yy1);
  const float inter = w * h;
  const float ovr = inter / (ai + aj - inter);
  return (double)ovr > thr;
}

__global__ void __launch_bounds__(kNmsThreads) det_nms_kernel(DetArgs a) {
  __shared__ unsigned long long skeys[kSortLds];
  __shared__ float4 kbox[kMaxDetCap];
  __shared__ float karea[kMaxDetCap];
  __shared__ int kanchor[kMaxDetCap];
  const int b = blockIdx.x;
  const int n = a.cnt[2 * b];
  const int ncand = a.cnt[2 * b + 1];
  if (a.cand_count && threadIdx.x == 0) a.cand_count[b] = ncand;
  // cand_gate (yoloDetects2.py:124-127): too few candidates -> no NMS, no detections
  if (n == 0 || ncand < a.cand_gate) {
    if (threadIdx.x == 0) a.det_count[b] = 0;
    return;
  }
  int npad = 1;
  while (npad < n) npad <<= 1;
  unsigned long long* keys = a.keys + (int64_t)b * a.apad;
  unsigned long long* sk = npad <= kSortLds ? skeys : keys;
  for (int i = threadIdx.x; i < npad; i += blockDim.x) sk[i] = i < n ? keys[i] : ~0ull;
  __syncthreads();
  bitonic(sk, npad);
  const int m = min(n, a.max_nms);                                 // general.py:671-672
  if (threadIdx.x >= 64) return;                                   // NMS: one wave
  const int lane = threadIdx.x;
  const float* rows = a.rows + (int64_t)b * a.A * 6;
  int nk = 0;
  for (int s = 0; s < m && nk < a.max_det; s += 64) {
    const int c = s + lane;
    bool alive = c < m;
    float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
    float ar = 0.f;
    int anc = 0;
    if (alive) {
      anc = (int)(sk[c] & 0xffffffffull);
      const float* r = rows + (int64_t)anc * 6;
      // boxes + class offset (general.py:675-676): c = cls * 4096 in f32, then the f32 add
      const float co = a.agnostic ? 0.0f : r[5] * (float)kMaxWh;
      bx = make_float4(r[0] + co, r[1] + co, r[2] + co, r[3] + co);
      ar = (bx.z - bx.x) * (bx.w - bx.y);                         // areas_t
      for (int k = 0; k < nk && alive; ++k)
        if (suppresses(kbox[k], karea[k], bx, ar, a.iou_thres)) alive = false;
    }
    unsigned long long mask = __ballot(alive);
    while (mask && nk < a.max_det) {
      const int i = __ffsll((long long)mask) - 1;
      const float4 bi = make_float4(__shfl(bx.x, i), __shfl(bx.y, i), __shfl(bx.z, i), __shfl(bx.w, i));
      const float ai = __shfl(ar, i);
      const int anci = __shfl(anc, i);
      if (lane == 0) { kbox[nk] = bi; karea[nk] = ai; kanchor[nk] = anci; }
      ++nk;
      if (lane > i && alive && suppresses(bi, ai, bx, ar, a.iou_thres)) alive = false;
      if (lane == i) alive = false;
      mask = __ballot(alive);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_wave_barrier();
  // outputs in keep order: x[i] rows (un-offset boxes), then scale_coords + xyxy2xywh
  for (int k = lane; k < nk; k += 64) {
    const float* r = rows + (int64_t)kanchor[k] * 6;
    float* o = a.det + ((int64_t)b * a.max_det + k) * 6;
#pragma unroll
    for (int e = 0; e < 6; ++e) o[e] = r[e];
    if (a.xywh) {
      float c4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = r[e] - ((e & 1) ? a.pad_h : a.pad_w);            // coords[:, [0,2]] -= pad[0] ...
        v = v / a.gain;                                            // coords[:, :4] /= gain
        v = t_clamp(v, 0.0f, (e & 1) ? a.clip_h : a.clip_w);       // clip_coords
        c4[e] = rintf(v);                                          // .round(): half to even
      }
      float* q = a.xywh + ((int64_t)b * a.max_det + k) * 4;
      q[0] = (c4[0] + c4[2]) / 2.0f;
      q[1] = (c4[1] + c4[3]) / 2.0f;
      q[2] = c4[2] - c4[0];
      q[3] = c4[3] - c4[1];
    }
  }
  if (lane == 0) a.det_count[b] = nk;
}

__global__ void __launch_bounds__(256) zero_i32_kernel(int* p, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0;
}

__global__ void __launch_bounds__(256) train_rois_kernel(const float* __restrict__ boxes, int64_t N, float sx,
                                                         float sy, float wmax, float hmax, float min_size,
                                                         float* __restrict__ rois) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const float* bx = boxes + i * 4;
  // sort coords (trainingCard.py:46-50)
  float x1 = t_minimum(bx[0], bx[2]), y1 = t_minimum(bx[1], bx[3]);
  float x2 = t_maximum(bx[0], bx[2]), y2 = t_maximum(bx[1], bx[3]);
  // image -> feature (:53-58): the Python-float scale is rounded to f32 by the in-place mul
  x1 *= sx; x2 *= sx; y1 *= sy; y2 *= sy;
  x1 = t_clamp(x1, 0.0f, wmax); x2 = t_clamp(x2, 0.0f, wmax);      // :60-63
  y1 = t_clamp(y1, 0.0f, hmax); y2 = t_clamp(y2, 0.0f, hmax);
  if (min_size > 0.0f) {                                           // :65-69
    x2 = t_clamp(t_maximum(x2, x1 + min_size), 0.0f, wmax);
    y2 = t_clamp(t_maximum(y2, y1 + min_size), 0.0f, hmax);
  }
  float* o = rois + i * 5;
  o[0] = 0.0f; o[1] = x1; o[2] = y1; o[3] = x2; o[4] = y2;
}

int pow2_at_least(int64_t n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

}  // namespace

extern "C" size_t trk_det_workspace_bytes(int64_t B, int64_t A) {
  if (B <= 0 || A <= 0) return 0;
  const size_t apad = (size_t)pow2_at_least(A);
  return 256 + (size_t)B * apad * 8 + (size_t)B * (size_t)A * 24;
}

extern "C" int trk_det_nms(const float* pred, int64_t B, int64_t A, int64_t no, float conf_thres, double iou_thres,
                           int max_det, int max_nms, int agnostic, int cand_gate, float* det, int32_t* det_count,
                           int32_t* cand_count, const float* host_scale, float* xywh, void* workspace,
                           size_t workspace_bytes, void* stream) {
  TRK_REQUIRE(B >= 0 && A >= 0 && A < (1ll << 30) && no >= 6 && no < (1 << 20),
              "det_nms: need 0 <= A < 2^30 anchors and no = 5 + nc >= 6 values per anchor");
  TRK_REQUIRE(max_det >= 1 && max_det <= kMaxDetCap && max_nms >= 1,
              "det_nms: need 1 <= max_det <= %d and max_nms >= 1", kMaxDetCap);
  TRK_REQUIRE(iou_thres == iou_thres && conf_thres == conf_thres, "det_nms: NaN threshold");
  if (B == 0) return TRK_OK;
  TRK_REQUIRE(det && det_count, "det_nms: null output");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (A == 0) {
    // no anchors: every image has no detections
    hipLaunchKernelGGL(zero_i32_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, det_count, (int)B);
    if (cand_count)
      hipLaunchKernelGGL(zero_i32_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, cand_count, (int)B);
    return trk::check_launch("zero_i32_kernel");
  }
  TRK_REQUIRE(pred, "det_nms: null pred");
  TRK_REQUIRE(workspace && workspace_bytes >= trk_det_workspace_bytes(B, A) &&
                  (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
              "det_nms: workspace must be 16-B aligned and >= trk_det_workspace_bytes(B, A)");
  DetArgs a{};
  a.pred = pred; a.A = A; a.no = (int)no; a.nc = (int)no - 5;
  a.conf_thres = conf_thres; a.iou_thres = iou_thres;
  a.max_det = max_det; a.max_nms = max_nms; a.agnostic = agnostic ? 1 : 0; a.cand_gate = cand_gate;
  a.apad = pow2_at_least(A);
  unsigned char* ws = reinterpret_cast<unsigned char*>(workspace);
  a.cnt = reinterpret_cast<int*>(ws);
  TRK_REQUIRE(2 * B * 4 <= 256, "det_nms: at most 32 images per call");
  a.keys = reinterpret_cast<unsigned long long*>(ws + 256);
  a.rows = reinterpret_cast<float*>(ws + 256 + (size_t)B * a.apad * 8);
  a.det = det; a.det_count = det_count; a.cand_count = cand_count;
  if (xywh) {
    // host_scale = {gain, pad_w, pad_h, orig_w, orig_h}: scale_coords' Python doubles,
    // rounded to f32 by the tensor ops they meet (general.py:320-341)
    TRK_REQUIRE(host_scale && host_scale[0] > 0.f, "det_nms: xywh output needs host_scale with gain > 0");
    a.gain = host_scale[0]; a.pad_w = host_scale[1]; a.pad_h = host_scale[2];
    a.clip_w = host_scale[3]; a.clip_h = host_scale[4];
    a.xywh = xywh;
  }
  hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(256), 0, st, a.cnt, (int)(2 * B));
  hipLaunchKernelGGL(det_filter_kernel, dim3((unsigned)((A + 255) / 256), (unsigned)B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(det_nms_kernel, dim3((unsigned)B), dim3(kNmsThreads), 0, st, a);
  return trk::check_launch("det_nms_kernel");
}

extern "C" int trk_train_rois(const float* boxes, int64_t N, int64_t Hf, int64_t Wf, double img_h, double img_w,
                              float enforce_min_size, float* rois, void* stream) {
  TRK_REQUIRE(N >= 0 && Hf > 0 && Wf > 0 && img_h > 0 && img_w > 0, "train_rois: need N >= 0 and positive sizes");
  if (N == 0) return TRK_OK;
  TRK_REQUIRE(boxes && rois, "train_rois: null pointer");
  // scale_x = Wf / float(img_w) is a Python double; `boxes[:, 1] *= scale_x` rounds it to f32
  const float sx = (float)((double)Wf / img_w), sy = (float)((double)Hf / img_h);
  hipLaunchKernelGGL(train_rois_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), boxes, N, sx, sy, (float)(Wf - 1), (float)(Hf - 1),
                     enforce_min_size, rois);
  return trk::check_launch("train_rois_kernel");
}
