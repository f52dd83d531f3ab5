// Rectangular linear sum assignment on gfx950 (MI355X), batched over matrices.
//
// Replaces scipy.optimize.linear_sum_assignment as called at reference
// model/utils/costTool/hung.py:28 (hungarian_assign, hung.py:5-45), index for
// index: Crouse's shortest augmenting path exactly as scipy's rectangular_lsap
// runs it (oracle/trk_oracle.c:ora_lsap) -- float64 duals, the
// reversed `remaining` list with swap-remove, and scipy's tie rule
//     pick it if spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)
// which selects, among the minimum entries, the LAST unassigned column in
// `remaining` order, else the FIRST one.  The serial scan becomes a wavefront
// argmin over the lexicographic key (spc, unassigned ? -1-it : it).
//
// Latency design: one 64-lane wavefront per matrix, so every
// lane-to-lane hand-off is LDS traffic of one wave (in order), synchronised by
// wavefront-scope fences only -- no s_barrier, no vmcnt drains.  All solver
// state lives in LDS.  The cost matrix is cached whole in LDS when it fits;
// otherwise the row of the NEXT augmentation (cur+1, known in advance) is
// prefetched into registers while row cur is solved and parked in an LDS row
// buffer, so the common tracking case (one scan per row) never waits on L2.
// Removed columns are swapped to the tail of `remaining` (same order for the
// live prefix as scipy's overwrite), so SC = remaining[nrem:] and the visited
// rows are kept in a list: nothing is reset per row except spc and remaining.
// Only +,- and comparisons touch the duals (no FMA to contract); the file is
// still built with -ffp-contract=off.
#include "trk_common.h"

namespace {

constexpr int kMaxBatch = 64;
constexpr int kPrefetchCols = 512;  // row prefetch up to nc <= 512 (8 regs per lane)

struct LsapArgs {
  const void* C;
  int64_t ld, batch_stride, kmax, nr_max;
  int64_t* rows;
  int64_t* cols;
  int32_t* count;
  int32_t* status;
  int32_t* assign;
  double cost_max;
  int cache;  // 1: whole (working) cost matrix copied into LDS
  int nr[kMaxBatch];
  int nc[kMaxBatch];
};

__device__ __forceinline__ bool key_less(double v1, int k1, double v2, int k2) {
  return v1 < v2 || (v1 == v2 && k1 < k2);
}

// single-wavefront workgroup: order LDS traffic between lanes without s_barrier
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// LDS bytes used by the solver state for a WORKING (nr <= nc) problem
__host__ __device__ inline size_t state_bytes(int nr, int nc) {
  return 8 * (size_t)(nr + 2 * nc)          // u, v, spc
         + 4 * (size_t)(3 * nc + 2 * nr)    // path, row4col, rem, col4row, srlist
         + 16;
}

template <typename T>
__global__ void __launch_bounds__(64)
lsap_kernel(const LsapArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  const int nr0 = A.nr[f], nc0 = A.nc[f];
  const T* C = reinterpret_cast<const T*>(A.C) + (int64_t)f * A.batch_stride;
  int32_t* assign = A.assign ? A.assign + (int64_t)f * A.nr_max : nullptr;
  int64_t* orows = A.rows + (int64_t)f * A.kmax;
  int64_t* ocols = A.cols + (int64_t)f * A.kmax;
  if (assign)
    for (int r = lane; r < nr0; r += 64) assign[r] = -1;
  if (nr0 == 0 || nc0 == 0) {
    if (lane == 0) { A.count[f] = 0; A.status[f] = 0; }
    return;
  }
  const bool tr = nc0 < nr0;
  const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;
  const int64_t ld = A.ld;

  double* u = reinterpret_cast<double*>(smem);
  double* v = u + nr;
  double* spc = v + nc;
  int* path = reinterpret_cast<int*>(spc + nc);
  int* row4col = path + nc;
  int* rem = row4col + nc;
  int* col4row = rem + nc;
  int* srlist = col4row + nr;
  T* extra = reinterpret_cast<T*>(
      (reinterpret_cast<uintptr_t>(srlist + nr) + 15) & ~uintptr_t(15));
  // extra = whole matrix (cache) or 2 row buffers of nc (prefetch mode)
  const bool cache = A.cache != 0;
  const bool prefetch = !cache && nc <= kPrefetchCols;

  auto gload = [&](int i, int j) -> T {  // working-matrix element from global
    return tr ? C[(int64_t)j * ld + i] : C[(int64_t)i * ld + j];
  };

  // ---- validity scan (NaN / -inf -> "invalid numeric entries") + LDS cache
  int bad = 0;
  for (int64_t q = lane; q < (int64_t)nr0 * nc0; q += 64) {
    const int r = (int)(q / nc0), c = (int)(q % nc0);
    const T x = C[(int64_t)r * ld + c];
    if (x != x || x == (T)-INFINITY) bad = 1;
    if (cache) {
      if (tr) extra[(int64_t)c * nc + r] = x;
      else extra[q] = x;
    }
  }
  if (__any(bad)) {
    if (lane == 0) { A.count[f] = 0; A.status[f] = -1; }
    return;
  }

  for (int r = lane; r < nr; r += 64) { u[r] = 0.0; col4row[r] = -1; }
  for (int c = lane; c < nc; c += 64) { v[c] = 0.0; path[c] = -1; row4col[c] = -1; }
  T pre[kPrefetchCols / 64];
  if (prefetch) {  // row 0 straight into buffer 0
    for (int c = lane; c < nc; c += 64) extra[c] = gload(0, c);
  }
  wave_sync();

  int status = 0;
  for (int cur = 0; cur < nr; ++cur) {
    const T* rowbuf = prefetch ? extra + (int64_t)(cur & 1) * nc : nullptr;
    // prefetch row cur+1 into registers; committed to LDS after this row
    if (prefetch && cur + 1 < nr) {
#pragma unroll
      for (int k = 0; k < kPrefetchCols / 64; ++k) {
        const int c = lane + 64 * k;
        if (c < nc) pre[k] = gload(cur + 1, c);
      }
    }
    for (int c = lane; c < nc; c += 64) {
      rem[c] = nc - c - 1;
      spc[c] = INFINITY;
    }
    wave_sync();
    double minVal = 0.0;
    int nrem = nc, i = cur, sink = -1, nsr = 0;
    while (sink == -1) {
      if (lane == 0) srlist[nsr] = i;
      ++nsr;
      const double ui = u[i];
      double best = INFINITY;
      int bkey = 0x7fffffff;
      for (int it = lane; it < nrem; it += 64) {
        const int j = rem[it];
        T cij;
        if (cache) cij = extra[(int64_t)i * nc + j];
        else if (prefetch && i == cur) cij = rowbuf[j];
        else cij = gload(i, j);
        const double r = ((minVal + (double)cij) - ui) - v[j];
        double s = spc[j];
        if (r < s) { path[j] = i; spc[j] = r; s = r; }
        const int key = row4col[j] == -1 ? -1 - it : it;
        if (key_less(s, key, best, bkey)) { best = s; bkey = key; }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int ok = __shfl_xor(bkey, off);
        if (key_less(ob, ok, best, bkey)) { best = ob; bkey = ok; }
      }
      minVal = best;
      if (minVal == INFINITY) { status = -2; break; }
      const int idx = bkey < 0 ? -1 - bkey : bkey;
      wave_sync();
      const int j = rem[idx];
      const int rj = row4col[j];
      if (rj == -1) sink = j; else i = rj;
      wave_sync();
      if (lane == 0) {  // swap-remove: live prefix matches scipy, SC = tail
        rem[idx] = rem[nrem - 1];
        rem[nrem - 1] = j;
      }
      --nrem;
      wave_sync();
    }
    if (status) break;
    // dual update (scipy order: u[cur] first, then the other visited rows,
    // then the removed columns); visited rows are distinct, as are columns
    if (lane == 0) u[cur] += minVal;
    wave_sync();
    for (int q = lane + 1; q < nsr; q += 64) {
      const int r = srlist[q];
      u[r] += minVal - spc[col4row[r]];
    }
    for (int it = nrem + lane; it < nc; it += 64) {
      const int c = rem[it];
      v[c] -= minVal - spc[c];
    }
    wave_sync();
    if (lane == 0) {  // augment along path
      int j = sink;
      for (;;) {
        const int r = path[j];
        row4col[j] = r;
        const int t = col4row[r];
        col4row[r] = j;
        j = t;
        if (r == cur) break;
      }
    }
    if (prefetch && cur + 1 < nr) {
      T* nb = extra + (int64_t)((cur + 1) & 1) * nc;
#pragma unroll
      for (int k = 0; k < kPrefetchCols / 64; ++k) {
        const int c = lane + 64 * k;
        if (c < nc) nb[c] = pre[k];
      }
    }
    wave_sync();
  }

  if (status) {
    if (lane == 0) { A.count[f] = 0; A.status[f] = status; }
    return;
  }
  const int k = nr;  // = min(nr0, nc0)
  if (!tr) {
    for (int q = lane; q < nr; q += 64) {
      const int c = col4row[q];
      orows[q] = q;
      ocols[q] = c;
      if (assign) assign[q] = ((double)C[(int64_t)q * ld + c] <= A.cost_max) ? c : -1;
    }
  } else {
    // argsort(col4row): col4row[q] (an original row) is distinct per q
    int* pos = reinterpret_cast<int*>(spc);  // nc (= original nr) ints fit in spc
    for (int c = lane; c < nc; c += 64) pos[c] = -1;
    wave_sync();
    for (int q = lane; q < nr; q += 64) pos[col4row[q]] = q;
    wave_sync();
    if (lane == 0) {
      int w = 0;
      for (int r = 0; r < nc; ++r)
        if (pos[r] >= 0) { orows[w] = r; ocols[w] = pos[r]; ++w; }
    }
    for (int q = lane; q < nr; q += 64) {
      const int r0 = col4row[q];  // original row matched to original column q
      if (assign) assign[r0] = ((double)C[(int64_t)r0 * ld + q] <= A.cost_max) ? q : -1;
    }
  }
  if (lane == 0) { A.count[f] = k; A.status[f] = 0; }
}

}  // namespace

extern "C" int trk_lsap(int64_t F, const void* C, int dtype, int64_t ld, int64_t batch_stride,
                        const int32_t* host_nr, const int32_t* host_nc, int64_t kmax,
                        int64_t* rows, int64_t* cols, int32_t* count, int32_t* status,
                        int32_t* assign, int64_t nr_max, double cost_max, void* stream) {
  TRK_REQUIRE(F >= 0, "lsap: negative batch");
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_F64, "lsap: dtype must be f32 or f64");
  if (F == 0) return TRK_OK;
  TRK_REQUIRE(host_nr && host_nc && rows && cols && count && status, "lsap: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t esz = dtype == TRK_F32 ? 4 : 8;
  const size_t lds_limit = 150 * 1024;
  for (int64_t f0 = 0; f0 < F; f0 += kMaxBatch) {
    const int nf = (int)std::min<int64_t>(kMaxBatch, F - f0);
    LsapArgs a;
    memset(&a, 0, sizeof a);
    size_t lds_state = 0, lds_cache = 0, lds_rows = 0;
    for (int q = 0; q < nf; ++q) {
      const int r = host_nr[f0 + q], c = host_nc[f0 + q];
      TRK_REQUIRE(r >= 0 && c >= 0 && r <= TRK_LSAP_MAX_DIM && c <= TRK_LSAP_MAX_DIM,
                  "lsap: matrix %lld shape (%d, %d) outside [0, %d]", (long long)(f0 + q), r, c,
                  TRK_LSAP_MAX_DIM);
      TRK_REQUIRE(c <= ld || r == 0, "lsap: ld %lld < nc %d", (long long)ld, c);
      TRK_REQUIRE(std::min(r, c) <= kmax, "lsap: kmax %lld < min(nr, nc)", (long long)kmax);
      TRK_REQUIRE(!assign || r <= nr_max, "lsap: nr_max %lld < nr %d", (long long)nr_max, r);
      a.nr[q] = r;
      a.nc[q] = c;
      const int wr = std::min(r, c), wc = std::max(r, c);  // working (transposed if tall)
      lds_state = std::max(lds_state, state_bytes(wr, wc));
      lds_cache = std::max(lds_cache, esz * (size_t)r * c);
      lds_rows = std::max(lds_rows, wc <= kPrefetchCols ? 2 * esz * (size_t)wc : 0);
    }
    TRK_REQUIRE(C, "lsap: null cost pointer");
    a.C = reinterpret_cast<const char*>(C) + (size_t)f0 * batch_stride * esz;
    a.ld = ld;
    a.batch_stride = batch_stride;
    a.kmax = kmax;
    a.nr_max = nr_max;
    a.rows = rows + f0 * kmax;
    a.cols = cols + f0 * kmax;
    a.count = count + f0;
    a.status = status + f0;
    a.assign = assign ? assign + f0 * nr_max : nullptr;
    a.cost_max = cost_max;
    a.cache = lds_state + lds_cache <= lds_limit ? 1 : 0;
    const size_t lds = lds_state + (a.cache ? lds_cache : lds_rows);
    static bool attr_set = false;
    if (!attr_set) {  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per CU)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lsap_kernel<float>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lsap_kernel<double>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    if (dtype == TRK_F32)
      hipLaunchKernelGGL(lsap_kernel<float>, dim3(nf), dim3(64), lds, st, a);
    else
      hipLaunchKernelGGL(lsap_kernel<double>, dim3(nf), dim3(64), lds, st, a);
    if (int e = trk::check_launch("lsap_kernel")) return e;
  }
  return TRK_OK;
}
