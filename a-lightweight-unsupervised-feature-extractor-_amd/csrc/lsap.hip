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
// One 64-lane wavefront per matrix (latency-bound: every augmentation step is
// a dependent scan); matrices of a batch run on separate CUs.  All solver
// state lives in LDS; the cost matrix is cached in LDS too when it fits, else
// each scan gathers its row from L2.  Only +,- and comparisons touch the duals
// (no FMA to contract) -- the file is still built with -ffp-contract=off.
#include "trk_common.h"

namespace {

constexpr int kMaxBatch = 64;

struct LsapArgs {
  const void* C;
  int64_t ld, batch_stride, kmax, nr_max;
  int64_t* rows;
  int64_t* cols;
  int32_t* count;
  int32_t* status;
  int32_t* assign;
  double cost_max;
  int cache;  // 1: cost matrix copied into LDS
  int nr[kMaxBatch];
  int nc[kMaxBatch];
};

__device__ __forceinline__ bool key_less(double v1, int k1, double v2, int k2) {
  return v1 < v2 || (v1 == v2 && k1 < k2);
}

template <typename T>
__global__ void __launch_bounds__(64)
lsap_kernel(const LsapArgs A, int f_base) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  const int nr0 = A.nr[f], nc0 = A.nc[f];
  const T* C = reinterpret_cast<const T*>(A.C) + (int64_t)f * A.batch_stride;
  int32_t* assign = A.assign ? A.assign + (int64_t)f * A.nr_max : nullptr;
  int64_t* orows = A.rows + (int64_t)f * A.kmax;
  int64_t* ocols = A.cols + (int64_t)f * A.kmax;
  (void)f_base;
  if (assign)
    for (int r = lane; r < nr0; r += 64) assign[r] = -1;
  if (nr0 == 0 || nc0 == 0) {
    if (lane == 0) { A.count[f] = 0; A.status[f] = 0; }
    return;
  }
  const bool tr = nc0 < nr0;
  const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;
  const int64_t ld = A.ld;

  // ---- LDS carve (8-byte arrays first)
  double* u = reinterpret_cast<double*>(smem);
  double* v = u + nr;
  double* spc = v + nc;
  int* path = reinterpret_cast<int*>(spc + nc);
  int* row4col = path + nc;
  int* col4row = row4col + nc;
  int* rem = col4row + nr;
  unsigned char* SR = reinterpret_cast<unsigned char*>(rem + nc);
  unsigned char* SC = SR + nr;
  T* cache = reinterpret_cast<T*>(
      (reinterpret_cast<uintptr_t>(SC + nc) + 15) & ~uintptr_t(15));

  // element (i, j) of the (possibly transposed) working matrix
  auto elem_g = [&](int i, int j) -> double {
    return tr ? (double)C[(int64_t)j * ld + i] : (double)C[(int64_t)i * ld + j];
  };

  // ---- validity scan (NaN / -inf -> "invalid numeric entries") + LDS cache
  int bad = 0;
  for (int64_t q = lane; q < (int64_t)nr0 * nc0; q += 64) {
    const int r = (int)(q / nc0), c = (int)(q % nc0);
    const double x = (double)C[(int64_t)r * ld + c];
    if (x != x || x == -INFINITY) bad = 1;
    if (A.cache) {
      if (tr) cache[(int64_t)c * nc + r] = (T)x;
      else cache[q] = (T)x;
    }
  }
  if (__any(bad)) {
    if (lane == 0) { A.count[f] = 0; A.status[f] = -1; }
    return;
  }
  auto elem = [&](int i, int j) -> double {
    return A.cache ? (double)cache[(int64_t)i * nc + j] : elem_g(i, j);
  };

  for (int r = lane; r < nr; r += 64) { u[r] = 0.0; col4row[r] = -1; }
  for (int c = lane; c < nc; c += 64) { v[c] = 0.0; path[c] = -1; row4col[c] = -1; }
  __syncthreads();

  int status = 0;
  for (int cur = 0; cur < nr; ++cur) {
    // augmenting_path(): reset per row
    for (int c = lane; c < nc; c += 64) {
      rem[c] = nc - c - 1;
      SC[c] = 0;
      spc[c] = INFINITY;
    }
    for (int r = lane; r < nr; r += 64) SR[r] = 0;
    __syncthreads();
    double minVal = 0.0;
    int nrem = nc, i = cur, sink = -1;
    while (sink == -1) {
      if (lane == 0) SR[i] = 1;
      const double ui = u[i];
      double best = INFINITY;
      int bkey = 0x7fffffff;
      for (int it = lane; it < nrem; it += 64) {
        const int j = rem[it];
        const double r = ((minVal + elem(i, j)) - ui) - v[j];
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
      __syncthreads();  // every lane's spc/path writes of this scan are in
      const int j = rem[idx];
      const int rj = row4col[j];
      if (rj == -1) sink = j; else i = rj;
      __syncthreads();
      if (lane == 0) {
        SC[j] = 1;
        rem[idx] = rem[nrem - 1];
      }
      --nrem;
      __syncthreads();
    }
    if (status) break;
    // dual update (scipy order: u[cur] first, then other SR rows, then SC cols)
    if (lane == 0) u[cur] += minVal;
    __syncthreads();
    for (int r = lane; r < nr; r += 64)
      if (SR[r] && r != cur) u[r] += minVal - spc[col4row[r]];
    for (int c = lane; c < nc; c += 64)
      if (SC[c]) v[c] -= minVal - spc[c];
    __syncthreads();
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
    __syncthreads();
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
    __syncthreads();
    for (int q = lane; q < nr; q += 64) pos[col4row[q]] = q;
    __syncthreads();
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

size_t state_bytes(int nr, int nc) {
  return 8 * (size_t)(nr + 2 * nc) + 4 * (size_t)(3 * nc + 2 * nr) + (size_t)(nr + nc) + 16;
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
  for (int64_t f0 = 0; f0 < F; f0 += kMaxBatch) {
    const int nf = (int)std::min<int64_t>(kMaxBatch, F - f0);
    LsapArgs a;
    memset(&a, 0, sizeof a);
    size_t lds_state = 0, lds_cache = 0;
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
      lds_state = std::max(lds_state, state_bytes(r, c));
      lds_cache = std::max(lds_cache, esz * (size_t)r * c);
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
    const size_t lds_limit = 150 * 1024;
    a.cache = lds_state + lds_cache <= lds_limit ? 1 : 0;
    const size_t lds = lds_state + (a.cache ? lds_cache : 0);
    static bool attr_set = false;
    if (!attr_set) {  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per CU)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lsap_kernel<float>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lsap_kernel<double>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    if (dtype == TRK_F32)
      hipLaunchKernelGGL(lsap_kernel<float>, dim3(nf), dim3(64), lds, st, a, (int)f0);
    else
      hipLaunchKernelGGL(lsap_kernel<double>, dim3(nf), dim3(64), lds, st, a, (int)f0);
    if (int e = trk::check_launch("lsap_kernel")) return e;
  }
  return TRK_OK;
}
