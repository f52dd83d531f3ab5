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
// argmin over the lexicographic key (spc, unassigned ? -1-pos : pos), where
// pos is the column's position in `remaining`.
//
// Latency design.  One workgroup per matrix = 1 solver wave
// + 3 loader waves.
//  * Solver (wave 0): column j lives in lane j % 64, slot j / 64, and ALL
//    per-column state (v, spc, path, row4col, position in `remaining`) is held
//    in registers, so a scan touches LDS only for the cost row and u[i].  The
//    swap-remove of `remaining` is one register update in the lane owning the
//    moved column; SC = "existed and no longer alive"; the visited rows are the
//    row4col of the removed non-sink columns, so the dual update is register-
//    local plus one scatter to u[] in LDS.  Lane-to-lane hand-offs inside the
//    solver wave need only a compiler barrier (LDS ops of a wave are in order).
//  * Loaders (waves 1-3) stream the rows the solver will augment next (row cur
//    is known in advance) into an LDS ring of RB rows, check every entry for
//    NaN / -inf on the way (scipy's validity test), and publish each row with a
//    per-slot ready word.  The solver spins (s_sleep) only when it outruns
//    them.  Loaders stay at most LA rows ahead, so the RB - LA most recently
//    solved rows remain resident and a revisited row (an assigned row on an
//    augmenting path) is read from LDS too unless it is older than that; only
//    then is it gathered from global memory.  When the whole matrix fits
//    (RB >= nr) nothing is ever evicted.
// Only +,- and comparisons touch the duals (no FMA); built -ffp-contract=off.
#include "trk_common.h"

#include <type_traits>

trk::DiagBuf g_lsap_prof;  // trk_lsap_set_prof (diagnostics)
int g_lsap_dev_lds_kb = 24;  // trk_set_tuning("lsap_dev_lds_kb"): LDS budget of trk_lsap_dev workgroups.  Small
                             // enough to be placed beside the encoder's workgroups (a CU's whole LDS would wait for
                             // a CU free of them); the leading-row shortcut needs no ring, the sequential rows re-read
                             // revisited rows from L2 when the ring is short

namespace {

constexpr int kMaxBatch = 64;
constexpr int kLoaders = 3;
constexpr uint32_t kSpinLimit = 1u << 26;  // bounded waits (never expected to trigger)

struct LsapArgs {
  const void* C;
  int64_t ld, batch_stride, kmax, nr_max;
  int64_t* rows;
  int64_t* cols;
  int32_t* count;
  int32_t* status;
  int32_t* assign;
  double cost_max;
  int ring_rows;  // RB (ring capacity in rows) for the largest working nc of the batch
  int lds_bytes;  // > 0: the launch's whole LDS budget; RB is then sized for each matrix's own nc
  unsigned long long* prof;  // trk_set_tuning("lsap_prof"): per-matrix solver cycle breakdown, else null
  const int32_t* dev_nr;  // trk_lsap_dev: shapes in device memory, bounded by nr_bound / nc_bound
  const int32_t* dev_nc;
  int nr_bound, nc_bound;
  int nr[kMaxBatch];
  int nc[kMaxBatch];
};

// shader-clock stamp (diagnostic builds of the breakdown only: A.prof != null)
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

__device__ __forceinline__ bool key_less(double v1, int k1, double v2, int k2) {
  return v1 < v2 || (v1 == v2 && k1 < k2);
}

__device__ __forceinline__ void wave_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int ld_relaxed(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ int ld_acquire(int* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void st_release(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }

// One step of a wavefront argmin over (value, key, column) with DPP lane moves
// (no LDS crossbar): lanes whose DPP source is out of range read the identity.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void argmin_step(double& v, int& key, int& col) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int olo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(0x7ff00000, hi, CTRL, ROWMASK, 0xF, false);  // +inf
  const int ok = __builtin_amdgcn_update_dpp(0x7fffffff, key, CTRL, ROWMASK, 0xF, false);
  const int oc = __builtin_amdgcn_update_dpp(-1, col, CTRL, ROWMASK, 0xF, false);
  const double ov = __hiloint2double(ohi, olo);
  const bool take = key_less(ov, ok, v, key);
  v = take ? ov : v;
  key = take ? ok : key;
  col = take ? oc : col;
}

// all-reduce over a DPP row of 16 lanes (row_ror 1, 2, 4, 8: every lane ends with the result)
template <int CTRL>
__device__ __forceinline__ int ror16(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ float row16_min(float v) {
  v = fminf(v, __int_as_float(ror16<0x121>(__float_as_int(v))));
  v = fminf(v, __int_as_float(ror16<0x122>(__float_as_int(v))));
  v = fminf(v, __int_as_float(ror16<0x124>(__float_as_int(v))));
  return fminf(v, __int_as_float(ror16<0x128>(__float_as_int(v))));
}
__device__ __forceinline__ double row16_min(double v) {
  auto step = [](double x, auto ctrl) {
    constexpr int C = decltype(ctrl)::value;
    const double o = __hiloint2double(ror16<C>(__double2hiint(x)), ror16<C>(__double2loint(x)));
    return o < x ? o : x;
  };
  v = step(v, std::integral_constant<int, 0x121>{});
  v = step(v, std::integral_constant<int, 0x122>{});
  v = step(v, std::integral_constant<int, 0x124>{});
  return step(v, std::integral_constant<int, 0x128>{});
}
__device__ __forceinline__ int row16_sum(int v) {
  v += ror16<0x121>(v);
  v += ror16<0x122>(v);
  v += ror16<0x124>(v);
  return v + ror16<0x128>(v);
}
__device__ __forceinline__ int row16_mini(int v) {
  v = min(v, ror16<0x121>(v));
  v = min(v, ror16<0x122>(v));
  v = min(v, ror16<0x124>(v));
  return min(v, ror16<0x128>(v));
}

// lexicographic min over the wave; the result is returned wave-uniform
// (row_shr 1/2/4/8 inside each row of 16, then row_bcast15 / row_bcast31,
// total in lane 63).  (value, key) pairs are unique per column, so the order
// of combination cannot change the result.
__device__ __forceinline__ void wave_argmin(double& v, int& key, int& col) {
  argmin_step<0x111, 0xF>(v, key, col);  // row_shr:1
  argmin_step<0x112, 0xF>(v, key, col);  // row_shr:2
  argmin_step<0x114, 0xF>(v, key, col);  // row_shr:4
  argmin_step<0x118, 0xF>(v, key, col);  // row_shr:8
  argmin_step<0x142, 0xA>(v, key, col);  // row_bcast:15
  argmin_step<0x143, 0xC>(v, key, col);  // row_bcast:31
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  v = __hiloint2double(hi, lo);
  key = __builtin_amdgcn_readlane(key, 63);
  col = __builtin_amdgcn_readlane(col, 63);
}

// One matrix's solve with KS column slots per lane (nc <= 64 * KS).  lsap_kernel
// picks the smallest KS that holds the matrix, so a launch sized for a larger bound
// (trk_lsap_dev: live tracks + detections in flight) pays only for the columns the
// matrix has: every per-column loop below is unrolled over KS.
template <typename T, int KS>
__device__ __forceinline__ void lsap_body(const LsapArgs& A, unsigned char* smem, const int f, const int nr0,
                                          const int nc0, const T* C, int32_t* assign, int64_t* orows,
                                          int64_t* ocols) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool tr = nc0 < nr0;
  const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;  // working problem: nr <= nc
  const int64_t ld = A.ld;
  const int RB = A.lds_bytes > 0
                     ? min(max((A.lds_bytes - 12 * nr - 48) / (nc * (int)sizeof(T) + 4), 2), nr)
                     : min(A.ring_rows, nr);
  const bool whole = RB >= nr;
  // loaders run at most LA rows ahead of the solver, so the RB - LA most
  // recently solved rows stay resident for revisits (rows on augmenting paths)
  const int LA = whole ? RB : max(1, min(16, RB / 2));

  // LDS: u[nr] f64 | col4row[nr] i32 | ready[RB] i32 | ctl[8] i32 | ring[RB][nc] T
  double* u = reinterpret_cast<double*>(smem);
  int* col4row = reinterpret_cast<int*>(u + nr);
  int* ready = col4row + nr;     // ready[s] = q + 1 when ring slot s holds row q
  int* ctl = ready + RB;         // [0] rows finished by the solver, [1] invalid entry seen,
                                 // [2] solver status, [3] shortcut prefix, [4] loader stall
  // offset arithmetic on the LDS base (an integer round trip would turn every
  // ring access into a flat load)
  const size_t ring_off = ((size_t)(12 * nr + 4 * RB + 32) + 15) & ~size_t(15);
  T* ring = reinterpret_cast<T*>(smem + ring_off);

  // diagnostics: workgroup phase stamps [entry, shortcut pass done, solver done, end]
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (A.prof) ts[0] = stamp();
  for (int q = threadIdx.x; q < RB; q += blockDim.x) ready[q] = 0;
  if (threadIdx.x < 8) ctl[threadIdx.x] = 0;

  auto gload = [&](int i, int j) -> T {  // working-matrix element from global
    return tr ? C[(int64_t)j * ld + i] : C[(int64_t)i * ld + j];
  };

  // ---- exact shortcut for the leading rows.  Row cur of the SAP starts with
  // u[cur] = 0 and, as long as every earlier row was solved by its first scan,
  // v = 0: its first scan sees spc[j] = ((0 + C[cur][j]) - 0) - 0 over all
  // columns.  If that minimum is unique and finite and its column is not the
  // minimum of an earlier row (so still unassigned), the row ends right there:
  // col4row[cur] = that column, u[cur] = 0 + minimum, v unchanged.  So the
  // longest prefix of rows with a unique finite minimum in a column no earlier
  // row's minimum took is solved in one parallel pass with exactly the state
  // the sequential algorithm reaches; the solver continues after it.
  const int ks = (nc + 63) >> 6;  // column slots in use (<= KS)
  int* firstrow = reinterpret_cast<int*>(ring);  // [nc]: the ring is idle until the loaders start
  for (int j = threadIdx.x; j < nc; j += blockDim.x) firstrow[j] = 0x7fffffff;
  if (threadIdx.x == 0) ctl[3] = nr;
  __syncthreads();
  if (A.prof) ts[7] = stamp();
  {
    // Each working row's minimum, the first column holding it and how many entries equal it.
    // A row of C (the untransposed case) is read by a 16-lane group, 4 consecutive columns
    // per lane per 64-column chunk, so a load instruction covers 4 rows x 256 contiguous
    // bytes; the group reduces with DPP row rotations (min, count, first column).  One lane
    // per row would read 64 rows per instruction (64 L2 line requests: 72K cycles for a
    // 256 x 256 frame); one wave per row spent ~150 instructions per row on wave-wide
    // reductions (64K).  A transposed problem's working rows are C's columns, so there one
    // lane per row reads contiguous memory.
    int bad = 0;
    auto publish = [&](int i, T m, int col, int cnt) {
      const bool uniq = m < (T)INFINITY && cnt == 1;
      u[i] = (double)m;
      col4row[i] = uniq ? col : -1;
      if (uniq) atomicMin(&firstrow[col], i);
      else atomicMin(&ctl[3], i);
    };
    if (tr) {
      constexpr int CH = sizeof(T) == 4 ? 64 : 32;
      for (int i0 = wave * 64; i0 < nr; i0 += 4 * 64) {
        const int i = i0 + lane, ii = min(i, nr - 1);
        T m = (T)INFINITY;
        int col = 0, cnt = 0;
        for (int j0 = 0; j0 < nc; j0 += CH) {
          T e[CH];
#pragma unroll
          for (int q = 0; q < CH; ++q) e[q] = gload(ii, min(j0 + q, nc - 1));
#pragma unroll
          for (int q = 0; q < CH; ++q) {
            const T x = e[q];
            const bool in = j0 + q < nc;
            bad |= (int)(in & ((x != x) | (x == (T)-INFINITY)));
            const bool lt = in & (x < m), eq = in & (x == m);
            col = lt ? j0 + q : col;
            cnt = lt ? 1 : cnt + (eq ? 1 : 0);
            m = lt ? x : m;
          }
        }
        if (i < nr) publish(i, m, col, cnt);
      }
    } else {
      constexpr int VEC = 4, CW = 64;                       // columns per lane / per chunk
      constexpr int CG = KS < 4 ? KS : 4;                   // chunks loaded per round
      constexpr int RR = KS <= 4 ? 4 : (KS == 8 ? 2 : 1);   // rows per lane group
      const int grp = lane >> 4, p = lane & 15;
      for (int i0 = wave * 4 * RR; i0 < nr; i0 += 16 * RR) {
        // lane-local (minimum, count, first column) over the lane's entries of each row, then
        // one 16-lane reduction per row (the group's minimum; count and first column of the
        // lanes holding it)
        T m[RR];
        int col[RR], cnt[RR];
#pragma unroll
        for (int r = 0; r < RR; ++r) {
          m[r] = (T)INFINITY;
          col[r] = 0x7fffffff;
          cnt[r] = 0;
        }
        for (int c0 = 0; c0 < ks; c0 += CG) {
          T e[CG][RR][VEC];
#pragma unroll
          for (int c = 0; c < CG; ++c)
#pragma unroll
            for (int r = 0; r < RR; ++r)
#pragma unroll
              for (int v = 0; v < VEC; ++v)
                e[c][r][v] = gload(min(i0 + grp + 4 * r, nr - 1), min((c0 + c) * CW + p * VEC + v, nc - 1));
#pragma unroll
          for (int c = 0; c < CG; ++c)
#pragma unroll
            for (int r = 0; r < RR; ++r)
#pragma unroll
              for (int v = 0; v < VEC; ++v) {
                const int cc = (c0 + c) * CW + p * VEC + v;
                const T x = e[c][r][v];
                const bool in = cc < nc;
                bad |= (int)(in & ((x != x) | (x == (T)-INFINITY)));
                const bool lt = in & (x < m[r]), eq = in & (x == m[r]);
                col[r] = lt ? cc : col[r];             // columns rise along (c, v): the first stays
                cnt[r] = lt ? 1 : cnt[r] + (int)eq;
                m[r] = lt ? x : m[r];
              }
        }
#pragma unroll
        for (int r = 0; r < RR; ++r) {
          const T gm = row16_min(m[r]);
          const bool mine = m[r] == gm;
          cnt[r] = row16_sum(mine ? cnt[r] : 0);
          col[r] = row16_mini(mine ? col[r] : 0x7fffffff);
          m[r] = gm;
        }
        if (p == 0) {
#pragma unroll
          for (int r = 0; r < RR; ++r) {
            const int i = i0 + grp + 4 * r;
            if (i < nr) publish(i, m[r], col[r], cnt[r]);
          }
        }
      }
    }
    if (__any(bad) && lane == 0) ctl[1] = 1;
  }
  if (A.prof) ts[4] = stamp();
  __syncthreads();
  if (A.prof) ts[5] = stamp();
  for (int i = threadIdx.x; i < nr; i += blockDim.x) {
    const int c = col4row[i];
    if (c >= 0 && firstrow[c] != i) atomicMin(&ctl[3], i);  // an earlier row's minimum took c
  }
  __syncthreads();
  if (A.prof) ts[6] = stamp();
  const int kpre = ctl[1] ? nr : ctl[3];  // invalid entries: the result is the error, solve nothing
  for (int i = threadIdx.x; i < nr; i += blockDim.x) {
    if (i < kpre) {
      const double spc0 = ((0.0 + u[i]) - 0.0) - 0.0;  // the first scan's spc, exactly
      u[i] = 0.0 + spc0;                              // u[cur] += minVal
    } else {
      u[i] = 0.0;
      col4row[i] = -1;
    }
  }
  int r4c_pre[KS];  // the solver's row4col for the prefix's columns
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int j = lane + 64 * k;
    const int fr = (k < ks && j < nc) ? firstrow[j] : 0x7fffffff;
    r4c_pre[k] = fr < kpre ? fr : -1;
  }
  if (threadIdx.x == 0) ctl[0] = kpre;
  __syncthreads();  // firstrow read: the ring is the loaders' from here
  if (A.prof) ts[1] = stamp();

  if (wave > 0) {
    // ------------------------------------------------------------ loaders
    int bad = 0;
    for (int q = kpre + wave - 1; q < nr; q += kLoaders) {
      // at most LA rows ahead of the solver (ctl[0] = rows it has finished);
      // this also keeps slot q % RB free (row q - RB is long finished)
      uint32_t spins = 0;
      bool stalled = false;
      while (q >= ld_relaxed(&ctl[0]) + LA) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) { stalled = true; break; }
      }
      if (stalled) {  // never overwrite a slot the solver may still read: report and stop
        if (lane == 0) ctl[4] = 1;
        break;
      }
      T* dst = ring + (int64_t)(q % RB) * nc;
      constexpr int U = 8;  // loads in flight per lane
      for (int c0 = lane; c0 < nc; c0 += 64 * U) {
        T tmp[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const int c = c0 + 64 * k;
          tmp[k] = c < nc ? gload(q, c) : (T)0;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const int c = c0 + 64 * k;
          if (c < nc) {
            if (tmp[k] != tmp[k] || tmp[k] == (T)-INFINITY) bad = 1;
            dst[c] = tmp[k];
          }
        }
      }
      if (__any(bad) && lane == 0) ctl[1] = 1;
      wave_sync();
      if (lane == 0) st_release(&ready[q % RB], q + 1);
    }
  } else {
    // ------------------------------------------------------------- solver
    double v[KS], spc[KS];
    int path[KS], r4c[KS], pos[KS];
    bool exists[KS], alive[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      exists[k] = lane + 64 * k < nc;
      v[k] = 0.0;
      path[k] = -1;
      r4c[k] = r4c_pre[k];
    }
    int status = 0;
    const bool prof = A.prof != nullptr;
    unsigned long long p_wait = 0, p_scan = 0, p_dual = 0, p_aug = 0, p_iter = 0, p_t0 = 0, p_t = 0;
    if (prof) p_t0 = p_t = stamp();
    for (int cur = kpre; cur < nr; ++cur) {
      {  // wait for row cur
        uint32_t spins = 0;
        while (ld_acquire(&ready[cur % RB]) != cur + 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kSpinLimit) { status = -3; break; }
        }
        if (status) break;
      }
      if (ld_relaxed(&ctl[1])) { status = -1; break; }  // invalid entry (a loader's check): stop early
      if (prof) { const unsigned long long t = stamp(); p_wait += t - p_t; p_t = t; }
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        spc[k] = INFINITY;
        alive[k] = exists[k];
        pos[k] = nc - 1 - (lane + 64 * k);  // remaining = [nc-1, ..., 0]
      }
      double minVal = 0.0;
      int nrem = nc, i = cur, sink = -1;
      while (sink == -1) {
        const double ui = u[i];
        // the row comes from the LDS ring (row cur, or any row when the whole
        // matrix is resident) or, for a revisited row, from global memory --
        // two separate loops so the LDS one compiles to ds_read (a merged
        // pointer would become flat_load + a full s_waitcnt per element)
        T cv[KS];
        // row i < cur is still resident unless a loader may be overwriting it:
        // loaders write rows <= cur + LA - 1, evicting rows <= cur + LA - 1 - RB
        if (i == cur || (i >= kpre && (whole || i >= cur + LA - RB))) {  // prefix rows never enter the ring
          const int slot = whole ? i : i % RB;
          const T* lrow = ring + (int64_t)slot * nc;
#pragma unroll
          for (int k = 0; k < KS; ++k) cv[k] = (k < ks && exists[k]) ? lrow[lane + 64 * k] : (T)0;
        } else {
#pragma unroll
          for (int k = 0; k < KS; ++k) cv[k] = (k < ks && alive[k]) ? gload(i, lane + 64 * k) : (T)0;
        }
        double best = INFINITY;
        int bkey = 0x7fffffff, bcol = -1;
#pragma unroll
        for (int k = 0; k < KS; ++k) {  // branch-free: dead columns are masked
          // (k < ks: uniform skip of the slots past the matrix width)
          const double r = ((minVal + (double)cv[k]) - ui) - v[k];
          const bool upd = k < ks && alive[k] && r < spc[k];
          path[k] = upd ? i : path[k];
          spc[k] = upd ? r : spc[k];
          const int key = r4c[k] == -1 ? -1 - pos[k] : pos[k];
          const bool take = k < ks && alive[k] && key_less(spc[k], key, best, bkey);
          best = take ? spc[k] : best;
          bkey = take ? key : bkey;
          bcol = take ? lane + 64 * k : bcol;
        }
        wave_argmin(best, bkey, bcol);
        minVal = best;
        if (minVal == INFINITY) { status = -2; break; }
        const int idx = bkey < 0 ? -1 - bkey : bkey;  // position in `remaining`
        const int j = bcol;
        const int jk = j >> 6;
        int rsel = -1;
#pragma unroll
        for (int k = 0; k < KS; ++k) rsel = (k == jk) ? r4c[k] : rsel;
        const int rj = __builtin_amdgcn_readlane(rsel, j & 63);
        if (rj == -1) sink = j; else i = rj;
#pragma unroll
        for (int k = 0; k < KS; ++k) {  // swap-remove: pos nrem-1 moves to idx
          const bool me = lane + 64 * k == j;
          pos[k] = (alive[k] && !me && pos[k] == nrem - 1) ? idx : pos[k];
          alive[k] = alive[k] && !me;
        }
        --nrem;
        if (prof) ++p_iter;
      }
      if (status) break;
      if (prof) { const unsigned long long t = stamp(); p_scan += t - p_t; p_t = t; }
      // dual update (scipy order: u[cur], the other visited rows, the columns)
      if (lane == 0) u[cur] += minVal;
      wave_sync();
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        if (k >= ks || !exists[k] || alive[k]) continue;
        const double d = minVal - spc[k];
        if (lane + 64 * k != sink) u[r4c[k]] += d;
        v[k] -= d;
      }
      wave_sync();
      if (prof) { const unsigned long long t = stamp(); p_dual += t - p_t; p_t = t; }
      // augment along path (serial; one owner lane per step)
      int j = sink;
      for (;;) {
        const int ol = j & 63, ok = j >> 6;
        int pr = -1;
#pragma unroll
        for (int k = 0; k < KS; ++k) pr = (k == ok) ? path[k] : pr;
        const int r = __builtin_amdgcn_readlane(pr, ol);
#pragma unroll
        for (int k = 0; k < KS; ++k) r4c[k] = (lane == ol && k == ok) ? r : r4c[k];
        const int t = col4row[r];
        wave_sync();
        if (lane == 0) col4row[r] = j;
        wave_sync();
        j = t;
        if (r == cur) break;
      }
      if (lane == 0) st_release(&ctl[0], cur + 1);  // slot cur % RB may be refilled
      if (prof) { const unsigned long long t = stamp(); p_aug += t - p_t; p_t = t; }
    }
    if (prof && lane == 0) {
      unsigned long long* o = A.prof + (int64_t)f * 16;
      o[0] = p_wait; o[1] = p_scan; o[2] = p_dual; o[3] = p_aug; o[4] = p_iter;
      o[5] = p_t - p_t0; o[6] = (unsigned long long)nr; o[7] = (unsigned long long)nc;
    }
    if (lane == 0) {
      ctl[2] = status;
      if (status) ctl[0] = 0x3fffffff;  // release any waiting loader
    }
    // the transposed result lives in r4c registers: park it in the (now idle) ring
    if (tr) {
      int* r4c_out = reinterpret_cast<int*>(ring);
#pragma unroll
      for (int k = 0; k < KS; ++k)
        if (exists[k]) r4c_out[lane + 64 * k] = r4c[k];
    }
  }
  __syncthreads();
  if (A.prof) ts[2] = stamp();
  int status = ctl[2];
  if (ctl[4]) status = -3;  // a loader stalled: not a property of the matrix
  if (ctl[1]) status = -1;  // an invalid entry anywhere -> scipy raises (checked first)
  if (status) {
    if (assign)
      for (int r = threadIdx.x; r < nr0; r += blockDim.x) assign[r] = -1;
    if (threadIdx.x == 0) { A.count[f] = 0; A.status[f] = status; }
    return;
  }
  auto prof_end = [&]() {
    if (A.prof && threadIdx.x == 0) {
      ts[3] = stamp();
      unsigned long long* o = A.prof + (int64_t)f * 16 + 8;
      o[0] = ts[1] - ts[0];  // shortcut pass (incl. set-up)
      o[1] = ts[2] - ts[1];  // loaders + solver
      o[2] = ts[3] - ts[2];  // outputs
      o[3] = ts[3] - ts[0];
      o[4] = ts[7] - ts[0];  // set-up (ring words, firstrow)
      o[5] = ts[4] - ts[7];  // the row scans
      o[6] = ts[5] - ts[4];  // their barrier
      o[7] = ts[1] - ts[5];  // claim check, duals, hand-over
    }
  };
  if (!tr) {
    // a matrix solved whole by the shortcut: no augmenting path moved any row or dual since,
    // so u[q] still is C[q][col4row[q]] (exactly: the float minimum widened to double)
    const int kp = ctl[3] >= nr ? nr : 0;
    for (int q = threadIdx.x; q < nr; q += blockDim.x) {
      const int c = col4row[q];
      orows[q] = q;
      ocols[q] = c;
      if (assign) assign[q] = ((q < kp ? u[q] : (double)C[(int64_t)q * ld + c]) <= A.cost_max) ? c : -1;
    }
  } else {
    // argsort(col4row): working column j (= original row j) is matched to
    // working row r4c[j] (= original column); emit in ascending j
    const int* r4c_out = reinterpret_cast<const int*>(ring);
    if (assign)
      for (int r = threadIdx.x; r < nr0; r += blockDim.x) assign[r] = -1;
    if (wave == 0) {
      int base = 0;
      for (int j0 = 0; j0 < nc; j0 += 64) {
        const int j = j0 + lane;
        const int rc = j < nc ? r4c_out[j] : -1;
        const uint64_t bal = __ballot(rc >= 0);
        if (rc >= 0) {
          const int w = base + __popcll(bal & ((1ull << lane) - 1));
          orows[w] = j;
          ocols[w] = rc;
        }
        base += __popcll(bal);
      }
    }
    __syncthreads();
    if (assign)
      for (int j = threadIdx.x; j < nc; j += blockDim.x) {
        const int rc = r4c_out[j];
        if (rc >= 0) assign[j] = ((double)C[(int64_t)j * ld + rc] <= A.cost_max) ? rc : -1;
      }
  }
  if (threadIdx.x == 0) { A.count[f] = nr; A.status[f] = 0; }
  prof_end();
}

constexpr int lsap_ks_next(int k) { return k == 1 ? 4 : 2 * k; }

template <typename T, int KS, int KSMAX>
__device__ __forceinline__ void lsap_pick(const int ks, const LsapArgs& A, unsigned char* smem, const int f,
                                          const int nr0, const int nc0, const T* C, int32_t* assign,
                                          int64_t* orows, int64_t* ocols) {
  if constexpr (KS >= KSMAX) {
    lsap_body<T, KSMAX>(A, smem, f, nr0, nc0, C, assign, orows, ocols);
  } else {
    if (ks <= KS) lsap_body<T, KS>(A, smem, f, nr0, nc0, C, assign, orows, ocols);
    else lsap_pick<T, lsap_ks_next(KS), KSMAX>(ks, A, smem, f, nr0, nc0, C, assign, orows, ocols);
  }
}

// one workgroup per matrix; KSMAX = the column slots the launch's widest (bound) matrix
// needs, the body run = the smallest of 1 / 4 / 8 / 16 / 32 slots this matrix fits
template <typename T, int KSMAX>
__global__ void __launch_bounds__(256)
lsap_kernel(const LsapArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int f = blockIdx.x;
  int nr0 = A.nr[f], nc0 = A.nc[f];
  const T* C = reinterpret_cast<const T*>(A.C) + (int64_t)f * A.batch_stride;
  int32_t* assign = A.assign ? A.assign + (int64_t)f * A.nr_max : nullptr;
  int64_t* orows = A.rows + (int64_t)f * A.kmax;
  int64_t* ocols = A.cols + (int64_t)f * A.kmax;
  if (A.dev_nr) {
    nr0 = A.dev_nr[f];
    nc0 = A.dev_nc[f];
    const bool out = nr0 < 0 || nc0 < 0 || nr0 > A.nr_bound || nc0 > A.nc_bound;
    if (out) {  // outside the launch's sizing
      if (assign)
        for (int r = threadIdx.x; r < A.nr_bound; r += blockDim.x) assign[r] = -1;
      if (threadIdx.x == 0) { A.count[f] = 0; A.status[f] = -4; }
      return;
    }
  }
  if (nr0 == 0 || nc0 == 0) {
    if (assign)
      for (int r = threadIdx.x; r < nr0; r += blockDim.x) assign[r] = -1;
    if (threadIdx.x == 0) { A.count[f] = 0; A.status[f] = 0; }
    return;
  }
  const int ks = (max(nr0, nc0) + 63) >> 6;  // the working problem's column slots (nc = max)
  lsap_pick<T, 1, KSMAX>(ks, A, smem, f, nr0, nc0, C, assign, orows, ocols);
}

template <typename T>
int launch_ks(int wc, dim3 g, size_t lds, hipStream_t st, const LsapArgs& a) {
  auto go = [&](auto ks) {
    constexpr int KS = decltype(ks)::value;
    static bool attr_set = false;
    if (!attr_set) {  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per CU)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lsap_kernel<T, KS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    hipLaunchKernelGGL((lsap_kernel<T, KS>), g, dim3(64 * (1 + kLoaders)), lds, st, a);
  };
  if (wc <= 64) go(std::integral_constant<int, 1>{});
  else if (wc <= 256) go(std::integral_constant<int, 4>{});
  else if (wc <= 512) go(std::integral_constant<int, 8>{});
  else if (wc <= 1024) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, 32>{});
  return trk::check_launch("lsap_kernel");
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
  const size_t lds_limit = 156 * 1024;
  for (int64_t f0 = 0; f0 < F; f0 += kMaxBatch) {
    const int nf = (int)std::min<int64_t>(kMaxBatch, F - f0);
    LsapArgs a;
    memset(&a, 0, sizeof a);
    int wr_max = 1, wc_max = 1;
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
      wr_max = std::max(wr_max, std::min(r, c));
      wc_max = std::max(wc_max, std::max(r, c));
    }
    TRK_REQUIRE(C, "lsap: null cost pointer");
    // fixed part: u (8) + col4row (4) per working row, control words, alignment
    const size_t fixed = 12 * (size_t)wr_max + 64;
    const size_t row_bytes = esz * (size_t)wc_max + 4;  // + its ready word
    TRK_REQUIRE(fixed + 2 * row_bytes <= lds_limit, "lsap: matrix too wide for the LDS ring");
    int rb = (int)std::min<size_t>((lds_limit - fixed) / row_bytes, (size_t)wr_max);
    rb = std::max(rb, 2);
    a.ring_rows = rb;
    const size_t lds = fixed + (size_t)rb * row_bytes + 16;
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
    a.prof = g_lsap_prof.get() ? g_lsap_prof.get() + f0 * 16 : nullptr;
    int e = dtype == TRK_F32 ? launch_ks<float>(wc_max, dim3(nf), lds, st, a)
                             : launch_ks<double>(wc_max, dim3(nf), lds, st, a);
    if (e) return e;
  }
  return TRK_OK;
}

extern "C" int trk_lsap_dev(int64_t F, const void* C, int dtype, int64_t ld, int64_t batch_stride,
                            const int32_t* dev_nr, const int32_t* dev_nc, int64_t nr_bound, int64_t nc_bound,
                            int64_t kmax, int64_t* rows, int64_t* cols, int32_t* count, int32_t* status,
                            int32_t* assign, int64_t nr_max, double cost_max, void* stream) {
  TRK_REQUIRE(F >= 0, "lsap_dev: negative batch");
  TRK_REQUIRE(dtype == TRK_F32 || dtype == TRK_F64, "lsap_dev: dtype must be f32 or f64");
  if (F == 0) return TRK_OK;
  TRK_REQUIRE(dev_nr && dev_nc && rows && cols && count && status, "lsap_dev: null pointer");
  TRK_REQUIRE(nr_bound >= 0 && nc_bound >= 0 && nr_bound <= TRK_LSAP_MAX_DIM && nc_bound <= TRK_LSAP_MAX_DIM,
              "lsap_dev: bounds (%lld, %lld) outside [0, %d]", (long long)nr_bound, (long long)nc_bound,
              TRK_LSAP_MAX_DIM);
  TRK_REQUIRE(nc_bound <= ld, "lsap_dev: ld %lld < nc bound %lld", (long long)ld, (long long)nc_bound);
  TRK_REQUIRE(std::min(nr_bound, nc_bound) <= kmax, "lsap_dev: kmax < min(nr, nc) bound");
  TRK_REQUIRE(!assign || nr_bound <= nr_max, "lsap_dev: nr_max < nr bound");
  TRK_REQUIRE(C, "lsap_dev: null cost pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t esz = dtype == TRK_F32 ? 4 : 8;
  const size_t lds_limit = 156 * 1024;
  const int wr_max = (int)std::max<int64_t>(1, std::min(nr_bound, nc_bound));
  const int wc_max = (int)std::max<int64_t>(1, std::max(nr_bound, nc_bound));
  const size_t fixed = 12 * (size_t)wr_max + 64;
  const size_t row_bytes = esz * (size_t)wc_max + 4;
  TRK_REQUIRE(fixed + 2 * row_bytes <= lds_limit, "lsap_dev: matrix too wide for the LDS ring");
  // the budget, raised to what two ring rows of the widest bound need
  const size_t lds = std::min(lds_limit, std::max((size_t)g_lsap_dev_lds_kb * 1024, fixed + 2 * row_bytes + 16));
  const int rb = 2;  // unused: the kernel sizes RB per matrix from lds (a.lds_bytes)
  for (int64_t f0 = 0; f0 < F; f0 += kMaxBatch) {
    const int nf = (int)std::min<int64_t>(kMaxBatch, F - f0);
    LsapArgs a;
    memset(&a, 0, sizeof a);
    a.ring_rows = rb;
    a.lds_bytes = (int)lds;
    a.dev_nr = dev_nr + f0;
    a.dev_nc = dev_nc + f0;
    a.nr_bound = (int)nr_bound;
    a.nc_bound = (int)nc_bound;
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
    a.prof = g_lsap_prof.get() ? g_lsap_prof.get() + f0 * 16 : nullptr;
    const int e = dtype == TRK_F32 ? launch_ks<float>(wc_max, dim3(nf), lds, st, a)
                                   : launch_ks<double>(wc_max, dim3(nf), lds, st, a);
    if (e) return e;
  }
  return TRK_OK;
}

/* diagnostics: per-matrix solver cycle breakdown of later trk_lsap / trk_lsap_dev launches
 * into buf [F][16] u64 (solver: wait, scan, dual, augment, iterations, total, nr, nc; workgroup:
 * shortcut pass, loaders + solver, outputs, total, 0...); NULL = off */
extern "C" int trk_lsap_set_prof(unsigned long long* buf) {
  g_lsap_prof.set(buf);
  return TRK_OK;
}
