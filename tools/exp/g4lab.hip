// gemm4 laboratory (diagnostics, not product code): the product's gemm4 tile with
// switches, built beside the product into tools/exp/libg4lab.so
//   F & 1   every workgroup reads M tile 0's A rows (L2-resident)
//   F & 2   stop after the K loop          F & 8   no MFMAs     F & 16  no operand DMA
//   F & 32  prefetch the tile's A rows into L2 (one dword per line) before the K loop
//   F & 64  no activation (bias only)   F & 128 no ROI sums   F & 256 no output stores
#include "../../a-lightweight-unsupervised-feature-extractor-_amd/csrc/enc_gemm.hip"
namespace {
template <int EPI, bool WIDE, int HSWM, int F>
__device__ __forceinline__ void g4lab_tile(const EncGemmArgs& a, int64_t lb, unsigned char* smem) {
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
  const int64_t m0 = mt * 128;
  const uint16_t* Ag = a.A + (int64_t)g * a.K;
  const uint16_t* Bg = a.B + (int64_t)g * a.N * a.K;
  const int nk = a.K / BK;
  const int64_t roi_base = m0 / a.P;

  const uint16_t* asrc[2];
  const uint16_t* bsrc[4];
  int arow[2], achk[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    arow[q] = r;
    achk[q] = c;
    asrc[q] = Ag + ((F & 1) ? (int64_t)r : min(m0 + r, (int64_t)a.M - 1)) * a.lda + c * 8;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    bsrc[q] = Bg + (int64_t)(n0 + r) * a.K + c * 8;
  }
  auto issue = [&](int kt) {
    if (F & 16) return;
    uint4* d = ring + (kt % 3) * G4_BUF + wave * 64;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * 256), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * BK), LPTR(d + 512 + q * 256), 16, 0, 0);
  };

  const float* stile = reinterpret_cast<const float*>(smem + G4_RING);
  const float* srow[2] = {stile, stile};
  if constexpr (EPI == EPI_TRANS) {
    const int per = a.kscale / 4;
    const int64_t nroi = ((int64_t)a.M + a.P - 1) / a.P;
#pragma unroll
    for (int q = 0; q < G4_SQ; ++q) {
      const int p = q * 256 + tid;
      const int slot = min(p / per, G4_SLOTS - 1);
      const int64_t roi = min(roi_base + slot, nroi - 1);
      const float* src = a.scale + roi * a.kscale + (p % per) * 4;
      __builtin_amdgcn_global_load_lds(GPTR(src), LPTR(reinterpret_cast<uint4*>(smem + G4_RING) + q * 256 + wave * 64),
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
        const uint32_t d = lds_addr(ring + (kt % 3) * G4_BUF + tid);
        u32x4 v[2], s4[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          v[q] = lds_read128(d + q * 256 * 16);
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
          lds_write128(d + q * 256 * 16, o);
        }
      }
    }
  };

  const int fr = lane & 15, fc = lane >> 4;
  const int lterm = fr * 4 + (fc ^ x16(fr));
  const int aoff = (wr * 64) * 4 + lterm;            // + mt * 64
  const int boff = 512 + (wc * 128) * 4 + lterm;     // + nt * 64

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
  uint32_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (F & 32) {  // one dword per 128-B line of this tile's A rows (K x 2 B per row)
    const int lpr = a.K * 2 / 128;   // lines per row
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int l = tid + 256 * i;
      if (l < 128 * lpr) {
        const int64_t row = min(m0 + l / lpr, (int64_t)a.M - 1);
        const uint16_t* pa = Ag + row * a.lda + (l % lpr) * 64;
        asm volatile("global_load_dword %0, %1, off" : "+v"(pf[i]) : "v"(pa) : "memory");
      }
    }
  }
  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  transform(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (F & 32) {  // the prefetch loads are older than the DMA: retired by the wait above
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(pf[i]));
  }
  g4_barrier();

  // tile kt + 2's DMA is issued after step kt's MFMAs (its buffer was last read in
  // step kt - 1): the MFMAs start as soon as the fragments are read, and the DMA
  // issue -- which stalls while the memory pipeline is full -- runs beside them
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * G4_BUF;
    bf8v bfr[8], afr[4];
#pragma unroll
    for (int t = 0; t < 8; ++t) bfr[t] = *reinterpret_cast<const bf8v*>(buf + boff + t * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) afr[i] = *reinterpret_cast<const bf8v*>(buf + aoff + i * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (!(F & 8)) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[t], acc[i][t], 0, 0, 0);
    if (kt + 2 < nk) {
      __builtin_amdgcn_sched_barrier(0);
      issue(kt + 2);
    }
    if (kt + 1 < nk) {
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      transform(kt + 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_barrier();
  }

  if (prof) pst[1] = eg_stamp();
  if (F & 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(acc[i][t]));
    return;
  }
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
        if (!(F & 64)) v = hsw ? hswish2(v) : silu2(v);
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
  float* part = reinterpret_cast<float*>(smem + (EPI == EPI_DSC ? G4_STAGE : (size_t)0));  // [2][SLOTS][256]
  if (!(F & 128)) {
    const int64_t r0w = m0 + wr * 64;
    const int64_t roiw = r0w / a.P;
    const int wslot0 = (int)(roiw - roi_base);
    const int P = a.P;
    const int nxt0 = P - (int)(r0w - roiw * P);
    const bool full = r0w + 64 <= (int64_t)a.M;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      constexpr int WS = WIDE ? 2 : G4_WSLOTS, TS = WIDE ? 3 : G4_SLOTS;
      float ssum[WS];
#pragma unroll
      for (int q = 0; q < WS; ++q) ssum[q] = 0.f;
      int slot = 0, nxt = nxt0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f4v v = acc[k][t];
        if (full && nxt >= 16 * k + 16) {
          const float x = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
          for (int q = 0; q < WS; ++q)
            if (q == slot) ssum[q] += x;
        } else {
          float lo = 0.f, hi = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * k + fc * 4 + e;
            const float x = (r0w + row < a.M) ? v[e] : 0.f;
            if (row < nxt) lo += x;
            else hi += x;
          }
#pragma unroll
          for (int q = 0; q < WS; ++q) {
            if (q == slot) ssum[q] += lo;
            if (q == slot + 1) ssum[q] += hi;
          }
        }
        if (nxt <= 16 * k + 16) {
          ++slot;
          nxt += P;
        }
      }
#pragma unroll
      for (int q = 0; q < WS; ++q) {
        ssum[q] = sum_xor16(ssum[q]);
        ssum[q] = sum_xor32(ssum[q]);
      }
      if (lane < 16) {
#pragma unroll
        for (int ts = 0; ts < TS; ++ts) {
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < WS; ++q)
            if (q <= slot && wslot0 + q == ts) v = ssum[q];
          part[(wr * G4_SLOTS + ts) * 256 + colq + t * 16] = v;
        }
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
  if (!(F & 128)) {
    const int64_t last_row = min(m0 + 128, (int64_t)a.M) - 1;
    const int nslot = (int)(last_row / a.P - roi_base) + 1;
    for (int q = tid; q < nslot * 256; q += 256) {
      const int slot = q >> 8, c = q & 255;
      const int64_t roi = roi_base + slot;
      const int j = (int)(m0 / kPartRows - roi * a.P / kPartRows);
      a.sums[(roi * kPart + j) * a.ld_sums + g * a.N + n0 + c] =
          llrintf(part[slot * 256 + c] * kFix) + llrintf(part[(G4_SLOTS + slot) * 256 + c] * kFix);
    }
  }
  if (prof) pst[5] = eg_stamp();
  if (EPI == EPI_DSC && !(F & 256)) {
    const uint32_t* stage = reinterpret_cast<const uint32_t*>(smem);
    const int64_t cbase = (int64_t)g * a.N + n0;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int p = q * 256 + tid, rl = p >> 5, c8 = (p & 31) * 8;
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

template <int EPI, int F>
__global__ void __launch_bounds__(256, 2) g4lab_kernel(EncGemmArgs a, int64_t ntiles) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t lb = xcd_remap(blockIdx.x, ntiles);
  if (EPI == EPI_DSC && (lb % (a.N / 256 * a.groups)) / (a.N / 256) == 1) g4lab_tile<EPI, true, 1, F>(a, lb, smem);
  else g4lab_tile<EPI, true, 0, F>(a, lb, smem);
}
}  // namespace

template <int EPI, int F>
static int lab4(const EncGemmArgs& a, void* stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g4lab_kernel<EPI, F>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)G4_LDS);
    attr = true;
  }
  const int64_t nwg = ((int64_t)a.M + 127) / 128 * (a.N / 256) * a.groups;
  hipLaunchKernelGGL((g4lab_kernel<EPI, F>), dim3((unsigned)nwg), dim3(256), G4_LDS, reinterpret_cast<hipStream_t>(stream), a, nwg);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

#define LAB_CASES(E) \
  switch (flags) { \
    case 0: return lab4<E, 0>(a, stream); case 1: return lab4<E, 1>(a, stream); \
    case 2: return lab4<E, 2>(a, stream); case 3: return lab4<E, 3>(a, stream); \
    case 10: return lab4<E, 10>(a, stream); case 18: return lab4<E, 18>(a, stream); \
    case 32: return lab4<E, 32>(a, stream); case 34: return lab4<E, 34>(a, stream); \
    case 64: return lab4<E, 64>(a, stream); case 128: return lab4<E, 128>(a, stream); \
    case 256: return lab4<E, 256>(a, stream); case 192: return lab4<E, 192>(a, stream); \
    case 448: return lab4<E, 448>(a, stream); \
    default: return -1; }

extern "C" int lab_dsc(int flags, const void* Y2, int64_t M, int64_t P, const void* W2, const float* bias, void* XRN,
                       long long* sums, void* stream) {
  EncGemmArgs a{};
  a.A = (const uint16_t*)Y2; a.lda = 1024; a.B = (const uint16_t*)W2; a.bias = bias;
  a.C = (uint16_t*)XRN; a.ldc = 1024; a.sums = sums; a.ld_sums = 1024;
  a.M = (int)M; a.N = 512; a.K = 512; a.P = (int)P; a.groups = 2; a.kscale = 0;
  LAB_CASES(EPI_DSC)
}

extern "C" int lab_trans(int flags, const void* XRN, int64_t M, int64_t P, const float* s, const void* Wt,
                         const float* bias, long long* sums, void* stream) {
  EncGemmArgs a{};
  a.A = (const uint16_t*)XRN; a.lda = 1024; a.B = (const uint16_t*)Wt; a.bias = bias;
  a.sums = sums; a.ld_sums = 512; a.scale = s;
  a.M = (int)M; a.N = 512; a.K = 1024; a.P = (int)P; a.groups = 1; a.kscale = 512;
  LAB_CASES(EPI_TRANS)
}
