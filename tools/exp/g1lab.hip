// g1dw4 laboratory (diagnostics, not product code): the product's g1dw4 kernel with
// switches, built beside the product into tools/exp/libg1lab.so
//   F & 1   every workgroup reads M tile 0's rows (A always L2-resident)
//   F & 2   stop after the K loop (no depthwise, no Y2 stores)
//   F & 4   depthwise, Y2 stores into a 1-tile scratch (every workgroup the same rows)
//   F & 8   no MFMAs          F & 16  no operand DMA
#include "../../a-lightweight-unsupervised-feature-extractor-_amd/csrc/enc_gemm.hip"
namespace {
template <int QY, int QX, int YS, int MODE>
__device__ __forceinline__ void dw5q_lab(const uint32_t* __restrict__ src, const dw_pair_t (&w)[25],
                                          uint32_t* __restrict__ dst, int ldd) {
  constexpr int OY0 = 5 * QY, X0 = 5 * QX;
  constexpr int IY0 = OY0 - 2 < 0 ? 0 : OY0 - 2, IY1 = OY0 + 6 > G1_S - 1 ? G1_S - 1 : OY0 + 6;
  constexpr int IX0 = X0 - 2 < 0 ? 0 : X0 - 2, IX1 = X0 + 6 > G1_S - 1 ? G1_S - 1 : X0 + 6;
  constexpr int NX = IX1 - IX0 + 1;
  dw_pair_t acc[5][5];
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) acc[oy][ox] = dw_pair_t{0.f, 0.f};
  uint32_t nxt[NX];
#pragma unroll
  for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[(IY0 * G1_S + IX0 + ix) * YS];
#pragma unroll
  for (int iy = IY0; iy <= IY1; ++iy) {
    dw_pair_t in[NX];
#pragma unroll
    for (int ix = 0; ix < NX; ++ix) in[ix] = dw_pair_t{__uint_as_float(nxt[ix] << 16), __uint_as_float(nxt[ix] & 0xffff0000u)};
    if (iy < IY1) {
#pragma unroll
      for (int ix = 0; ix < NX; ++ix) nxt[ix] = src[((iy + 1) * G1_S + IX0 + ix) * YS];
    }
    // groups of up to 5 independent FMAs (the 5 outputs of a row for one tap), each group
    // closed by an empty asm on its accumulators: left to itself the compiler ran every
    // output's taps as one dependent chain (an s_nop between dependent v_pk_fma_f32) at 2
    // waves per SIMD (a sched_barrier alone does not hold: the FMAs have no chain edge)
#pragma unroll
    for (int oy = 0; oy < 5; ++oy) {
      const int ky = iy - (OY0 + oy) + 2;
      if (ky < 0 || ky > 4) continue;
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
#pragma unroll
        for (int ox = 0; ox < 5; ++ox) {
          const int ix = X0 + ox + kx - 2;
          if (ix >= IX0 && ix <= IX1)
            acc[oy][ox] = MODE == 2 ? in[ix - IX0] : __builtin_elementwise_fma(w[ky * 5 + kx], in[ix - IX0], acc[oy][ox]);
        }
        asm volatile("" : "+v"(acc[oy][0]), "+v"(acc[oy][1]), "+v"(acc[oy][2]), "+v"(acc[oy][3]), "+v"(acc[oy][4]));
      }
    }
  }
#pragma unroll
  for (int oy = 0; oy < 5; ++oy)
#pragma unroll
    for (int ox = 0; ox < 5; ++ox) {
      const uint32_t v = pack_bf16x2(acc[oy][ox].x, acc[oy][ox].y);
      if (MODE == 1) asm volatile("" ::"v"(v));
      else dst[((OY0 + oy) * G1_S + X0 + ox) * ldd] = v;
    }
}

template <int F>
__global__ void __launch_bounds__(256, 2) g1lab_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W1,
                                                        const float* __restrict__ wdw, uint16_t* __restrict__ Y2,
                                                        int M, int N) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntile_n = N / G1_BN;
  const int n0 = (int)(lb % ntile_n) * G1_BN;
  const int64_t m0 = (lb / ntile_n) * (2 * G1_P);
  constexpr int K = 512, NK = K / BK;

  // DMA: A slots p = q * 256 + tid (q = 0..2 every wave, q = 3 wave 0 only: 832 slots),
  // B slots 832 + q * 256 + tid (q = 0, 1); slot p holds row p >> 2, chunk (p & 3) ^ x16(row)
  const uint16_t* asrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = min(q * 256 + tid, G1Q_AP - 1), r = p >> 2, c = (p & 3) ^ x16(r);
    asrc[q] = X + ((F & 1) ? (int64_t)r : min(m0 + r, (int64_t)M - 1)) * K + c * 8;
  }
  const uint16_t* bsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 256 + tid, r = p >> 2, c = (p & 3) ^ x16(r);
    bsrc[q] = W1 + (int64_t)(n0 + r) * K + c * 8;
  }
  auto issue = [&](int kt) {
    if (F & 16) return;
    uint4* d = ring + (kt % 3) * G1Q_BUF + wave * 64;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(asrc[q] + kt * BK), LPTR(d + q * 256), 16, 0, 0);
    if (wave == 0) __builtin_amdgcn_global_load_lds(GPTR(asrc[3] + kt * BK), LPTR(d + 3 * 256), 16, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(GPTR(bsrc[q] + kt * BK), LPTR(d + G1Q_AP + q * 256), 16, 0, 0);
  };
  // retire all but the newest stage's DMA ops (wave 0 issues 6 per stage, the others 5)
  auto wait_prev = [&]() {
    if (F & 16) return;
    if (wave == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  };

  const int fr = lane & 15, fc = lane >> 4;
  const int lterm = fr * 4 + (fc ^ x16(fr));
  const int aoff = (wr * 112) * 4 + lterm;           // + i * 64
  const int boff = G1Q_AP + (wc * 64) * 4 + lterm;   // + t * 64
  const int ntm = wr == 0 ? 7 : 6;

  f4v acc[7][4];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};

  const int nk = NK;
  issue(0);
  issue(1);
  wait_prev();
  g4_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const uint4* buf = ring + (kt % 3) * G1Q_BUF;
    {
      // 11 fragment reads up front (wr = 1's seventh reads B slots, unused), then counted
      // lgkmcnt waits: row tile i's MFMAs start once its A fragment has landed
      const uint32_t bb = lds_addr(buf + boff), ab = lds_addr(buf + aoff);
      u32x4 bq[4], aq[7];
#pragma unroll
      for (int t = 0; t < 4; ++t) bq[t] = lds_read128(bb + t * 1024);
#pragma unroll
      for (int i = 0; i < 7; ++i) aq[i] = lds_read128(ab + i * 1024);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        __builtin_amdgcn_sched_barrier(0);  // keep each wait in front of its own row tile's MFMAs
        if (i == 0) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(aq[0]));
        else if (i == 1) asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(aq[1]));
        else if (i == 2) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(aq[2]));
        else if (i == 3) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(aq[3]));
        else if (i == 4) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(aq[4]));
        else if (i == 5) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(aq[5]));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aq[6]));
        if (i < ntm && !(F & 8)) {
          const bf8v a = __builtin_bit_cast(bf8v, aq[i]);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8v, bq[t]), acc[i][t], 0, 0, 0);
        }
      }
    }
    if (kt + 2 < nk) {
      __builtin_amdgcn_sched_barrier(0);
      issue(kt + 2);
    }
    if (kt + 1 < nk) {
      if (kt + 2 < nk) wait_prev();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_barrier();
  }

  if (F & 2) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) asm volatile("" ::"v"(acc[i][t]));
    return;
  }
  // depthwise weights: every wave needs the same 25 taps of its lane's channel pair, so
  // each lane loads them straight into registers (issued now, used after the Y1 writes)
  dw_pair_t wreg[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) wreg[k] = *reinterpret_cast<const dw_pair_t*>(wdw + (int64_t)k * N + n0 + 2 * lane);
  // Y1 (bf16 pairs, rows < 200) -> LDS [200][64]: lane pairs (fr, fr ^ 1) trade values so each
  // lane writes two column pairs: even fr rows +0, +1, odd fr rows +2, +3 (as gemm4's staging)
  uint32_t* y1 = reinterpret_cast<uint32_t*>(smem);
  {
    const bool odd = fr & 1;
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if (i < ntm)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f4v v = acc[i][t];
          const float x0 = lane_xor1(odd ? v[0] : v[2]);
          const float x1 = lane_xor1(odd ? v[1] : v[3]);
          const int rb = wr * 112 + i * 16 + fc * 4 + (odd ? 2 : 0);
          const int cp = (wc * 64 + t * 16 + fr) >> 1;
          if (rb < 2 * G1_P) y1[rb * G1Q_YS + cp] = odd ? pack_bf16x2(x0, v[2]) : pack_bf16x2(v[0], x0);
          if (rb + 1 < 2 * G1_P) y1[(rb + 1) * G1Q_YS + cp] = odd ? pack_bf16x2(x1, v[3]) : pack_bf16x2(v[1], x1);
        }
  }
  __syncthreads();
  if (F & 64) return;

  // depthwise 5x5: wave = output quadrant, for each of the two ROIs; lane = channel pair
  const int ldd = N / 2;
  if (F & 4) { (void)ldd; }
#pragma unroll 1
  for (int roi = 0; roi < 2; ++roi) {
    const int64_t rbase = m0 + roi * G1_P;
    if (rbase >= M) break;
    int l = ldd;
    asm volatile("" : "+s"(l));  // per ROI: keeps the 25 store offsets out of the loop (SGPR spills)
    const uint32_t* src = y1 + roi * G1_P * G1Q_YS + lane;
    uint32_t* dst = reinterpret_cast<uint32_t*>(Y2 + ((F & 128) ? (int64_t)roi * G1_P : rbase) * N + n0) + lane;
    constexpr int MD = (F & 4) ? 1 : (F & 32) ? 2 : 0;
    switch (wave) {
      case 0: dw5q_lab<0, 0, G1Q_YS, MD>(src, wreg, dst, l); break;
      case 1: dw5q_lab<0, 1, G1Q_YS, MD>(src, wreg, dst, l); break;
      case 2: dw5q_lab<1, 0, G1Q_YS, MD>(src, wreg, dst, l); break;
      default: dw5q_lab<1, 1, G1Q_YS, MD>(src, wreg, dst, l); break;
    }
  }
}

}  // namespace

template <int F>
static int lab_launch(const void* X, int64_t M, const void* W1, int64_t N, const float* wdw, void* Y2, void* stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(g1lab_kernel<F>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)G1Q_LDS);
    attr = true;
  }
  const int64_t nwg = (M / 200 + (M % 200 ? 1 : 0)) * (N / 128);
  hipLaunchKernelGGL(g1lab_kernel<F>, dim3((unsigned)nwg), dim3(256), G1Q_LDS, reinterpret_cast<hipStream_t>(stream),
                     (const uint16_t*)X, (const uint16_t*)W1, wdw, (uint16_t*)Y2, (int)M, (int)N);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int lab_g1(int flags, const void* X, int64_t M, const void* W1, int64_t N, const float* wdw, void* Y2,
                      void* stream) {
  switch (flags) {
    case 0: return lab_launch<0>(X, M, W1, N, wdw, Y2, stream);
    case 1: return lab_launch<1>(X, M, W1, N, wdw, Y2, stream);
    case 2: return lab_launch<2>(X, M, W1, N, wdw, Y2, stream);
    case 3: return lab_launch<3>(X, M, W1, N, wdw, Y2, stream);
    case 10: return lab_launch<10>(X, M, W1, N, wdw, Y2, stream);
    case 18: return lab_launch<18>(X, M, W1, N, wdw, Y2, stream);
    case 19: return lab_launch<19>(X, M, W1, N, wdw, Y2, stream);
    case 4: return lab_launch<4>(X, M, W1, N, wdw, Y2, stream);
    case 32: return lab_launch<32>(X, M, W1, N, wdw, Y2, stream);
    case 64: return lab_launch<64>(X, M, W1, N, wdw, Y2, stream);
    case 128: return lab_launch<128>(X, M, W1, N, wdw, Y2, stream);
    case 129: return lab_launch<129>(X, M, W1, N, wdw, Y2, stream);
    default: return -1;
  }
}
