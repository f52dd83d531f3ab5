// Experiment harness (not product code): bf16 NT GEMM C[M,N] = A[M,K] . B[N,K]^T + bias
// on MFMA 32x32x16, BM=128, BK=32, 8 waves (2 x 4), register-staged double buffer.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t nx = 8;
  if (nwg < nx) return bid;
  int64_t q = nwg / nx, r = nwg % nx, x = bid % nx;
  int64_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + bid / nx;
}

template <int BN, int EPI, int BKT, bool SWAP>
__global__ void __launch_bounds__(512) gemm(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                           const float* __restrict__ bias, uint16_t* __restrict__ Cm, int M,
                                           int N, int K) {
  constexpr int BM = 128, BK = BKT, LDK = BK + 8;  // padded LDS row
  constexpr int WN = BN / 4, TM = 2, TN = WN / 32;
  constexpr int BPC = BN * BK / 8 / 512;           // B pieces per thread
  __shared__ __align__(16) uint16_t As[2][BM * LDK];
  __shared__ __align__(16) uint16_t Bs[2][BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int ntn = N / BN;
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (int)(lb / ntn), nt = (int)(lb % ntn);
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  // staging coordinates
  constexpr int KP = BK / 8;                   // 16-B pieces per row
  constexpr int APC = BM * KP / 512;
  uint4 ra[APC], rb[BPC];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < APC; ++i) {
      const int q = tid + 512 * i, r = q / KP, kk = (q % KP) * 8;
      ra[i] = *reinterpret_cast<const uint4*>(A + (m0 + r) * K + k0 + kk);
    }
#pragma unroll
    for (int i = 0; i < BPC; ++i) {
      const int q = tid + 512 * i, br = q / KP, bk = (q % KP) * 8;
      rb[i] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + br) * K + k0 + bk);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APC; ++i) {
      const int q = tid + 512 * i, r = q / KP, kk = (q % KP) * 8;
      *reinterpret_cast<uint4*>(&As[buf][r * LDK + kk]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BPC; ++i) {
      const int q = tid + 512 * i, br = q / KP, bk = (q % KP) * 8;
      *reinterpret_cast<uint4*>(&Bs[buf][br * LDK + bk]) = rb[i];
    }
  };
  f16v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  gload(0);
  swrite(0);
  __syncthreads();
  const int nk = K / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf8 af[TM], bfr[TN];
      const int kk = ks * 16 + 8 * (lane >> 5);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf8*>(&As[buf][(wm * 64 + i * 32 + (lane & 31)) * LDK + kk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf8*>(&Bs[buf][(wn * WN + j * 32 + (lane & 31)) * LDK + kk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(buf ^ 1);
    __syncthreads();
  }
  // epilogue
  if (EPI == 2) {  // no store (K-loop timing): keep the accumulators alive
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    if (t == 1234.5f) Cm[0] = 1;
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!SWAP) {  // lane = column, registers = rows: 2-B stores
        const int col = n0 + wn * WN + j * 32 + (lane & 31);
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          Cm[(m0 + row) * N + col] = f2bf(acc[i][j][r] + bv);
        }
      } else {      // lane = row, registers = 4-column groups: 8-B stores
        const int64_t row = m0 + wm * 64 + i * 32 + (lane & 31);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = n0 + wn * WN + j * 32 + 8 * g + 4 * (lane >> 5);
          const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0, 0, 0, 0);
          uint2 pk;
          pk.x = (uint32_t)f2bf(acc[i][j][4 * g + 0] + bv.x) | ((uint32_t)f2bf(acc[i][j][4 * g + 1] + bv.y) << 16);
          pk.y = (uint32_t)f2bf(acc[i][j][4 * g + 2] + bv.z) | ((uint32_t)f2bf(acc[i][j][4 * g + 3] + bv.w) << 16);
          *reinterpret_cast<uint2*>(Cm + row * N + col) = pk;
        }
      }
    }
}

template <int BN, int EPI, int BK, bool SW>
static float run_t(const void* A, const void* B, const float* bias, void* C, int M, int N, int K, int reps) {
  const int nwg = (M / 128) * (N / BN);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((gemm<BN, EPI, BK, SW>), dim3(nwg), dim3(512), 0, 0, (const uint16_t*)A, (const uint16_t*)B,
                     bias, (uint16_t*)C, M, N, K);
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gemm<BN, EPI, BK, SW>), dim3(nwg), dim3(512), 0, 0, (const uint16_t*)A,
                       (const uint16_t*)B, bias, (uint16_t*)C, M, N, K);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

extern "C" float gemm_run(int bn, int epi, int bk, int sw, const void* A, const void* B, const float* bias, void* C,
                          int M, int N, int K, int reps) {
#define V(BN_, E_, BK_, SW_) \
  if (bn == BN_ && epi == E_ && bk == BK_ && sw == SW_) return run_t<BN_, E_, BK_, SW_>(A, B, bias, C, M, N, K, reps);
  V(128, 0, 32, 0) V(128, 0, 32, 1) V(128, 2, 32, 0) V(128, 0, 64, 0) V(128, 0, 64, 1) V(128, 2, 64, 0)
  V(256, 0, 32, 1) V(256, 2, 32, 0) V(256, 0, 64, 1) V(256, 2, 64, 0)
  return -1.f;
}
