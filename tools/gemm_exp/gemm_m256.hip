// EXPERIMENT (tools/gemm_exp, not part of the extension): a batch-256 decode GEMM (M <= 256, NT:
// activations [M, K] x weight [N, K]^T) with ONE barrier-bracketed section per K-step, against
// the production form on gemm_big_kernel (256 x 128 tiles, four phases of 8 MFMAs per wave per
// K-step, each between two barriers, the two wave groups staggered). Split-K fp32 slabs (qkv / o /
// down of the rollout decode step) or the SwiGLU epilogue (gate / up).
//
// Here: a barrier, the LDS-DMA issue of the step two ahead, 16 ds_read_b128 per wave and 32 MFMAs
// that start as their fragments land. Three K-step stages (3 x 48 KiB LDS; one workgroup of 8
// waves per CU), waves 4 (M) x 2 (N) of 64 x 64 — a fifth less LDS read per MAC than 128 x 32.
// Same LDS image, source-side swizzle and per-element MFMA order as gemm_big_kernel: the slabs and
// the SwiGLU output are bitwise gemm_big's.
//
// Result (profiles/r4/m256_one_section_kernel_ab.log, tools/gemm_exp/m256_main.cpp): the same time
// within noise (qkv 21.1 vs 22.0 us, o 16.5 vs 17.9, down 39.4 vs 39.5, gate_up 74.1 vs 72.2). With
// the MFMAs removed (GM_EXP=1) the operand stream alone takes 17.4 / 14.6 / 37.8 / 67.5 us; with the
// LDS-DMA removed after the prologue (GM_EXP=2) reads + MFMAs alone take 18.1 / 14.4 / 31.0 / 56.5.
// Both halves are within 10-25 % of the whole, so the schedule is not what bounds these GEMMs: the
// LDS-DMA stream runs at ~45 GB/s per CU against the ~68 GB/s per CU the microarchitecture guide
// measured for a loader-only ring (MI355X_MICROARCH.md 'ring-gemm'), and at 256 rows only two
// K-steps (96 KiB) fit in flight. Not adopted.
#include "rt_common.h"

namespace rt {

namespace gm {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int KS = 64;                 // K per step
constexpr int IMG_A = 256 * 128;       // A image of one step: 256 rows x 128 B
constexpr int IMG_B = 128 * 128;       // B image: 128 weight rows x 128 B
constexpr int STAGE = IMG_A + IMG_B;   // 48 KiB
constexpr int NSTAGE = 3;

enum Epi { SLAB = 0, SWIGLU = 1 };

struct Args {
  const bf16_t* A; long lda;   // [M, K]
  const bf16_t* B; long ldb;   // [N, K] (SWIGLU: [gate; up], N = 2F)
  void* C; long ldc;           // SLAB: fp32 [nsplit][M][ldc]; SWIGLU: bf16 [M, ldc] (F columns)
  int M, N, K, nsplit;
};

__device__ __forceinline__ int row_swz(int row) { return (row >> 1) & 7; }

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_m256_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;  // wave rows 64 wm .., columns 64 wn ..
  const int frow = lane & 15, fq = lane >> 4;
  const int tn = blockIdx.x, split = blockIdx.y;
  const int n0 = tn * 128;
  const int F = p.N / 2;
  const int nk = p.K / KS;
  const int t_begin = (int)((long)split * nk / p.nsplit), t_end = (int)((long)(split + 1) * nk / p.nsplit);

  // ---- LDS-DMA sources: instruction j of this wave moves 8 rows x 128 B (lane -> row + lane / 8,
  // 16-B slot lane % 8 holding k-chunk slot ^ row_swz(row)); A: 4 per wave, B: 2 per wave ----
  const bf16_t* srcA[4];
  const bf16_t* srcB[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (wid * 4 + j) * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ row_swz(row);
    srcA[j] = p.A + (long)min(row, p.M - 1) * p.lda + kc * 8;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wid * 2 + j) * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ row_swz(row);
    const int wrow = EPI == SWIGLU ? (row < 64 ? tn * 64 + row : F + tn * 64 + row - 64) : n0 + row;
    srcB[j] = p.B + (long)wrow * p.ldb + kc * 8;
  }
  auto stage = [&](int t) {
#if defined(GM_EXP) && GM_EXP == 2
    if (t >= 2) return;  // experiment: no operand traffic after the prologue (stale LDS)
#endif
    char* img = smem + (t % NSTAGE) * STAGE;
    const long adv = (long)t * KS;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + adv), (lds_void*)(img + (wid * 4 + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + adv), (lds_void*)(img + IMG_A + (wid * 2 + j) * 1024), 16,
                                       0, 0);
  };
  auto rd_row = [&](const char* img, int row) -> i32x8 {
    const i32x4 lo = *(const i32x4*)(img + row * 128 + ((fq ^ row_swz(row)) << 4));
    const i32x4 hi = *(const i32x4*)(img + row * 128 + (((4 + fq) ^ row_swz(row)) << 4));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto half = [](const i32x8& v, int h) -> bf16x8 {
    return h == 0 ? __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3))
                  : __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
  };

  // acc[i][j][r] = C[64 wm + 16 i + frow][64 wn + 16 j + 4 fq + r] (weight fragment as the MFMA's
  // A operand: each lane owns 4 consecutive output columns of one row)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t_begin < t_end) {
    stage(t_begin);
    if (t_begin + 1 < t_end) stage(t_begin + 1);
    for (int t = t_begin; t < t_end; ++t) {
      // retire this wave's DMA of step t (step t + 1's 6 instructions may stay in flight); the
      // barrier publishes every wave's step-t rows and closes every wave's reads of step t - 1,
      // whose stage the DMA of step t + 2 then overwrites
      if (t + 1 < t_end) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      if (t + 2 < t_end) stage(t + 2);
      const char* img = smem + (t % NSTAGE) * STAGE;
      i32x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = rd_row(img, wm * 64 + i * 16 + frow);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = rd_row(img + IMG_A, wn * 64 + j * 16 + frow);
#if defined(GM_EXP) && GM_EXP == 1
      // experiment: no MFMAs (fragments folded into one accumulator lane so the reads stay live)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][0][0] += __builtin_bit_cast(float, fa[i][0] ^ fb[i][0]);
#else
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(fb[j], kk), half(fa[i], kk), acc[i][j], 0, 0, 0);
#endif
    }
  }

  if constexpr (EPI == SLAB) {
    // every split writes its whole slab (a split with no K-steps writes zeros)
    float* C = (float*)p.C + (long)split * p.M * p.ldc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + frow;
      if (row < p.M) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = n0 + wn * 64 + j * 16 + fq * 4;
          float4 v;
          v.x = acc[i][j][0]; v.y = acc[i][j][1]; v.z = acc[i][j][2]; v.w = acc[i][j][3];
          *(float4*)(C + (long)row * p.ldc + col) = v;
        }
      }
    }
  } else {
    // gate (tile columns 0-63) and up (64-127) rounded to bf16 through LDS, then f = silu(g) * u
    // in fp32 (the arithmetic of gemm_big_kernel's E_SWIGLU epilogue)
    constexpr int LDT = 128 + 8;
    bf16_t* tile = (bf16_t*)smem;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 64 + i * 16 + frow, col = wn * 64 + j * 16 + fq * 4;
        *(uint2*)(tile + row * LDT + col) =
            make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3]));
      }
    __syncthreads();
    bf16_t* Cf = (bf16_t*)p.C;
    const int cc = tid & 7;  // 8-column chunk of the 64 gate columns
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int row = pass * 64 + (tid >> 3);
      if (row < p.M) {
        const uint4 g4 = *(const uint4*)(tile + row * LDT + cc * 8);
        const uint4 u4 = *(const uint4*)(tile + row * LDT + 64 + cc * 8);
        float g[8], u[8], f[8];
        unpack8(g4, g);
        unpack8(u4, u);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = g[e] / (1.f + __expf(-g[e])) * u[e];
        *(uint4*)(Cf + (long)row * p.ldc + tn * 64 + cc * 8) = pack8(f);
      }
    }
  }
}

}  // namespace gm

}  // namespace rt

using namespace rt;

// C = split-K fp32 slabs of A B^T (epi 0: C [nsplit][M][ldc]) or silu(A Bg^T) * (A Bu^T) bf16
// (epi 1: B = [gate; up] with N = 2F rows, C [M, ldc], F columns). Requirements: 1 <= M <= 256,
// K % 64 == 0, N % 128 == 0, 16-B aligned rows (lda, ldb % 8 == 0), ldc % 4 (slab) / % 8 (bf16).
extern "C" int rt_gemm_m256(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int nsplit, int epi, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 256 || K % gm::KS || N % 128 || lda % 8 || ldb % 8 || nsplit < 1 || (epi != 0 && epi != 1)) return -1;
  if (epi == 0 && (ldc % 4 || ldc < N)) return -2;
  if (epi == 1 && (nsplit != 1 || ldc % 8 || ldc < N / 2)) return -3;
  gm::Args p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K; p.nsplit = nsplit;
  const dim3 grid(N / 128, nsplit), block(512);
  if (epi == 0) hipLaunchKernelGGL((gm::gemm_m256_kernel<gm::SLAB>), grid, block, 0, stream, p);
  else hipLaunchKernelGGL((gm::gemm_m256_kernel<gm::SWIGLU>), grid, block, 0, stream, p);
  return (int)hipGetLastError();
}
