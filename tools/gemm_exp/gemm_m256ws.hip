// EXPERIMENT (tools/gemm_exp, round 6): batch-256 decode GEMM with WAVE-SPECIALISED operand streams.
//
// gemm_m256.hip (round 4) showed the 256-row decode GEMMs are bound by their LDS-DMA operand stream
// (~45 GB/s per CU) and that only two 48-KiB K-steps fit in flight: `vmcnt` retires a wave's loads
// in issue order, so a wave that issues both the activation (L2-resident) and the weight (HBM) DMA
// cannot keep the weight stream deeper than the activation stream. Here the two streams come from
// different waves, each with its own `vmcnt`: waves 0-3 move the activation K-steps (XS-stage ring,
// XS-1 in flight), waves 4-7 the weight K-steps (WS-stage ring, WS-1 in flight), optionally with the
// non-temporal policy (GM_NT: weights are read once per decode step). All 8 waves still compute
// (4 x 2 waves of 64 x 64, 32 MFMA 16x16x32 per K-step); one barrier per K-step. Same LDS image,
// swizzle and per-element MFMA order as gemm_big_kernel: outputs are bitwise gemm_big's.
//
// Build: GM_XS (2 / 3), GM_WS (4 / 6), GM_NT (0 / 1); tools/gemm_exp/build_m256ws.sh. GM_EXP=3 / 4:
// timing-only variants that stream only the activations / only the weights after the prologue.
#include "rt_common.h"

#ifndef GM_XS
#define GM_XS 3
#endif
#ifndef GM_WS
#define GM_WS 4
#endif
#ifndef GM_NT
#define GM_NT 0
#endif

namespace rt {

namespace gm {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int KS = 64;                 // K per step
constexpr int IMG_A = 256 * 128;       // activation image of one step: 256 rows x 128 B
constexpr int IMG_B = 128 * 128;       // weight image: 128 weight rows x 128 B
constexpr int XS = GM_XS, WS = GM_WS;
constexpr int LDS_BYTES = XS * IMG_A + WS * IMG_B;
static_assert(LDS_BYTES <= 163840, "LDS");

enum Epi { SLAB = 0, SWIGLU = 1 };

struct Args {
  const bf16_t* A; long lda;   // [M, K]
  const bf16_t* B; long ldb;   // [N, K] (SWIGLU: [gate; up], N = 2F)
  void* C; long ldc;           // SLAB: fp32 [nsplit][M][ldc]; SWIGLU: bf16 [M, ldc] (F columns)
  int M, N, K, nsplit;
};

__device__ __forceinline__ int row_swz(int row) { return (row >> 1) & 7; }

// wait until at most n of this wave's loads are outstanding (n a small run-time value)
template <int PER>
__device__ __forceinline__ void wait_vm(int n_steps) {
  switch (n_steps) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * PER) : "memory"); break;
  }
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_m256_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const ximg0 = smem;
  char* const wimg0 = smem + XS * IMG_A;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;  // wave rows 64 wm .., columns 64 wn ..
  const int frow = lane & 15, fq = lane >> 4;
  const int tn = blockIdx.x, split = blockIdx.y;
  const int n0 = tn * 128;
  const int F = p.N / 2;
  const int nk = p.K / KS;
  const int t_begin = (int)((long)split * nk / p.nsplit), t_end = (int)((long)(split + 1) * nk / p.nsplit);
  const bool xw = wid < 4;  // activation loader (waves 0-3) or weight loader (4-7)

  // LDS-DMA sources: one instruction moves 8 rows x 128 B (lane -> row + lane / 8, 16-B slot lane % 8
  // holding k-chunk slot ^ row_swz(row)). Activation waves: 8 instructions (64 rows) each; weight
  // waves: 4 instructions (32 weight rows) each.
  const bf16_t* src[8];
  const int lw = wid & 3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (xw) {
      const int row = (lw * 8 + j) * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ row_swz(row);
      src[j] = p.A + (long)min(row, p.M - 1) * p.lda + kc * 8;
    } else {
      const int row = ((lw * 4 + (j & 3)) * 8 + (lane >> 3));
      const int kc = (lane & 7) ^ row_swz(row);
      const int wrow = EPI == SWIGLU ? (row < 64 ? tn * 64 + row : F + tn * 64 + row - 64) : n0 + row;
      src[j] = p.B + (long)wrow * p.ldb + kc * 8;
    }
  }
  auto stage_x = [&](int t) {
#if defined(GM_EXP) && GM_EXP == 4
    if (t >= t_begin + XS - 1) return;  // experiment: weight stream only (stale activations)
#endif
    char* img = ximg0 + (t % XS) * IMG_A;
    const long adv = (long)t * KS;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(src[j] + adv), (lds_void*)(img + (lw * 8 + j) * 1024), 16, 0, 0);
  };
  auto stage_w = [&](int t) {
#if defined(GM_EXP) && GM_EXP == 3
    if (t >= t_begin + WS - 1) return;  // experiment: activation stream only (stale weights)
#endif
    char* img = wimg0 + (t % WS) * IMG_B;
    const long adv = (long)t * KS;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(src[j] + adv), (lds_void*)(img + (lw * 4 + j) * 1024), 16, 0,
                                       GM_NT ? 2 : 0);
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

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t_begin < t_end) {
    if (xw) {
      for (int s = 0; s < XS - 1 && t_begin + s < t_end; ++s) stage_x(t_begin + s);
    } else {
      for (int s = 0; s < WS - 1 && t_begin + s < t_end; ++s) stage_w(t_begin + s);
    }
    for (int t = t_begin; t < t_end; ++t) {
      // retire this wave's DMA of step t; later steps of its own stream may stay in flight
      if (xw) wait_vm<8>(min(XS - 2, t_end - 1 - t));
      else wait_vm<4>(min(WS - 2, t_end - 1 - t));
      asm volatile("s_barrier" ::: "memory");
      // the barrier also closed every wave's reads of step t - 1, whose stages these refill
      if (xw) {
        if (t + XS - 1 < t_end) stage_x(t + XS - 1);
      } else {
        if (t + WS - 1 < t_end) stage_w(t + WS - 1);
      }
      const char* ximg = ximg0 + (t % XS) * IMG_A;
      const char* wimg = wimg0 + (t % WS) * IMG_B;
      i32x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = rd_row(ximg, wm * 64 + i * 16 + frow);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = rd_row(wimg, wn * 64 + j * 16 + frow);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(fb[j], kk), half(fa[i], kk), acc[i][j], 0, 0, 0);
    }
  }

  if constexpr (EPI == SLAB) {
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
    const int cc = tid & 7;
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
