// Experiment (round 5): the 256x256 NT GEMM with the B operand (the weight) streamed straight
// into VGPRs from an MFMA-fragment-ordered image, so B never touches LDS; A keeps the LDS-DMA
// granules of gemm_big (four K-step buffers, 128 KiB). Timing + bitwise check against gemm_big in
// tools/gemm_exp/bd_main.cpp. NT only (A [M][K], W [N][K]), bf16 out, no epilogue variants,
// N % 256 == 0, K % 64 == 0.
//
// Fragment image (bd_shuffle): for every 16-row block nb of W and K-step ks, 2 KiB laid out
// [kk half][lane][8 bf16] = W[16 nb + lane % 16][64 ks + 32 kk + 8 (lane / 16) + e], i.e. exactly
// the 32 B per lane a 16x16x32 MFMA fragment pair holds; one buffer_load_dwordx4 per wave reads a
// contiguous 1 KiB.
//
// Per wave and K-step t (8 waves, 2 x 4, 128 x 64 outputs each, the phase order of gemm_big):
//   p1: read a0(t) from LDS; issue B(t+1) (8 loads into the other register set); issue a0(t+2)
//   p2: issue a1(t+2)
//   p3: read a1(t) from LDS
//   p4: retire a0 / a1 (t+1) (counted vmcnt: younger are B(t+1) and A(t+2))
// B(t) was issued a whole step earlier; hipcc places the wait for it before its first MFMA.
#include "rt_common.h"

namespace bd {
using namespace rt;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int ABUF = 32768;  // A image of one K-step (256 rows x 64 k)

__device__ __forceinline__ int row_swz(int row) { return (row >> 1) & 7; }

#define BD_BARRIER() asm volatile("s_barrier" ::: "memory")

__global__ __launch_bounds__(512, 2) void bd_kernel(const bf16_t* __restrict__ A, long lda,
                                                   const bf16_t* __restrict__ Bimg, bf16_t* __restrict__ C,
                                                   long ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[4 * ABUF];
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256, nwg = tiles_m * tiles_n;
  const int nk = K / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int frow = lane & 15, fq = lane >> 4;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int GM = 4;
  const int group = bid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (bid % gsz);
  const int tn = (bid % (GM * tiles_n)) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  // ---- A: LDS-DMA granules (gemm_big's ROW geometry, op 0) ----
  uint32_t aoff[2][2];
  int adst[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o = wid * 2 + j;
      const int rb = (o >> 3) * 128 + s * 64 + (o & 7) * 8;
      const int row = rb + (lane >> 3);
      const int kc = (lane & 7) ^ row_swz(row);
      aoff[s][j] = (uint32_t)min(m0 + row, M - 1) * (uint32_t)lda + (uint32_t)(kc * 8);
      adst[s][j] = rb * 128;
    }
  auto stage_a = [&](int s, int t) {
    const bf16_t* base = A + (long)t * 64;
    char* img = smem + (t & 3) * ABUF;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(base + aoff[s][j]), (lds_void*)(img + adst[s][j]), 16, 0, 0);
  };
  i32x8 fa[4];
  auto read_a = [&](int t, int s) {
    const char* img = smem + (t & 3) * ABUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 128 + s * 64 + i * 16 + frow;
      const i32x4 lo = *(const i32x4*)(img + row * 128 + ((fq ^ row_swz(row)) << 4));
      const i32x4 hi = *(const i32x4*)(img + row * 128 + (((4 + fq) ^ row_swz(row)) << 4));
      fa[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };

  // ---- B: fragment image -> VGPRs (asm loads: absent from hipcc's wait bookkeeping, so the
  // only waits are the counted ones below; form (ii) of the guide: the wait statement names every
  // destination "+v") ----
  const uint32_t bptr_lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)Bimg);
  const uint32_t bptr_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)Bimg >> 32));
  const int nbytes = __builtin_amdgcn_readfirstlane((int)((long)N * K * 2));
  const i32x4 brs = {(int)bptr_lo, (int)(bptr_hi & 0xFFFF), nbytes, 0x00020000};
  const int voff = lane * 16;
  const int nb0 = __builtin_amdgcn_readfirstlane(n0 / 16 + wc * 4);
  // fb[s][j][kk]: B sub-block s, fragment j, k half kk
  auto load_b = [&](int t, i32x4 (&fb)[2][2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#if BD_HOT  // diagnostic: every step re-reads the K-step-0 fragments (L1 / L2 resident, wrong C)
        const int so = __builtin_amdgcn_readfirstlane(((nb0 + s * 2 + j) * nk + 0 * t) * 2048);
#else
        const int so = __builtin_amdgcn_readfirstlane(((nb0 + s * 2 + j) * nk + t) * 2048);
#endif
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(fb[s][j][0]) : "v"(voff), "s"(brs), "s"(so));
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:1024" : "=v"(fb[s][j][1]) : "v"(voff), "s"(brs), "s"(so));
      }
  };
#define BD_WAIT_B(N, FB)                                                                     \
  asm volatile("s_waitcnt vmcnt(" #N ")"                                                    \
               : "+v"(FB[0][0][0]), "+v"(FB[0][0][1]), "+v"(FB[0][1][0]), "+v"(FB[0][1][1]), \
                 "+v"(FB[1][0][0]), "+v"(FB[1][0][1]), "+v"(FB[1][1][0]), "+v"(FB[1][1][1])  \
               :: "memory")
  auto half = [](const i32x8& v, int h) -> bf16x8 {
    return h == 0 ? __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3))
                  : __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
  };
  auto bh = [](const i32x4& v) -> bf16x8 { return __builtin_bit_cast(bf16x8, v); };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define BD_MMA(SA, SB, FB)                                                                   \
  do {                                                                                      \
    BD_BARRIER();                                                                           \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    __builtin_amdgcn_s_setprio(1);                                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                           \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                         \
        _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                    \
          acc[(SA) * 4 + i][(SB) * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(         \
              bh(FB[(SB)][j][kk]), half(fa[i], kk), acc[(SA) * 4 + i][(SB) * 2 + j], 0, 0, 0); \
    __builtin_amdgcn_s_setprio(0);                                                          \
    BD_BARRIER();                                                                           \
  } while (0)

#define BD_STEP(T, CB, NB)                                                                   \
  do {                                                                                      \
    const int t_ = (T);                                                                     \
    const bool n1 = t_ + 1 < nk, n2 = t_ + 2 < nk;                                          \
    read_a(t_, 0);                                                                          \
    if (n1) load_b(t_ + 1, NB);                                                             \
    if (n2) stage_a(0, t_ + 2);                                                             \
    BD_WAIT_B(0, CB);                                                                       \
    BD_MMA(0, 0, CB);                                                                       \
    if (n2) stage_a(1, t_ + 2);                                                             \
    BD_MMA(0, 1, CB);                                                                       \
    read_a(t_, 1);                                                                          \
    BD_MMA(1, 1, CB);                                                                       \
    if (n1) {                                                                               \
      if (n2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");                             \
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                                 \
    }                                                                                       \
    BD_MMA(1, 0, CB);                                                                       \
  } while (0)

#define BD_FAST(T, CB, NB)                                                                   \
  do {                                                                                      \
    const int t_ = (T);                                                                     \
    read_a(t_, 0);                                                                          \
    load_b(t_ + 1, NB);                                                                     \
    stage_a(0, t_ + 2);                                                                     \
    BD_WAIT_B(14, CB);                                                                      \
    BD_MMA(0, 0, CB);                                                                       \
    stage_a(1, t_ + 2);                                                                     \
    BD_MMA(0, 1, CB);                                                                       \
    read_a(t_, 1);                                                                          \
    BD_MMA(1, 1, CB);                                                                       \
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");                                       \
    BD_MMA(1, 0, CB);                                                                       \
  } while (0)

  i32x4 bP[2][2][2], bQ[2][2][2];
  stage_a(0, 0);
  stage_a(1, 0);
  load_b(0, bP);
  if (nk > 1) {
    stage_a(0, 1);
    stage_a(1, 1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  BD_BARRIER();
  if (wr == 1) BD_BARRIER();
  // steady state: both steps of a pair issue B(t+1) and A(t+2) unconditionally (straight-line
  // code, so hipcc's own wait for the B registers is a counted vmcnt, not a drain)
  int t = 0;
  for (; t + 3 < nk; t += 2) {
    BD_FAST(t, bP, bQ);
    BD_FAST(t + 1, bQ, bP);
  }
  for (; t + 1 < nk; t += 2) {
    BD_STEP(t, bP, bQ);
    BD_STEP(t + 1, bQ, bP);
  }
  if (t < nk) BD_STEP(t, bP, bQ);
  if (wr == 0) BD_BARRIER();
#undef BD_STEP
#undef BD_FAST
#undef BD_WAIT_B
#undef BD_MMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: bf16 through LDS, two 128-row halves (gemm_big's plain form) ----
  constexpr int LDT = 256 + 4;
  bf16_t* tile = (bf16_t*)smem;
  auto col_of = [&](int j) -> int { return wc * 64 + j * 16; };
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (wr == hh) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = i * 16 + frow, col = col_of(j) + fq * 4;
          *(uint2*)(tile + row * LDT + col) =
              make_uint2(pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3]));
        }
    }
    __syncthreads();
    constexpr int CH = 256 / 8;
    const int cc = tid % CH;
#pragma unroll
    for (int pass = 0; pass < 128 * CH / 512; ++pass) {
      const int row = pass * (512 / CH) + tid / CH;
      const int grow = m0 + hh * 128 + row, gcol = n0 + cc * 8;
      if (grow < M) {
        const uint2 lo = *(const uint2*)(tile + row * LDT + cc * 8);
        const uint2 hi = *(const uint2*)(tile + row * LDT + cc * 8 + 4);
        *(uint4*)(C + (long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    }
    __syncthreads();
  }
}

__global__ void bd_shuffle_kernel(const bf16_t* __restrict__ W, long ldw, bf16_t* __restrict__ img, int N, int K) {
  // one thread per 16-B image chunk: chunk c -> (nb, ks, kk, lane)
  const long nchunk = (long)N * K / 8;
  const int nk = K / 64;
  for (long c = (long)blockIdx.x * blockDim.x + threadIdx.x; c < nchunk; c += (long)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63), kk = (int)((c >> 6) & 1);
    const long blk = c >> 7;
    const int ks = (int)(blk % nk);
    const long nb = blk / nk;
    const long row = nb * 16 + (lane & 15);
    const long k = (long)ks * 64 + kk * 32 + (lane >> 4) * 8;
    *(uint4*)(img + c * 8) = *(const uint4*)(W + row * ldw + k);
  }
}

}  // namespace bd

extern "C" int bd_gemm(const void* A, long lda, const void* Bimg, void* C, long ldc, int M, int N, int K,
                       hipStream_t st) {
  if (N % 256 || K % 64 || K < 128 || (long)N * K * 2 >= (1L << 31)) return -1;
  const int nwg = ((M + 255) / 256) * (N / 256);
  hipLaunchKernelGGL(bd::bd_kernel, dim3(nwg), dim3(512), 0, st, (const rt::bf16_t*)A, lda, (const rt::bf16_t*)Bimg,
                     (rt::bf16_t*)C, ldc, M, N, K);
  return 0;
}

extern "C" int bd_shuffle(const void* W, long ldw, void* img, int N, int K, hipStream_t st) {
  if (N % 16 || K % 64) return -1;
  hipLaunchKernelGGL(bd::bd_shuffle_kernel, dim3(4096), dim3(256), 0, st, (const rt::bf16_t*)W, ldw, (rt::bf16_t*)img, N, K);
  return 0;
}
