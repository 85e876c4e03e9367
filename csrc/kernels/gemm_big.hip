// Token-parallel bf16 GEMM family for gfx950 (M > 64): prefill, reference scoring, and the
// forward / backward GEMMs of LoRA SFT, PPO and full fine-tuning.
//
//   C[M,N] = epi( A·B  +  A2·B2 )          (A2·B2 = LoRA K-extension, optional)
//
// Operand layouts (per operand, template parameters):
//   ROW  : the operand's K index is contiguous — A stored [M][K], B stored [N][K] (nn.Linear
//          weight [out, in]). LDS image [256 rows][128 B], 16-B slot = k-chunk ^ ((row>>1)&7),
//          read with ds_read_b128 (conflict-free over every 16-lane group).
//   KMAJ : the operand's M/N index is contiguous — A stored [K][M], B stored [K][N]. LDS image
//          8 blocks of [64 k][32 mn] (64-B rows), 16-B chunk ^ (((k>>3)&1)<<1), read with
//          ds_read_b64_tr_b16 (hardware transpose; conflict-free over each 32-lane half).
// so NT (forward: X·Wᵀ) = ROW/ROW, NN (dX = dY·W) = ROW/KMAJ, TN (dW = dYᵀ·X) = KMAJ/KMAJ.
// The reference's forward and backward passes (reinforcement_learning_optimization_after_rag.py
// :200-209 policy/value forwards, :229 backward) are these GEMMs.
//
// Block: 256x256 output tile, 8 waves (2 x 4), each wave 128 x 64 = 8 x 4 fragments of
// mfma_f32_16x16x32_bf16, K-step 64, two K-step buffers (128 KiB LDS, 1 block per CU).
// The K-step is computed in four phases of 16 MFMAs per wave (quadrants a0b0, a0b1, a1b1,
// a1b0). LDS-DMA (global_load_lds, 16 B / lane) moves one 16-KiB GRANULE per phase:
//   a0 / a1 = A rows with bit 6 = 0 / 1 (A sub-block 0 / 1 of every wave),
//   b0 / b1 = B rows with bit 5 = 0 / 1 (B sub-block 0 / 1 of every wave).
// Issue schedule (global phase P = 4t + p, p = 1..4):  a0(u) at P = 4u-5, b0(u) 4u-4,
// b1(u) 4u-3, a1(u) 4u-2  — i.e. granules of step u+2 are written into the buffer of step u
// two or more phases after their last ds_read there (WAR), and every granule has ~4 phases
// (≈ 2 µs) to land; counted `s_waitcnt vmcnt(2n)` (never 0 in the loop) retire a granule in
// the phase BEFORE the one that reads it, behind a raw s_barrier (cdna_hip_programming.md §5
// 'Pipelining across barriers', 'Read a staged buffer one phase AFTER the wait').
// Waves 4-7 run one barrier behind waves 0-3, so each SIMD pairs one wave's MFMA cluster with
// its partner's LDS reads / DMA issue (guide §5 T3-T5). All LDS is one __shared__ array.
// Tiles: XCD-aware bijective remap + grouped (GROUP_M) order; split-K over blockIdx.y with fp32
// atomic accumulation (narrow outputs with a deep reduction, e.g. LoRA dA / dB).
// Reduction tails (K % 64 != 0) and the K-extension read a zero page for out-of-range k.
#include "rt_common.h"

#include <algorithm>

namespace rt {

namespace gb {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int GRAN = 16384;         // one granule
constexpr int OPB = 2 * GRAN;       // one operand's K-step image (256 x 64 bf16)
constexpr int BUF = 2 * OPB;        // A + B of one K-step
constexpr int GROUP_M = 4;

enum Layout { ROW = 0, KMAJ = 1 };
enum Out { O_BF16 = 0, O_F32 = 1, O_F32_ATOMIC = 2, O_F32_SLAB = 3 };
// E_DSWIGLU (NN, bf16 out): the SwiGLU backward in the epilogue of the down projection's dX GEMM.
// The accumulator is dF [M, F] (F = N); R = the forward's [gate | up] pre-activation [M, 2F] and C
// = d[gate | up] [M, 2F] (ldr = ldc = 2F rows): dF is rounded to bf16 first, then exactly the
// arithmetic of swiglu_bwd_kernel — bitwise the unfused GEMM + SwiGLU-backward pair, without the
// dF round trip through HBM.
// E_ROPE (NT, bf16 out): rotary embedding of the q / k heads of a fused qkv projection in the
// epilogue — output columns [0, rope_cols) are heads of rope_d columns whose halves (e, e + rope_d/2)
// rotate by the angle table row rope_pos[row] (cos / sin [positions, rope_d / 2] fp32). A head never
// straddles a tile (rope_d divides 128), so both halves are in the LDS-staged tile. Arithmetic of
// rope_qkv_kernel (sign +1) on the bf16-rounded GEMM output: bitwise the GEMM + rope pair.
enum Epi { E_NONE = 0, E_RELU = 1, E_GELU = 2, E_GELU_TANH = 3, E_SILU = 4, E_SWIGLU = 5, E_DSWIGLU = 6, E_ROPE = 7 };

struct Args {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  const bf16_t* A2; long lda2;    // K-extension operands (same layouts), K2 reduction length
  const bf16_t* B2; long ldb2;
  int K2;
  const bf16_t* bias;             // [N] (bf16) or null
  void* C; long ldc;
  bf16_t* C2; long ldc2;          // E_SWIGLU: optional pre-activation [M, 2F] ([gate | up])
  const bf16_t* R; long ldr;      // bf16 out: C = act(acc + bias) + R (residual / beta = 1 input), or null
  int M, N, K;                    // E_SWIGLU: N = 2F rows of the [gate; up] weight
  int act;
  int nsplit;                     // split-K factor (gridDim.y)
  const bf16_t* zpage;            // >= 128 zero bytes
  // F8 (W8A8, config 5): A / B are OCP e4m3fn bytes viewed as bf16 pairs (K and the strides in
  // 2-byte units), one MX-scaled 16x16x128 MFMA per fragment pair and K-step; C = acc * sa[row] *
  // sb[weight row] before bias / activation / SwiGLU
  const float* sa;
  const float* sb;
  int group_m;        // rows of tiles per L2 group (0 = GROUP_M); tuning gemm_group_m
  // E_ROPE: per-row rotary position, angle tables, rotated column count, head width
  const int* rope_pos;
  const float* rope_cos;
  const float* rope_sin;
  int rope_cols, rope_d;
};

__device__ __forceinline__ int row_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int kmaj_swz(int k) { return ((k >> 3) & 1) << 1; }

__device__ __forceinline__ float act_fn(float x, int act) {
  switch (act) {
    case E_RELU: return fmaxf(x, 0.f);
    case E_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case E_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
    }
    case E_SILU: return x / (1.f + __expf(-x));
    default: return x;
  }
}

// counted wait: leave the n newest granules (wave-uniform; n = 4, 2, 1 or 0 at the call sites) in
// flight. BN = 256: every granule is 2 LDS-DMA instructions per lane -> vmcnt(2n). BN = 128: the B
// granules are 1 instruction; at every call site the n newest granules are
//   n = 4: two A + two B granules -> 6;   n = 2: a1 + b1 -> 3;   n = 1: a1 -> 2
template <int BN>
__device__ __forceinline__ void wait_granules(int n) {
  if (BN == 256) {
    if (n >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

#define GB_BARRIER() asm volatile("s_barrier" ::: "memory")

// BN = 256 (default) or 128 output columns per tile. The 128-wide form keeps the A side, the phase
// structure and the issue order; its B granules are 64 rows (one LDS-DMA instruction per wave) and
// each wave owns 2 B fragments instead of 4 (columns 64 (wc >> 1) + 16 (wc & 1) + 32 s): used for
// M = 256 decode GEMMs (twice the workgroups, no split-K on the widest weights) and for the last,
// partial wave of tiles of a large GEMM (rt_gemm_big_planned).
template <int LA, int LB, int OUT, int EPI, int BN, bool F8 = false>
__global__ __launch_bounds__(512, 2) void gemm_big_kernel(Args p) {
  static_assert(BN == 256 || BN == 128, "BN");
  static_assert(!F8 || (LA == ROW && LB == ROW && (OUT == O_BF16 || OUT == O_F32_SLAB)),
                "F8: NT with a bf16 output or split-K slabs only");
  constexpr int NB = BN / 128;  // B fragments per wave and B sub-block; LDS-DMA instructions per B granule
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];  // the only __shared__ object


  const int tiles_m = (p.M + 255) / 256;
  const int tiles_n = EPI == E_SWIGLU ? p.N / BN : (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  // ---- K-steps ----
  const int nk1 = (p.K + 63) / 64;
  const int nk2 = p.A2 ? (p.K2 + 63) / 64 : 0;
  const int nk = nk1 + nk2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar LDS bases
  const int wr = wid >> 2, wc = wid & 3;
  const int frow = lane & 15, fq = lane >> 4;
  const int t_begin = (int)((long)blockIdx.y * nk / p.nsplit);
  const int t_end = (int)((long)(blockIdx.y + 1) * nk / p.nsplit);
  // ---- tile assignment: group_m-row groups (L2 reuse of B panels) over the remapped id ----
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int GM = p.group_m > 0 ? p.group_m : GROUP_M;
  const int group = bid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (bid % gsz);
  const int tn = (bid % (GM * tiles_n)) / gsz;
  const int m0 = tm * 256, n0 = tn * BN;
  const int Fh = p.N / 2;  // E_SWIGLU: gate rows [0, F), up rows [F, 2F)
  constexpr int HALF = BN / 2;  // E_SWIGLU: tile columns [0, HALF) gate, [HALF, BN) up


  // ---- LDS-DMA geometry of instruction j (0, 1) of this wave in granule g (0 a0, 1 a1, 2 b0, 3 b1) ----
  // ROW : 8 rows x 128 B per instruction; lane -> row rb + lane/8, 16-B slot lane%8 holding k-chunk
  //       slot ^ row_swz(row) (source-side swizzle, guide rule 21)
  // KMAJ: 16 k-rows x 64 B of one 32-wide block; lane -> k-row kr0 + lane/4, chunk lane%4 holding
  //       mn-chunk (lane%4) ^ kmaj_swz(kr)
  auto lds_dst = [&](int g, int j) -> int {  // byte offset of the instruction's 1 KiB in the K-step image
    const int op = g >> 1, s = g & 1, o = (op == 0 || NB == 2) ? wid * 2 + j : wid;
    if ((op ? LB : LA) == ROW) {
      const int rb = op == 0 ? (o >> 3) * 128 + s * 64 + (o & 7) * 8 : (o >> 2) * 64 + s * 32 + (o & 3) * 8;
      return op * OPB + rb * 128;
    }
    const int blk = op == 0 ? (o >> 3) * 4 + s * 2 + ((o >> 2) & 1) : (o >> 2) * 2 + s;
    return op * OPB + blk * 4096 + (o & 3) * 16 * 64;
  };
  // per-lane element offset of the source (relative to the operand base + K-step advance) and the
  // lane's reduction index within the K-step (for ragged tails)
  auto src_off = [&](int g, int j, long ld, bool main_w, int& kin) -> uint32_t {
    const int op = g >> 1, s = g & 1, o = (op == 0 || NB == 2) ? wid * 2 + j : wid;
    if ((op ? LB : LA) == ROW) {
      const int rb = op == 0 ? (o >> 3) * 128 + s * 64 + (o & 7) * 8 : (o >> 2) * 64 + s * 32 + (o & 3) * 8;
      const int row = rb + (lane >> 3);
      const int kc = (lane & 7) ^ row_swz(row);
      int grow;
      if (op == 0) grow = min(m0 + row, p.M - 1);
      // SwiGLU: tile rows [0, HALF) are gate rows, [HALF, BN) the matching up rows — for the weight
      // and for its K-extension (LoRA UB rows follow the weight's row order)
      else if (EPI == E_SWIGLU) grow = row < HALF ? tn * HALF + row : Fh + tn * HALF + row - HALF;
      else grow = min(n0 + row, p.N - 1);
      kin = kc * 8;
      return (uint32_t)grow * (uint32_t)ld + (uint32_t)(kc * 8);
    }
    const int blk = op == 0 ? (o >> 3) * 4 + s * 2 + ((o >> 2) & 1) : (o >> 2) * 2 + s;
    const int kr = (o & 3) * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ kmaj_swz(kr);
    const int col = min((op == 0 ? m0 : n0) + blk * 32 + ch * 8, (op == 0 ? p.M : p.N) - 8);
    kin = kr;
    return (uint32_t)kr * (uint32_t)ld + (uint32_t)col;
  };
  uint32_t off[4][2];
  int kin[2][2];  // reduction index of the lane within a K-step: A granules (ROW: k-chunk; KMAJ: k-row)
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int ki = 0;
      off[g][j] = (g < 2 || j < NB) ? src_off(g, j, (g >> 1) ? p.ldb : p.lda, true, ki) : 0u;
      if (g < 2) kin[g][j] = ki;
    }
  auto gdst = [&](int g, int j, int t) -> char* { return smem + (t & 1) * BUF + lds_dst(g, j); };
  // one granule g of K-step t into buffer t & 1 (g is a literal at every call site)
  auto stage = [&](int g, int t) {
    const int op = g >> 1;
    if (t < nk1) {
      const int k0 = t * 64;
      const long adv = ((op ? LB : LA) == ROW) ? (long)k0 : (long)k0 * (op ? p.ldb : p.lda);
      const bf16_t* base = (op ? p.B : p.A) + adv;
      if (k0 + 64 <= p.K) {
#pragma unroll
        for (int j = 0; j < (op ? NB : 2); ++j)
          __builtin_amdgcn_global_load_lds((const void*)(base + off[g][j]), (lds_void*)gdst(g, j, t), 16, 0, 0);
      } else {  // ragged reduction tail: out-of-range k reads the zero page
#pragma unroll
        for (int j = 0; j < (op ? NB : 2); ++j) {
          int ki;
          src_off(g, j, 1, true, ki);
          const bf16_t* src = k0 + ki < p.K ? base + off[g][j] : p.zpage + (lane & 7) * 8;
          __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)gdst(g, j, t), 16, 0, 0);
        }
      }
    } else {  // K-extension (LoRA): a few steps, offsets recomputed with the extension strides
      const int k0 = (t - nk1) * 64;
      const long ld2 = op ? p.ldb2 : p.lda2;
      const long adv = ((op ? LB : LA) == ROW) ? (long)k0 : (long)k0 * ld2;
      const bf16_t* base = (op ? p.B2 : p.A2) + adv;
#pragma unroll
      for (int j = 0; j < (op ? NB : 2); ++j) {
        int ki;
        const uint32_t o2 = src_off(g, j, ld2, false, ki);
        const bf16_t* src = k0 + ki < p.K2 ? base + o2 : p.zpage + (lane & 7) * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)gdst(g, j, t), 16, 0, 0);
      }
    }
  };
  (void)kin;

  // ---- fragment reads ----
  i32x8 fa[4], fb0[2], fb1[2];
  auto rd_row = [&](const char* img, int row) -> i32x8 {
    const i32x4 lo = *(const i32x4*)(img + row * 128 + ((fq ^ row_swz(row)) << 4));
    const i32x4 hi = *(const i32x4*)(img + row * 128 + (((4 + fq) ^ row_swz(row)) << 4));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  // KMAJ fragments by inline-asm transposed reads (the builtin makes hipcc drain every LDS-DMA in
  // flight before each read: rt_common.h). The 4 reads of a fragment are at +0, +256, +2048, +2304
  // bytes from its first (rows kr, kr + 4, kr + 32, kr + 36 share the chunk swizzle).
  auto kmaj_addr = [&](const char* img, int mn) -> uint32_t {
    const int blk = mn >> 5, c0 = mn & 31;
    const int q = frow >> 2, pp = frow & 3;
    const int col = c0 + 4 * pp;
    const int kr = fq * 8 + q;
    const int ch = (col >> 3) ^ kmaj_swz(kr);
    return lds_addr(img + blk * 4096 + kr * 64 + ch * 16 + (col & 7) * 2);
  };
  auto frag_of = [](const rt_s16x4* v) -> i32x8 {
    typedef __attribute__((ext_vector_type(16))) short s16x16;
    const s16x16 w = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3],
                      v[2][0], v[2][1], v[2][2], v[2][3], v[3][0], v[3][1], v[3][2], v[3][3]};
    return __builtin_bit_cast(i32x8, w);
  };
  auto read_a = [&](int buf, int s) {
    const char* img = smem + buf * BUF;
    if constexpr (LA == ROW) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = rd_row(img, wr * 128 + s * 64 + i * 16 + frow);
    } else {
      rt_s16x4 v[16];
      ds_tr16_frag4<256, 2048, 2304>(kmaj_addr(img, wr * 128 + s * 64), kmaj_addr(img, wr * 128 + s * 64 + 16),
                                     kmaj_addr(img, wr * 128 + s * 64 + 32), kmaj_addr(img, wr * 128 + s * 64 + 48), v);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_of(v + 4 * i);
    }
  };
  auto read_b = [&](int buf, int s, i32x8 (&fb)[2]) {
    const char* img = smem + buf * BUF + OPB;
    auto brow = [&](int j) {
      return NB == 2 ? (wc >> 1) * 128 + (wc & 1) * 64 + s * 32 + j * 16 : (wc >> 1) * 64 + s * 32 + (wc & 1) * 16;
    };
    if constexpr (LB == ROW) {
#pragma unroll
      for (int j = 0; j < NB; ++j) fb[j] = rd_row(img, brow(j) + frow);
    } else if constexpr (NB == 2) {
      rt_s16x4 v[8];
      ds_tr16_frag2<256, 2048, 2304>(kmaj_addr(img, brow(0)), kmaj_addr(img, brow(1)), v);
      fb[0] = frag_of(v);
      fb[1] = frag_of(v + 4);
    } else {
      rt_s16x4 v[4];
      ds_tr16_x4<256, 2048, 2304>(kmaj_addr(img, brow(0)), v[0], v[1], v[2], v[3]);
      fb[0] = frag_of(v);
    }
  };
  auto half = [](const i32x8& v, int h) -> bf16x8 {
    return h == 0 ? __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3))
                  : __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
  };

  f32x4 acc[8][2 * NB];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // tile column of accumulator column-fragment j (0 .. 2 NB - 1; j / NB = B sub-block)
  auto col_of = [&](int j) -> int { return NB == 2 ? wc * 64 + j * 16 : (wc >> 1) * 64 + (wc & 1) * 16 + j * 32; };

  // SWAP: B fragment as the MFMA's A operand -> the accumulator holds C^T, i.e. every lane owns
  // 4 CONSECUTIVE output columns of one row (16-B fp32 / 8-B bf16 epilogue stores instead of
  // 2-4-B scattered ones). The atomic form keeps C (16 consecutive columns per 16 lanes per row).
  constexpr bool SWAP = OUT != O_F32_ATOMIC;
#define GB_MMA(SA, SB, FB) GB_MMA_X(SA, SB, FB, false)
  // EXT (F8 only): a K-extension step (LoRA, bf16 operands) inside an fp8 GEMM -> bf16 MFMAs
#define GB_MMA_X(SA, SB, FB, EXT)                                                            \
  do {                                                                                      \
    GB_BARRIER();                                                                           \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    __builtin_amdgcn_s_setprio(1);                                                          \
    if (F8 && !(EXT)) {                                                                     \
      /* the 32 bytes of a lane are the same two 16-B chunks of A and B rows: one k pairing */ \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                         \
        _Pragma("unroll") for (int j = 0; j < NB; ++j)                                      \
          acc[(SA) * 4 + i][(SB) * NB + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4( \
              FB[j], fa[i], acc[(SA) * 4 + i][(SB) * NB + j], 0, 0, 0, 127, 0, 127);        \
    } else {                                                                                \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                           \
      _Pragma("unroll") for (int j = 0; j < NB; ++j)                                        \
        _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                    \
          acc[(SA) * 4 + i][(SB) * NB + j] = SWAP                                           \
              ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(FB[j], kk), half(fa[i], kk),   \
                                                        acc[(SA) * 4 + i][(SB) * NB + j], 0, 0, 0) \
              : __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(fa[i], kk), half(FB[j], kk),   \
                                                        acc[(SA) * 4 + i][(SB) * NB + j], 0, 0, 0); \
    }                                                                                       \
    __builtin_amdgcn_s_setprio(0);                                                          \
    GB_BARRIER();                                                                           \
  } while (0)

  if (t_begin < t_end) {
    // prologue: step t_begin complete (a0, b0, b1, a1) + a0, b0 of step t_begin + 1; granules are
    // always issued in key order a0(u) b0(u) b1(u) a1(u) a0(u+1) b0(u+1) ... (see header)
    const bool two = t_begin + 1 < t_end;
    stage(0, t_begin); stage(2, t_begin); stage(3, t_begin); stage(1, t_begin);
    if (two) { stage(0, t_begin + 1); stage(2, t_begin + 1); }
    wait_granules<BN>(two ? 4 : 2);  // retire a0, b0 of t_begin
    GB_BARRIER();  // raw: a __syncthreads() would drain the granules still in flight
    if (wr == 1) GB_BARRIER();

    // steady state: every granule staged by steps t < t_fast is a full main-K step (no tail, no
    // extension, no end-of-range checks): straight-line phases with fixed counted waits
    const int nk1f = p.K / 64;
    const int t_fast = min(t_end, nk1f) - 2;
    auto stage_fast = [&](int g, int u) {
      const int op = g >> 1;
      const long adv = ((op ? LB : LA) == ROW) ? (long)u * 64 : (long)u * 64 * (op ? p.ldb : p.lda);
      const bf16_t* base = (op ? p.B : p.A) + adv;
      char* img = smem + (u & 1) * BUF;
#pragma unroll
      for (int j = 0; j < (op ? NB : 2); ++j)
        __builtin_amdgcn_global_load_lds((const void*)(base + off[g][j]), (lds_void*)(img + lds_dst(g, j)), 16, 0, 0);
    };
    int t = t_begin;
    for (; t < t_fast; ++t) {
      const int buf = t & 1;
      read_a(buf, 0);
      read_b(buf, 0, fb0);
      stage_fast(3, t + 1);
      wait_granules<BN>(4);
      GB_MMA(0, 0, fb0);
      read_b(buf, 1, fb1);
      stage_fast(1, t + 1);
      wait_granules<BN>(4);
      GB_MMA(0, 1, fb1);
      read_a(buf, 1);
      stage_fast(0, t + 2);
      GB_MMA(1, 1, fb1);
      stage_fast(2, t + 2);
      wait_granules<BN>(4);
      GB_MMA(1, 0, fb0);
    }
    for (; t < t_end; ++t) {
      const int buf = t & 1;
      const bool n1 = t + 1 < t_end, n2 = t + 2 < t_end;
      const bool ext = F8 && t >= nk1;  // fp8 GEMM: the LoRA K-extension steps are bf16
      // p1: quadrant a0 x b0; stage b1(t+1); retire b1(t) (issued after it: a1(t), a0 / b0 / b1 (t+1))
      read_a(buf, 0);
      read_b(buf, 0, fb0);
      if (n1) stage(3, t + 1);
      wait_granules<BN>(n1 ? 4 : 1);
      GB_MMA_X(0, 0, fb0, ext);
      // p2: a0 x b1; stage a1(t+1); retire a1(t)
      read_b(buf, 1, fb1);
      if (n1) stage(1, t + 1);
      wait_granules<BN>(n1 ? 4 : 0);
      GB_MMA_X(0, 1, fb1, ext);
      // p3: a1 x b1; stage a0(t+2)
      read_a(buf, 1);
      if (n2) stage(0, t + 2);
      GB_MMA_X(1, 1, fb1, ext);
      // p4: a1 x b0; stage b0(t+2); retire a0 / b0 of t+1 (after them: b1 / a1 (t+1), a0 / b0 (t+2))
      if (n2) stage(2, t + 2);
      if (n1) wait_granules<BN>(n2 ? 4 : 2);
      GB_MMA_X(1, 0, fb0, ext);
    }
    if (wr == 0) GB_BARRIER();
  }
#undef GB_MMA
#undef GB_MMA_X
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue ----
  // SWAP: acc[i][j][r] = C[m0 + 128 wr + 16 i + frow][n0 + 64 wc + 16 j + 4 fq + r]
  // else: acc[i][j][r] = C[m0 + 128 wr + 16 i + 4 fq + r][n0 + 64 wc + 16 j + frow]
  if constexpr (OUT == O_F32_ATOMIC) {
    float* C = (float*)p.C;
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int col = n0 + col_of(j) + frow;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * 128 + i * 16 + fq * 4 + r;
          if (row < p.M && col < p.N)
            __hip_atomic_fetch_add(C + (long)row * p.ldc + col, acc[i][j][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
  } else if constexpr (OUT == O_F32 || OUT == O_F32_SLAB) {
    // O_F32_SLAB: split ks writes its partial tile to slab ks ([nsplit][M][ldc], plain stores);
    // splitk_reduce_kernel sums the slabs and runs the epilogue. N % 4 == 0 (launcher).
    // F8 (slabs): each split's partial carries the per-token x per-channel scales (the reduce is a
    // plain sum)
    float* C = (float*)p.C + (OUT == O_F32_SLAB ? (long)blockIdx.y * p.M * p.ldc : 0L);
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int col = n0 + col_of(j) + fq * 4;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      float sc[4] = {1.f, 1.f, 1.f, 1.f};
      if (OUT == O_F32 && p.bias && col < p.N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bf2f(p.bias[col + r]);
      }
      if (F8) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[r] = p.sb[min(col + r, p.N - 1)];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wr * 128 + i * 16 + frow;
        if (row < p.M && col < p.N) {
          const float sr = F8 ? p.sa[row] : 1.f;
          float4 v;
          v.x = act_fn((F8 ? acc[i][j][0] * (sr * sc[0]) : acc[i][j][0]) + bv[0], EPI);
          v.y = act_fn((F8 ? acc[i][j][1] * (sr * sc[1]) : acc[i][j][1]) + bv[1], EPI);
          v.z = act_fn((F8 ? acc[i][j][2] * (sr * sc[2]) : acc[i][j][2]) + bv[2], EPI);
          v.w = act_fn((F8 ? acc[i][j][3] * (sr * sc[3]) : acc[i][j][3]) + bv[3], EPI);
          *(float4*)(C + (long)row * p.ldc + col) = v;
        }
      }
    }
  } else {
    // bf16 through LDS (two 128-row halves; row stride 260 elements = 520 B: the 8-B ds_write of
    // 16 lanes in 16 rows hit 16 distinct bank pairs) for 16-B coalesced global stores
    constexpr int LDT = BN + 4;
    bf16_t* tile = (bf16_t*)smem;
    float bcol[2 * NB][4];
    float scol[2 * NB][4];  // F8: per-output-channel weight scale of the lane's columns
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int col = n0 + col_of(j) + fq * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bcol[j][r] = (EPI != E_SWIGLU && p.bias && col < p.N) ? bf2f(p.bias[col + r]) : 0.f;
        if constexpr (F8) {
          const int c = col_of(j) + fq * 4 + r;  // tile column -> weight row
          const int wrow = EPI == E_SWIGLU ? (c < HALF ? tn * HALF + c : Fh + tn * HALF + c - HALF) : min(n0 + c, p.N - 1);
          scol[j][r] = p.sb[wrow];
        }
      }
    }
    auto ld16 = [&](int row, int c8) -> uint4 {  // 8 bf16 at tile[row][8 c8], 8-B aligned
      const uint2 lo = *(const uint2*)(tile + row * LDT + c8 * 8);
      const uint2 hi = *(const uint2*)(tile + row * LDT + c8 * 8 + 4);
      return make_uint4(lo.x, lo.y, hi.x, hi.y);
    };
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (wr == hh) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          // F8: per-token activation scale of this fragment row (x the column's weight scale)
          const float srow = F8 ? p.sa[min(m0 + hh * 128 + i * 16 + frow, p.M - 1)] : 1.f;
#pragma unroll
          for (int j = 0; j < 2 * NB; ++j) {
            const int row = i * 16 + frow, col = col_of(j) + fq * 4;
            float y[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = F8 ? acc[i][j][r] * (srow * scol[j][r]) : acc[i][j][r];
              y[r] = EPI == E_SWIGLU ? v : act_fn(v + bcol[j][r], EPI);
            }
            *(uint2*)(tile + row * LDT + col) = make_uint2(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]));
          }
        }
      }
      __syncthreads();
      if constexpr (EPI == E_SWIGLU) {
        // tile columns [0,128) = gate F-cols tn*128.., [128,256) = up; f = silu(g) * u from the
        // bf16-rounded pre-activations (bitwise what a separate SwiGLU kernel would read)
        bf16_t* Cf = (bf16_t*)p.C;
        constexpr int CH = HALF / 8;  // 16-B chunks per row of the gate half
        const int cc = tid % CH;
#pragma unroll
        for (int pass = 0; pass < 128 * CH / 512; ++pass) {
          const int row = pass * (512 / CH) + tid / CH;
          const int grow = m0 + hh * 128 + row;
          if (grow < p.M) {
            const uint4 g4 = ld16(row, cc), u4 = ld16(row, CH + cc);
            float g[8], u[8], f[8];
            unpack8(g4, g);
            unpack8(u4, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = g[e] / (1.f + __expf(-g[e])) * u[e];
            const int fcol = tn * HALF + cc * 8;
            *(uint4*)(Cf + (long)grow * p.ldc + fcol) = pack8(f);
            if (p.C2) {
              *(uint4*)(p.C2 + (long)grow * p.ldc2 + fcol) = g4;
              *(uint4*)(p.C2 + (long)grow * p.ldc2 + Fh + fcol) = u4;
            }
          }
        }
      } else if constexpr (EPI == E_DSWIGLU) {
        bf16_t* C = (bf16_t*)p.C;
        const int F = p.N;
        constexpr int CH = BN / 8;
        const int cc = tid % CH;
#pragma unroll
        for (int pass = 0; pass < 128 * CH / 512; ++pass) {
          const int row = pass * (512 / CH) + tid / CH;
          const int grow = m0 + hh * 128 + row, gcol = n0 + cc * 8;
          if (grow < p.M && gcol < F) {
            float d[8], g[8], u[8], dg[8], du[8];
            unpack8(ld16(row, cc), d);
            unpack8(*(const uint4*)(p.R + (long)grow * p.ldr + gcol), g);
            unpack8(*(const uint4*)(p.R + (long)grow * p.ldr + F + gcol), u);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float sg = 1.f / (1.f + __expf(-g[e]));
              const float si = g[e] * sg;
              du[e] = d[e] * si;
              dg[e] = d[e] * u[e] * sg * (1.f + g[e] * (1.f - sg));
            }
            *(uint4*)(C + (long)grow * p.ldc + gcol) = pack8(dg);
            *(uint4*)(C + (long)grow * p.ldc + F + gcol) = pack8(du);
          }
        }
      } else {
        bf16_t* C = (bf16_t*)p.C;
        constexpr int CH = BN / 8;  // 16-B chunks per tile row
        const int cc = tid % CH;
#pragma unroll
        for (int pass = 0; pass < 128 * CH / 512; ++pass) {
          const int row = pass * (512 / CH) + tid / CH;
          const int grow = m0 + hh * 128 + row, gcol = n0 + cc * 8;
          if (grow < p.M && gcol < p.N) {
            uint4 v = ld16(row, cc);
            if constexpr (EPI == E_ROPE) {
              if (gcol < p.rope_cols) {
                const int hd2 = p.rope_d >> 1, e = gcol % p.rope_d;
                const bool lo = e < hd2;
                const uint4 pv = ld16(row, lo ? cc + (hd2 >> 3) : cc - (hd2 >> 3));  // the rotation partner
                float x[8], y[8], o8[8];
                unpack8(v, x);
                unpack8(pv, y);
                const long tb = (long)p.rope_pos[grow] * hd2 + (lo ? e : e - hd2);
                const float4 c0 = *(const float4*)(p.rope_cos + tb), c1 = *(const float4*)(p.rope_cos + tb + 4);
                const float4 s0 = *(const float4*)(p.rope_sin + tb), s1 = *(const float4*)(p.rope_sin + tb + 4);
                const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
                for (int k = 0; k < 8; ++k)  // lo: x1 c - x2 s ; hi: x2 c + x1 s (rope_qkv_kernel's fma order)
                  o8[k] = lo ? fmaf(x[k], cs[k], -(y[k] * sn[k])) : fmaf(x[k], cs[k], y[k] * sn[k]);
                v = pack8(o8);
              }
            }
            if (p.R) {  // residual in fp32 on the bf16-rounded GEMM result (= a separate add kernel)
              float y[8], r[8];
              unpack8(v, y);
              unpack8(*(const uint4*)(p.R + (long)grow * p.ldr + gcol), r);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[e] += r[e];
              v = pack8(y);
            }
            *(uint4*)(C + (long)grow * p.ldc + gcol) = v;
          }
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Small-tile GEMM for the narrow LoRA products (SURVEY K1 dA / dB / LoRA down-projection):
//   U  = X A_pad^T   [M, Rp]   (ROW / ROW)        dU = dY UB   [M, Rp]  (ROW / KMAJ)
//   dA = dU^T X      [Rp, K]   (KMAJ / KMAJ)      dB = dY^T U  [N, Rp]  (KMAJ / KMAJ)
// A 256x256 tile wastes 3/4 of its MFMAs and loads on a 64-wide side, so these run on 64x64 tiles:
// 4 waves (2 x 2, 32 x 32 each = 2 x 2 fragments), K-step 64 through a 3-slot LDS-DMA ring
// (one slot issued, one landing, one read; counted vmcnt + raw s_barrier), several workgroups per
// CU for latency hiding. Split-K over blockIdx.y with fp32 atomics for the token reductions.
// BM = 128: 128 x 64 tiles (4 waves stacked along M, 32 x 64 each = 2 x 4 fragments) for the
// products whose WIDE operand is A (dB = dY^T U, dU = dY UB, U = X A_pad^T): the narrow B image is
// then staged once per 128 rows of A instead of once per 64 (1.5x instead of 2x the A bytes
// through L2 -> LDS).
constexpr int SM_SLOTS = 3;

template <int LA, int LB, int OUT, int BM = 64>
__global__ __launch_bounds__(256, 2) void gemm_small_kernel(Args p) {
  static_assert(BM == 64 || BM == 128, "gemm_small: BM");
  constexpr int SM_A = BM * 128, SM_SLOT = SM_A + 64 * 128;  // A + B images of one K-step
  constexpr int WN = BM == 64 ? 2 : 1;                       // waves along N
  constexpr int NJ = 4 / WN;                                 // B fragments per wave (wave = 32 x 16 NJ)
  constexpr int NIA = BM / 32;                               // LDS-DMA instructions per wave for A
  __shared__ __attribute__((aligned(16))) char smem[SM_SLOTS * SM_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int tiles_n = (p.N + 63) / 64;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * 64;
  const int nk = (p.K + 63) / 64;
  const int t_begin = (int)((long)blockIdx.y * nk / p.nsplit), t_end = (int)((long)(blockIdx.y + 1) * nk / p.nsplit);

  // instruction j of this wave for operand op (NIA for A, 2 for B): ROW 8 rows x 128 B; KMAJ 16
  // k-rows x 64 B (blocks of 32 m / n columns)
  auto stage = [&](int t) {
    char* slot = smem + ((t - t_begin) % SM_SLOTS) * SM_SLOT;
    const int k0 = t * 64;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const bf16_t* base = op ? p.B : p.A;
      const long ld = op ? p.ldb : p.lda;
      const int lim = op ? p.N : p.M;
      const int mn0 = op ? n0 : m0;
      const int ni = op ? 2 : NIA;
      char* img = slot + (op ? SM_A : 0);
#pragma unroll
      for (int j = 0; j < (op ? 2 : NIA); ++j) {
        const int o = wid * ni + j;
        if ((op ? LB : LA) == ROW) {
          const int row = o * 8 + (lane >> 3);
          const int kc = (lane & 7) ^ row_swz(row);
          const int gr = min(mn0 + row, lim - 1);
          const int kk = k0 + kc * 8;
          const bf16_t* src = kk < p.K ? base + (long)gr * ld + kk : p.zpage + (lane & 7) * 8;
          __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(img + o * 1024), 16, 0, 0);
        } else {
          const int blk = o >> 2, kr0 = (o & 3) * 16;
          const int kr = kr0 + (lane >> 2);
          const int ch = (lane & 3) ^ kmaj_swz(kr);
          const int col = min(mn0 + blk * 32 + ch * 8, lim - 8);
          const bf16_t* src = (k0 + kr) < p.K ? base + (long)(k0 + kr) * ld + col : p.zpage + (lane & 3) * 8;
          __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(img + blk * 4096 + kr0 * 64), 16, 0, 0);
        }
      }
    }
  };
  auto rd_row = [&](const char* img, int row) -> i32x8 {
    const i32x4 lo = *(const i32x4*)(img + row * 128 + ((fq ^ row_swz(row)) << 4));
    const i32x4 hi = *(const i32x4*)(img + row * 128 + (((4 + fq) ^ row_swz(row)) << 4));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto kmaj_addr = [&](const char* img, int mn) -> uint32_t {  // first of a fragment's 4 reads
    const int blk = mn >> 5, c0 = mn & 31;
    const int q = frow >> 2, pp = frow & 3;
    const int col = c0 + 4 * pp;
    const int kr = fq * 8 + q;
    const int ch = (col >> 3) ^ kmaj_swz(kr);
    return lds_addr(img + blk * 4096 + kr * 64 + ch * 16 + (col & 7) * 2);
  };
  auto frag_of = [](const rt_s16x4* v) -> i32x8 {
    typedef __attribute__((ext_vector_type(16))) short s16x16;
    const s16x16 w = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3],
                      v[2][0], v[2][1], v[2][2], v[2][3], v[3][0], v[3][1], v[3][2], v[3][3]};
    return __builtin_bit_cast(i32x8, w);
  };
  auto half = [](const i32x8& v, int h) -> bf16x8 {
    return h == 0 ? __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3))
                  : __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
  };

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t_begin < t_end) {
    stage(t_begin);
    if (t_begin + 1 < t_end) stage(t_begin + 1);
    for (int t = t_begin; t < t_end; ++t) {
      // retire step t (NIA + 2 DMA instructions per lane per step); step t+1 may stay in flight
      if (t + 1 < t_end) {
        if constexpr (BM == 64) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_barrier" ::: "memory");
      // refill the slot read in iteration t-1 (every wave passed the barrier above after reading it)
      if (t + 2 < t_end) stage(t + 2);
      const char* slot = smem + ((t - t_begin) % SM_SLOTS) * SM_SLOT;
      i32x8 fa[2], fb[NJ];
      // KMAJ fragments by inline-asm transposed reads (the builtin drains the LDS-DMA ring)
      if constexpr (LA == ROW) {
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = rd_row(slot, wr * 32 + i * 16 + frow);
      } else {
        rt_s16x4 v[8];
        ds_tr16_frag2<256, 2048, 2304>(kmaj_addr(slot, wr * 32), kmaj_addr(slot, wr * 32 + 16), v);
        fa[0] = frag_of(v);
        fa[1] = frag_of(v + 4);
      }
      if constexpr (LB == ROW) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = rd_row(slot + SM_A, wc * 32 + j * 16 + frow);
      } else {
#pragma unroll
        for (int jj = 0; jj < NJ; jj += 2) {
          rt_s16x4 v[8];
          ds_tr16_frag2<256, 2048, 2304>(kmaj_addr(slot + SM_A, wc * 32 + jj * 16),
                                         kmaj_addr(slot + SM_A, wc * 32 + jj * 16 + 16), v);
          fb[jj] = frag_of(v);
          fb[jj + 1] = frag_of(v + 4);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(fa[i], kk), half(fb[j], kk), acc[i][j], 0, 0, 0);
    }
  }
  // lane holds C[m0 + 32 wr + 16 i + 4 fq + r][n0 + 32 wc + 16 j + frow]
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + wc * 32 + j * 16 + frow;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 32 + i * 16 + fq * 4 + r;
        if (row < p.M && col < p.N) {
          if constexpr (OUT == O_F32_ATOMIC)
            __hip_atomic_fetch_add((float*)p.C + (long)row * p.ldc + col, acc[i][j][r], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          else if constexpr (OUT == O_F32)
            ((float*)p.C)[(long)row * p.ldc + col] = acc[i][j][r];
          else if constexpr (OUT == O_F32_SLAB)  // split ks -> slab ks ([nsplit][M][ldc]); summed in a fixed order
            ((float*)p.C)[((long)blockIdx.y * p.M + row) * p.ldc + col] = acc[i][j][r];
          else
            ((bf16_t*)p.C)[(long)row * p.ldc + col] = f2bf(acc[i][j][r]);
        }
      }
  }
}

// Split-K reduction + epilogue of the O_F32_SLAB form (decode / small-M GEMMs, M <= 256):
//   C[m, c] = act( sum_s slab[s][m][c] + bias[c] ) + R[m, c]            (Nout = N)
//   C[m, c] = silu(bf16(g)) * bf16(u),  g / u = sum_s slab[s][m][c] / [F + c]   (SwiGLU, Nout = F)
// 8 output columns per thread, 16-B slab loads, all nsplit partial loads of a thread in flight.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs, int nsplit, int M, int N,
                                                            const bf16_t* __restrict__ bias, int act,
                                                            const bf16_t* __restrict__ R, long ldr,
                                                            bf16_t* __restrict__ C, long ldc) {
  const bool swiglu = act == E_SWIGLU;
  const int Nout = swiglu ? N / 2 : N;
  const int cpr = Nout / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)M * cpr) return;
  const int m = (int)(e / cpr), c0 = (int)(e % cpr) * 8;
  const long sstride = (long)M * N;
  float a[8], b[8];
  const float* base = slabs + (long)m * N + c0;
  sum_slabs8(base, sstride, nsplit, a);
  if (swiglu) sum_slabs8(base + Nout, sstride, nsplit, b);
  float y[8];
  if (swiglu) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float g = bf2f(f2bf(a[q])), u = bf2f(f2bf(b[q]));
      y[q] = g / (1.f + __expf(-g)) * u;
    }
  } else {
    float bb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, rr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (bias) unpack8(*(const uint4*)(bias + c0), bb);
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = act_fn(a[q] + bb[q], act);
    if (R) {
      // the residual adds to the bf16-rounded GEMM result (= a separate add kernel)
      unpack8(*(const uint4*)(R + (long)m * ldr + c0), rr);
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = bf2f(f2bf(y[q])) + rr[q];
    }
  }
  *(uint4*)(C + (long)m * ldc + c0) = pack8(y);
}

}  // namespace gb
}  // namespace rt

using namespace rt;
using namespace rt::gb;

// layout_a / layout_b: 0 = ROW (K contiguous), 1 = KMAJ (M / N contiguous).
// out: 0 bf16 (epilogue bias + act, or SwiGLU), 1 fp32 store (bias + act), 2 fp32 atomic add
// (split-K; C must be initialised by the caller). Requirements (checked): KMAJ operands have
// M / N % 8 == 0 and 16-B aligned rows; ROW operands 16-B aligned rows; K, K2 % 8 == 0;
// E_SWIGLU: ROW/ROW, bf16 out, N % 256 == 0, no K-extension of B beyond the weight rows.
static int launch_gemm_big(const Args& p, int layout_a, int layout_b, int act, int out, int bn, hipStream_t stream) {
  const int tiles_n = act == E_SWIGLU ? p.N / bn : (p.N + bn - 1) / bn;
  dim3 grid(((p.M + 255) / 256) * tiles_n, p.nsplit), block(512);
  const int key = layout_a * 100 + layout_b * 10 + out;
#define GB_LAUNCH(LA, LB, O, E, BN) hipLaunchKernelGGL((gemm_big_kernel<LA, LB, O, E, BN>), grid, block, 0, stream, p)
  if (bn == 128) {  // the 128-column tile: NT (bf16 / SwiGLU / fp32 / slab) and NN bf16
    switch (key * 10 + act) {
      case 0: GB_LAUNCH(ROW, ROW, O_BF16, E_NONE, 128); break;
      case E_SWIGLU: GB_LAUNCH(ROW, ROW, O_BF16, E_SWIGLU, 128); break;
      case E_ROPE: GB_LAUNCH(ROW, ROW, O_BF16, E_ROPE, 128); break;
      case 10: GB_LAUNCH(ROW, ROW, O_F32, E_NONE, 128); break;
      case 30: GB_LAUNCH(ROW, ROW, O_F32_SLAB, E_NONE, 128); break;
      case 100: GB_LAUNCH(ROW, KMAJ, O_BF16, E_NONE, 128); break;
      case 100 + E_DSWIGLU: GB_LAUNCH(ROW, KMAJ, O_BF16, E_DSWIGLU, 128); break;
      default: return -4;
    }
    } else if (key == 0) {  // NT, bf16 out: the activation is a template parameter (no runtime switch in the epilogue)
    switch (act) {
      case E_NONE: GB_LAUNCH(ROW, ROW, O_BF16, E_NONE, 256); break;
      case E_RELU: GB_LAUNCH(ROW, ROW, O_BF16, E_RELU, 256); break;
      case E_GELU: GB_LAUNCH(ROW, ROW, O_BF16, E_GELU, 256); break;
      case E_GELU_TANH: GB_LAUNCH(ROW, ROW, O_BF16, E_GELU_TANH, 256); break;
      case E_SILU: GB_LAUNCH(ROW, ROW, O_BF16, E_SILU, 256); break;
      case E_SWIGLU: GB_LAUNCH(ROW, ROW, O_BF16, E_SWIGLU, 256); break;
      case E_ROPE: GB_LAUNCH(ROW, ROW, O_BF16, E_ROPE, 256); break;
      default: return -4;
    }
  } else if (key == 10 && act == E_DSWIGLU) {
    GB_LAUNCH(ROW, KMAJ, O_BF16, E_DSWIGLU, 256);
  } else {
    if (act != E_NONE) return -5;  // fp32 outputs and the NN / TN forms carry no activation
    switch (key) {
      case 1: GB_LAUNCH(ROW, ROW, O_F32, E_NONE, 256); break;
      case 2: GB_LAUNCH(ROW, ROW, O_F32_ATOMIC, E_NONE, 256); break;
      case 3: GB_LAUNCH(ROW, ROW, O_F32_SLAB, E_NONE, 256); break;
      case 10: GB_LAUNCH(ROW, KMAJ, O_BF16, E_NONE, 256); break;
      case 11: GB_LAUNCH(ROW, KMAJ, O_F32, E_NONE, 256); break;
      case 12: GB_LAUNCH(ROW, KMAJ, O_F32_ATOMIC, E_NONE, 256); break;
      case 110: GB_LAUNCH(KMAJ, KMAJ, O_BF16, E_NONE, 256); break;
      case 111: GB_LAUNCH(KMAJ, KMAJ, O_F32, E_NONE, 256); break;
      case 112: GB_LAUNCH(KMAJ, KMAJ, O_F32_ATOMIC, E_NONE, 256); break;
      default: return -4;
    }
  }
#undef GB_LAUNCH
  RT_LAUNCH_CHECK();
  return 0;
}

static bool bn128_supported(int layout_a, int layout_b, int act, int out) {
  const int key = layout_a * 100 + layout_b * 10 + out;
  return (key == 0 && (act == E_NONE || act == E_SWIGLU || act == E_ROPE)) ||
         (act == E_NONE && (key == 1 || key == 3 || key == 10)) || (key == 10 && act == E_DSWIGLU);
}

static int query_num_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  return n;
}
// a device property, computed once (thread-safe static initialisation)
static int num_cus() {
  static const int n = query_num_cus();
  return n;
}

// Ratio of a 256x128 tile's time to a 256x256 tile's (same K), for the wave planner below.
static float bn128_cost() { return tuning().gemm_bn128_cost; }

static int gemm_big_planned(const Args& p, int layout_a, int layout_b, int act, int out, int bn, hipStream_t stream);

// layout_a / layout_b: 0 = ROW (K contiguous), 1 = KMAJ (M / N contiguous).
// out: 0 bf16 (epilogue bias + act, or SwiGLU), 1 fp32 store (bias + act), 2 fp32 atomic add
// (split-K; C must be initialised by the caller), 3 fp32 split-K slabs. bn: 256, 128, or 0 = plan:
// the tile rows are cut in two launches — rows [0, 256 m1) on 256x256 tiles, the rest on 256x128
// tiles — with m1 chosen so that the last, partial wave of workgroups is as short as possible
// (e.g. M = 9632 tokens x N = 4096: 608 tiles = 2.4 waves of 256 CUs -> 512 tiles + 192 half tiles).
// Requirements (checked): KMAJ operands have M / N % 8 == 0 and 16-B aligned rows; ROW operands
// 16-B aligned rows; K, K2 % 8 == 0; E_SWIGLU: ROW/ROW, bf16 out, N % 256 == 0.
extern "C" int rt_gemm_big(int layout_a, int layout_b, const void* A, long lda, const void* B, long ldb,
                           const void* A2, long lda2, const void* B2, long ldb2, int K2, const void* bias,
                           void* C, long ldc, void* C2, long ldc2, const void* R, long ldr, int M, int N, int K,
                           int act, int out, int nsplit, const void* zpage, int bn, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (act == E_ROPE) return -5;  // rt_gemm_big_rope (the rotary tables are its arguments)
  // a ROW operand reads 8-element k-chunks: its reduction length must be a multiple of 8
  const bool any_row = layout_a == ROW || layout_b == ROW;
  if ((any_row && (K % 8 || (A2 && K2 % 8))) || !zpage) return -1;
  if (R && (out != O_BF16 || act == E_SWIGLU)) return -6;
  // whole-chunk epilogue stores (8 bf16 / 4 fp32 from every valid column start): the row stride
  // must cover the padded width
  const int Nout = act == E_SWIGLU ? N / 2 : N;
  if (out != O_F32_ATOMIC && (ldc % 8 || (M > 1 && ldc < (long)((Nout + 7) / 8 * 8)))) return -7;
  if ((layout_a == KMAJ && M % 8) || (layout_b == KMAJ && N % 8)) return -1;
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 1 && out != O_F32_ATOMIC && out != O_F32_SLAB) return -2;
  if (act == E_SWIGLU && (layout_a != ROW || layout_b != ROW || out != O_BF16 || N % 256)) return -3;
  if (act == E_DSWIGLU) {
    // the SwiGLU backward epilogue: NN, bf16 d[gate | up] [M, 2N] from the pre-activation R [M, 2N]
    if (layout_a != ROW || layout_b != KMAJ || out != O_BF16 || !R || N % 8 || ldc < 2L * N || ldr < 2L * N ||
        nsplit != 1)
      return -5;
  } else if (act != E_NONE && (layout_a != ROW || layout_b != ROW || out != O_BF16)) {
    return -5;
  }
  if (bn != 0 && bn != 128 && bn != 256) return -8;
  if (bn == 128 && !bn128_supported(layout_a, layout_b, act, out)) return -8;
  Args p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.A2 = (A2 && B2) ? (const bf16_t*)A2 : nullptr; p.lda2 = lda2;
  p.B2 = (const bf16_t*)B2; p.ldb2 = ldb2; p.K2 = K2;
  p.bias = (const bf16_t*)bias; p.C = C; p.ldc = ldc; p.C2 = (bf16_t*)C2; p.ldc2 = ldc2;
  p.R = (const bf16_t*)R; p.ldr = ldr;
  p.M = M; p.N = N; p.K = K; p.act = act; p.nsplit = nsplit; p.zpage = (const bf16_t*)zpage;
  p.group_m = tuning().gemm_group_m;
  return gemm_big_planned(p, layout_a, layout_b, act, out, bn, stream);
}

// bn = 0: the wave planner over validated arguments p
static int gemm_big_planned(const Args& p, int layout_a, int layout_b, int act, int out, int bn, hipStream_t stream) {
  if (bn != 0) return launch_gemm_big(p, layout_a, layout_b, act, out, bn, stream);
  const int M = p.M, N = p.N, nsplit = p.nsplit;
  const long lda = p.lda, lda2 = p.lda2, ldc = p.ldc, ldc2 = p.ldc2, ldr = p.ldr;
  void* C = p.C;
  const bool can128 = bn128_supported(layout_a, layout_b, act, out);
  // ---- plan: m1 row tiles at BN = 256, the rest at BN = 128 ----
  const int tiles_m = (M + 255) / 256;
  const int tn256 = act == E_SWIGLU ? N / 256 : (N + 255) / 256;
  const int tn128 = act == E_SWIGLU ? N / 128 : (N + 127) / 128;
  const long cus = (long)num_cus() * 1;  // one 512-thread, 128-KiB-LDS workgroup per CU
  int m1 = tiles_m;
  float best = (float)((long)tiles_m * tn256 + cus - 1) / (float)cus;
  if (can128 && nsplit == 1 && (out == O_BF16 || out == O_F32)) {
    const float r = bn128_cost();
    best = 1e30f;
    for (int m = tiles_m; m >= 0; --m) {
      const long w256 = ((long)m * tn256 + cus - 1) / cus, w128 = ((long)(tiles_m - m) * tn128 + cus - 1) / cus;
      const float cost = (float)w256 + r * (float)w128;
      if (cost < best - 1e-3f) { best = cost; m1 = m; }
    }
  }
  if (m1 == tiles_m) return launch_gemm_big(p, layout_a, layout_b, act, out, 256, stream);
  const long r0 = (long)m1 * 256;
  if (m1 > 0) {
    Args q = p;
    q.M = (int)r0;
    const int rc = launch_gemm_big(q, layout_a, layout_b, act, out, 256, stream);
    if (rc) return rc;
  }
  Args q = p;
  q.M = M - (int)r0;
  q.A = p.A + (layout_a == ROW ? r0 * lda : r0);
  if (p.A2) q.A2 = p.A2 + (layout_a == ROW ? r0 * lda2 : r0);
  q.C = (char*)C + r0 * ldc * (out == O_BF16 ? 2 : 4);
  if (p.C2) q.C2 = p.C2 + r0 * ldc2;
  if (p.R) q.R = p.R + r0 * ldr;
  if (p.rope_pos) q.rope_pos = p.rope_pos + r0;
  return launch_gemm_big(q, layout_a, layout_b, act, out, 128, stream);
}

// NT GEMM + rotary epilogue (E_ROPE): C = rope(A B^T (+ A2 B2^T) + bias) for a fused qkv
// projection — output columns [0, rope_cols) are rope_d-wide heads rotated at position pos[row]
// with the [positions, rope_d / 2] fp32 tables; the rest (v heads) are stored as they are. Replaces
// the separate rope_qkv pass over the projection output (one read + write of every q / k element).
// Same wave planner as rt_gemm_big. Requirements: rope_d in {16, 32, 64, 128}, rope_cols % rope_d
// == 0, rope_cols <= N, bf16 out with ldc % 8 == 0, K (K2) % 8 == 0.
extern "C" int rt_gemm_big_rope(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                                const void* B2, long ldb2, int K2, const void* bias, void* C, long ldc, int M, int N,
                                int K, const int* pos, const float* cosT, const float* sinT, int rope_cols, int rope_d,
                                const void* zpage, int bn, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 8 || (A2 && K2 % 8) || !zpage || ldc % 8 || (M > 1 && ldc < (long)((N + 7) / 8 * 8))) return -1;
  if (!pos || !cosT || !sinT || (rope_d != 16 && rope_d != 32 && rope_d != 64 && rope_d != 128) ||
      rope_cols % rope_d || rope_cols > N || rope_cols < 0)
    return -5;
  if (bn != 0 && bn != 128 && bn != 256) return -8;
  Args p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.A2 = (A2 && B2) ? (const bf16_t*)A2 : nullptr; p.lda2 = lda2;
  p.B2 = (const bf16_t*)B2; p.ldb2 = ldb2; p.K2 = K2;
  p.bias = (const bf16_t*)bias; p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = E_ROPE; p.nsplit = 1; p.zpage = (const bf16_t*)zpage;
  p.group_m = tuning().gemm_group_m;
  p.rope_pos = pos; p.rope_cos = cosT; p.rope_sin = sinT; p.rope_cols = rope_cols; p.rope_d = rope_d;
  return gemm_big_planned(p, ROW, ROW, E_ROPE, O_BF16, bn, stream);
}

// W8A8 on the gemm_big schedule (config 5 prefill / reference scoring): A [M, K] e4m3fn with
// per-row scales sa, B [N, K] e4m3fn with per-row scales sb, C = act(A B^T * sa sb^T + bias) bf16
// (E_SWIGLU: B = [gate; up], C [M, N / 2]). The fp8 rows are the bf16 kernel's operands at half
// the K (the same 128-B LDS rows, one 16x16x128 MX MFMA per 64-bf16 K-step at twice the bf16
// rate), with the same wave planner: 256x256 tiles, the last partial wave on 256x128.
// A2 [M, K2] / B2 [N, K2] (bf16, optional): a K-extension (LoRA U / UB) run on bf16 MFMAs into
// the same accumulators — the caller pre-divides them by sa / sb so the epilogue scaling leaves
// A2 B2^T as it is. C2 (E_SWIGLU, optional): the bf16 [gate | up] pre-activation, as gemm_big.
extern "C" int rt_gemm_big_fp8(const void* A, long lda, const float* sa, const void* B, long ldb, const float* sb,
                               const void* bias, void* C, long ldc, int M, int N, int K, int act,
                               const void* A2, long lda2, const void* B2, long ldb2, int K2, void* C2, long ldc2,
                               const void* zpage, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 || lda % 16 || ldb % 16 || ldc % 8 || (act != E_NONE && act != E_SWIGLU)) return -1;
  if (act == E_SWIGLU && N % 256) return -3;
  if ((A2 || B2) && (!A2 || !B2 || K2 % 8 || !zpage)) return -4;
  Args p{};
  p.A = (const bf16_t*)A; p.lda = lda / 2; p.B = (const bf16_t*)B; p.ldb = ldb / 2;
  p.A2 = (const bf16_t*)A2; p.lda2 = lda2; p.B2 = (const bf16_t*)B2; p.ldb2 = ldb2; p.K2 = A2 ? K2 : 0;
  p.bias = (const bf16_t*)bias; p.C = C; p.ldc = ldc; p.C2 = (bf16_t*)C2; p.ldc2 = ldc2; p.R = nullptr; p.ldr = 0;
  p.M = M; p.N = N; p.K = K / 2; p.act = act; p.nsplit = 1; p.zpage = (const bf16_t*)(zpage ? zpage : A);
  p.sa = sa; p.sb = sb;
  const int tiles_m = (M + 255) / 256;
  const int tn256 = act == E_SWIGLU ? N / 256 : (N + 255) / 256;
  const int tn128 = act == E_SWIGLU ? N / 128 : (N + 127) / 128;
  const long cus = (long)num_cus();
  int m1 = tiles_m;
  float best = 1e30f;
  for (int m = tiles_m; m >= 0; --m) {
    const long w256 = ((long)m * tn256 + cus - 1) / cus, w128 = ((long)(tiles_m - m) * tn128 + cus - 1) / cus;
    const float cost = (float)w256 + bn128_cost() * (float)w128;
    if (cost < best - 1e-3f) { best = cost; m1 = m; }
  }
  auto launch = [&](const Args& q, int bn) {
    const int tn = bn == 256 ? (act == E_SWIGLU ? q.N / 256 : (q.N + 255) / 256) : (act == E_SWIGLU ? q.N / 128 : (q.N + 127) / 128);
    dim3 grid(((q.M + 255) / 256) * tn, 1), block(512);
    if (bn == 256) {
      if (act == E_SWIGLU) hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_BF16, E_SWIGLU, 256, true>), grid, block, 0, stream, q);
      else hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_BF16, E_NONE, 256, true>), grid, block, 0, stream, q);
    } else {
      if (act == E_SWIGLU) hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_BF16, E_SWIGLU, 128, true>), grid, block, 0, stream, q);
      else hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_BF16, E_NONE, 128, true>), grid, block, 0, stream, q);
    }
  };
  if (m1 > 0) {
    Args q = p;
    q.M = std::min(M, m1 * 256);
    launch(q, 256);
  }
  if (m1 < tiles_m) {
    const long r0 = (long)m1 * 256;
    Args q = p;
    q.M = M - (int)r0;
    q.A = p.A + r0 * p.lda;
    if (p.A2) q.A2 = p.A2 + r0 * p.lda2;
    q.sa = sa + r0;
    q.C = (char*)C + r0 * ldc * 2;
    if (p.C2) q.C2 = p.C2 + r0 * p.ldc2;
    launch(q, 128);
  }
  RT_LAUNCH_CHECK();
  return 0;
}

// W8A8 split-K into fp32 slabs [nsplit][M][N] (decode at batch > 64, config 5): the split
// partials carry sa[row] * sb[col] and are summed by the consumer (the norm / attention
// prologue, as the bf16 slab GEMMs' — ops.linear_deferred). bn 128 or 256, N % 8 == 0.
extern "C" int rt_gemm_big_fp8_slabs(const void* A, long lda, const float* sa, const void* B, long ldb, const float* sb,
                                     float* slabs, int M, int N, int K, int nsplit, int bn, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 || lda % 16 || ldb % 16 || N % 8 || nsplit < 1 || (bn != 128 && bn != 256)) return -1;
  Args p{};
  p.A = (const bf16_t*)A; p.lda = lda / 2; p.B = (const bf16_t*)B; p.ldb = ldb / 2;
  p.C = slabs; p.ldc = N;
  p.M = M; p.N = N; p.K = K / 2; p.act = E_NONE; p.nsplit = nsplit; p.zpage = (const bf16_t*)A;
  p.sa = sa; p.sb = sb;
  p.group_m = tuning().gemm_group_m;
  const int tn = bn == 256 ? (N + 255) / 256 : (N + 127) / 128;
  dim3 grid(((M + 255) / 256) * tn, nsplit), block(512);
  if (bn == 256) hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_F32_SLAB, E_NONE, 256, true>), grid, block, 0, stream, p);
  else hipLaunchKernelGGL((gemm_big_kernel<ROW, ROW, O_F32_SLAB, E_NONE, 128, true>), grid, block, 0, stream, p);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_gemm_splitk_reduce(const float* slabs, int nsplit, int M, int N, const void* bias, int act,
                                     const void* R, long ldr, void* C, long ldc, hipStream_t stream) {
  const int Nout = act == E_SWIGLU ? N / 2 : N;
  if (Nout % 8 || M <= 0) return M <= 0 ? 0 : -1;
  const long work = (long)M * (Nout / 8);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, slabs, nsplit,
                     M, N, (const bf16_t*)bias, act, (const bf16_t*)R, ldr, (bf16_t*)C, ldc);
  RT_LAUNCH_CHECK();
  return 0;
}

// 64x64-tile GEMM (narrow LoRA products). out: 0 bf16, 1 fp32 store, 2 fp32 atomic add (split-K),
// 3 fp32 split-K slabs [nsplit][M][ldc] summed in a fixed order by their consumer (the forward U,
// the backward dU, dA and dB: bitwise-reproducible LoRA products).
extern "C" int rt_gemm_small(int layout_a, int layout_b, const void* A, long lda, const void* B, long ldb, void* C,
                             long ldc, int M, int N, int K, int out, int nsplit, const void* zpage, int bm,
                             hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (!zpage || ((layout_a == ROW || layout_b == ROW) && K % 8)) return -1;
  if ((layout_a == KMAJ && M % 8) || (layout_b == KMAJ && N % 8)) return -1;
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 1 && out != O_F32_ATOMIC && out != O_F32_SLAB) return -2;
  Args p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K; p.nsplit = nsplit; p.zpage = (const bf16_t*)zpage;
  if (bm != 64 && bm != 128) return -5;
  dim3 grid(((M + bm - 1) / bm) * ((N + 63) / 64), nsplit), block(256);
  const int key = layout_a * 100 + layout_b * 10 + out;
#define GS_LAUNCH(LA, LB, O)                                                                   \
  do {                                                                                         \
    if (bm == 128) hipLaunchKernelGGL((gemm_small_kernel<LA, LB, O, 128>), grid, block, 0, stream, p); \
    else hipLaunchKernelGGL((gemm_small_kernel<LA, LB, O, 64>), grid, block, 0, stream, p);          \
  } while (0)
  switch (key) {
    case 0: GS_LAUNCH(ROW, ROW, O_BF16); break;
    case 1: GS_LAUNCH(ROW, ROW, O_F32); break;
    case 2: GS_LAUNCH(ROW, ROW, O_F32_ATOMIC); break;
    case 3: GS_LAUNCH(ROW, ROW, O_F32_SLAB); break;
    case 10: GS_LAUNCH(ROW, KMAJ, O_BF16); break;
    case 11: GS_LAUNCH(ROW, KMAJ, O_F32); break;
    case 12: GS_LAUNCH(ROW, KMAJ, O_F32_ATOMIC); break;
    case 13: GS_LAUNCH(ROW, KMAJ, O_F32_SLAB); break;
    case 112: GS_LAUNCH(KMAJ, KMAJ, O_F32_ATOMIC); break;
    case 113: GS_LAUNCH(KMAJ, KMAJ, O_F32_SLAB); break;
    case 111: GS_LAUNCH(KMAJ, KMAJ, O_F32); break;
    default: return -4;
  }
#undef GS_LAUNCH
  RT_LAUNCH_CHECK();
  return 0;
}
