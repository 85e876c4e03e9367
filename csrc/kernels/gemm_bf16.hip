// bf16 MFMA GEMM for gfx950 with a fused LoRA K-extension and bias/activation epilogue.
//
//   C[M,N] = act( A[M,K] · B[N,K]^T  +  U[M,Rp] · UB[N,Rp]^T  +  bias[N] )
//
// Both operands are K-contiguous ("NT"), which is the nn.Linear layout (weight [out,in]).
// The LoRA term of a LoRA-adapted projection  Y = X W^T + s (X A^T) B^T  is carried as extra
// K-steps: U = s·X·A^T (computed by a small pass, zero-padded to Rp = multiple of 64) and
// UB = B (zero-padded, block-diagonal when several adapters share one fused projection, e.g.
// q|k|v). The adapter product therefore runs on the same MFMA pipeline and accumulators as the
// frozen base weight — no separate output pass, no extra read/write of Y.
//
// The weight-streaming kernels for M <= 64 (decode / small batch): gemm_decode_kernel (64 columns
// per wave, split-K over waves and workgroups with an in-launch last-arriver reduction),
// gemv16_kernel (M <= 16 on tile-ordered weight images), gemm_m64_kernel (16 < M <= 64, LDS-DMA
// ring) and the W8A16 forms. M > 64 runs on the token-parallel family of gemm_big.hip.
//
// Replaces every projection GEMM of the reference's HF forward passes (reference
// call sites reinforcement_learning_optimization_after_rag.py:38,200,207,313,318).
#include "rt_common.h"
#include "rt_workspace.h"

#include <cmath>

namespace rt {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_TANH = 3, ACT_SILU = 4,
           // skinny kernels only: B = fused [gate; up] weight (2F rows), C[M, F] = silu(X gate^T) * (X up^T).
           // Column group g reads gate rows [32g, 32g+32) and up rows [F+32g, F+32g+32), so the pair of
           // every output lands in one lane (SwiGLU fused into the gate/up GEMM of a decode step)
           ACT_SWIGLU = 5 };

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
    }
    case ACT_SILU: return x / (1.f + __expf(-x));
    default: return x;
  }
}

struct GemmArgs {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  const bf16_t* U; long ldu;     // LoRA down-projection output (may be null)
  const bf16_t* UB; long ldub;   // LoRA up weight (may be null)
  int Rp;                        // padded LoRA rank (multiple of 64, 0 = none)
  const bf16_t* bias;            // [N] or null
  void* C; long ldc;
  int M, N, K;
  int act;
  // fp8 paths only: per-row scale of A (W8A8 tile kernel) and per-column scale of B (W8A8 and
  // W8A16 skinny kernel); A / B then point to OCP e4m3fn bytes with lda / ldb in elements (= bytes)
  const float* sa;
  const float* sb;
  // skinny kernels only (decode): residual added after the activation (C = act(..) + R, the new
  // residual stream) and RMS-normalised input (C = rstd(X) * X B'^T with the norm weight folded
  // into B'; rstd(X_row) = rsqrt(mean(X_row^2) + eps) is computed inside the GEMM, 0 = off)
  const bf16_t* R; long ldr;
  float norm_eps;
  // decode kernel only: B is in the MFMA-fragment order of shuffle_decode_weight (each 16-row x
  // 64-k tile = 2 KiB contiguous, one 1-KiB run per load instruction) instead of row-major
  int wshuf;
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

__device__ __forceinline__ i32x8 cat_frag(const bf16x8& lo, const bf16x8& hi) {
  const i32x4_t a = __builtin_bit_cast(i32x4_t, lo), b = __builtin_bit_cast(i32x4_t, hi);
  return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// 16-B slot swizzle of a 128-B-row LDS tile read by ds_read_b128 in 16-row lane groups: two rows
// share a 256-B bank row, so the XOR key must differ between rows r and r+8 of the same parity.
// (r >> 1) & 7 makes any 16 consecutive rows hit 16 distinct slots (conflict-free); (r & 7)
// would put rows r and r+8 on the same banks (2-way). Applied on the glds SOURCE address and on
// the read (rule 21).
__device__ __forceinline__ int lds_swz(int row) { return (row >> 1) & 7; }


// ---------------------------------------------------------------------------------------------
// Decode GEMM (M <= 64): weight streaming with split-K and an in-launch last-arriver reduction
// ---------------------------------------------------------------------------------------------
// Work unit: one column group of 64 output columns (4 MFMA B fragments) x a K range. A wave owns
// 64 columns x (K / (4*split)), so every X fragment feeds 4 MFMAs (X:W traffic 1:1 at M = 64
// instead of 4:1 with 16-column waves). Its W rows stream straight to VGPRs (read once: no LDS,
// cdna_hip_programming.md §5 'GEMV / M <= 16'), one 64-deep k-chunk ahead in two named register
// sets (no runtime-indexed register arrays). Per 64-chunk the fragments follow the MFMA's own k
// layout (lane group g = lane>>4 holds k [8g, 8g+8) of each 32-deep half), so each 16-B load
// instruction reads 64 contiguous bytes of 16 weight rows. (A layout where a lane group owned one
// 32-B run per row measured the same; an HBM pattern probe, tools/microbench/hbm_pattern.hip, puts
// this 16-rows x 128-B step at 5.9 TB/s vs 6.3-6.7 for 512-B..1-KiB row spans.)
// Reduction: the 4 waves of a block sum through LDS; the `split` blocks of a column group publish
// fp32 slabs and the LAST arriver (agent-scope release -> relaxed ticket -> agent-scope acquire,
// §6 Guideline 16 / §5 'In-launch split-K reduction') sums them and runs the epilogue (LoRA U*UB^T,
// bias, activation, bf16/fp32 store), then re-arms the ticket for the next launch (graph replay).
constexpr int DG_COLS = 64;

template <int MT>
struct DGRegs {
  uint4 w[4][2];
  uint4 x[MT][2];
};

// W8: the weight row is OCP e4m3fn bytes (W8A16): one 16-B load covers the lane's 16 k of a
// 64-deep chunk and is widened to two bf16x8 fragments in registers (per-column scale applied in
// the epilogue). The k order matches the bf16 X fragments (lane group g owns k [16g, 16g+16)).
template <int MT, bool W8>
__device__ __forceinline__ void dg_load(DGRegs<MT>& r, const char* const* wrow, const bf16_t* const* xrow, long c,
                                        long wstep, long hoff) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // weights are read once per launch: non-temporal (MI355X_MICROARCH.md 'nt-weights')
    if constexpr (W8) {
      r.w[j][0] = load_nt16(wrow[j] + c * 64);
    } else {
      r.w[j][0] = load_nt16(wrow[j] + c * wstep);
      r.w[j][1] = load_nt16(wrow[j] + c * wstep + hoff);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    r.x[m][0] = *(const uint4*)(xrow[m] + c * 64);
    r.x[m][1] = *(const uint4*)(xrow[m] + c * 64 + (W8 ? 8 : 32));
  }
}

template <int MT, bool W8>
__device__ __forceinline__ void dg_mma(const DGRegs<MT>& r, f32x4 (&acc)[MT][4]) {
  bf16x8 w0[4], w1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (W8) {
      w0[j] = fp8x8_to_bf16(r.w[j][0].x, r.w[j][0].y);
      w1[j] = fp8x8_to_bf16(r.w[j][0].z, r.w[j][0].w);
    } else {
      w0[j] = __builtin_bit_cast(bf16x8, r.w[j][0]);
      w1[j] = __builtin_bit_cast(bf16x8, r.w[j][1]);
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x[m][0]), w0[j], acc[m][j], 0, 0, 0);
      acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x[m][1]), w1[j], acc[m][j], 0, 0, 0);
    }
}

template <int MT, bool OUT_F32, bool W8, int DEPTH>
__global__ __launch_bounds__(256, 2) void gemm_decode_kernel(GemmArgs p, float* __restrict__ slabs,
                                                          unsigned* __restrict__ tickets, int split) {
  constexpr int ROWS = MT * 16;
  constexpr int LDR = DG_COLS + 1;
  __shared__ float red[4 * ROWS * LDR + 4 * ROWS];  // the ONLY __shared__ object (+ per-wave row sum-of-squares)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cg = blockIdx.x / split, sp = blockIdx.x % split;
  const int n0 = cg * DG_COLS;
  const int frow = lane & 15, g = lane >> 4;

  const int nc = p.K / 64;
  const int part = sp * 4 + wid, nparts = split * 4;
  const int c_begin = (int)((long)part * nc / nparts), c_end = (int)((long)(part + 1) * nc / nparts);

  constexpr int WSZ = W8 ? 1 : 2;  // bytes per weight element
  const bool pair = p.act == ACT_SWIGLU;
  const int F = p.N / 2;
  const char* wrow[4];
  const bf16_t* xrow[MT];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int wr_ = pair ? (j < 2 ? cg * 32 + j * 16 + frow : F + cg * 32 + (j - 2) * 16 + frow)
                         : min(n0 + j * 16 + frow, p.N - 1);
    // bf16: lane group g holds k [8g, 8g+8) and [32+8g, 32+8g+8) of each 64-deep chunk (the MFMA's
    // own layout: each load instruction reads 64 contiguous bytes per row); fp8: [16g, 16g+16)
    wrow[j] = (!W8 && p.wshuf) ? (const char*)p.B + ((long)(wr_ >> 4) * nc * 2048 + lane * 16)
                               : (const char*)p.B + ((long)wr_ * p.ldb + g * (W8 ? 16 : 8)) * WSZ;
  }
  // bytes between consecutive k-chunks of one lane / between its two 16-B loads of a chunk
  const long wstep = p.wshuf ? 2048 : 128, hoff = p.wshuf ? 1024 : 64;
#pragma unroll
  for (int m = 0; m < MT; ++m) xrow[m] = p.A + (long)min(m * 16 + frow, p.M - 1) * p.lda + g * (W8 ? 16 : 8);

  f32x4 acc[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool normed = p.norm_eps > 0.f;
  float sq[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) sq[m] = 0.f;
  auto xsq = [&](const DGRegs<MT>& r) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float f[8];
      unpack8(r.x[m][0], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) sq[m] += f[e] * f[e];
      unpack8(r.x[m][1], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) sq[m] += f[e] * f[e];
    }
  };

  // DEPTH register sets: DEPTH-1 chunks stay in flight while one is consumed (chunk c lives in set
  // (c - c_begin) % DEPTH; every index below is a compile-time constant after unrolling)
  DGRegs<MT> r[DEPTH];
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i)
    if (c_begin + i < c_end) dg_load<MT, W8>(r[i], wrow, xrow, c_begin + i, wstep, hoff);
  int c = c_begin;
  for (; c + DEPTH <= c_end; c += DEPTH) {
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
      if (c + i + DEPTH - 1 < c_end) dg_load<MT, W8>(r[(i + DEPTH - 1) % DEPTH], wrow, xrow, c + i + DEPTH - 1, wstep, hoff);
      dg_mma<MT, W8>(r[i], acc);
      if (normed) xsq(r[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i)
    if (c + i < c_end) {
      dg_mma<MT, W8>(r[i], acc);
      if (normed) xsq(r[i]);
    }

  // ---- intra-block reduction: acc[m][j] lane holds C[m*16 + 4g + r][j*16 + frow] ----
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wid * ROWS + m * 16 + g * 4 + r) * LDR + j * 16 + frow] = acc[m][j][r];
  // row sums of squares of X over this wave's k range: lanes of one row differ in g (xor 16, 32)
  float* rsq = red + 4 * ROWS * LDR;
  if (normed) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float t = sq[m];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if (g == 0) rsq[wid * ROWS + m * 16 + frow] = t;
    }
  }
  __syncthreads();
  constexpr int NE = ROWS * DG_COLS / 256;  // elements per thread
  float v[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = tid + 256 * i;
    const int row = e / DG_COLS, col = e % DG_COLS;
    v[i] = red[(0 * ROWS + row) * LDR + col] + red[(1 * ROWS + row) * LDR + col] + red[(2 * ROWS + row) * LDR + col] +
           red[(3 * ROWS + row) * LDR + col];
  }
  // block-level row sum of squares (split-K blocks publish it after their slab)
  float bsq = 0.f;  // thread tid < ROWS holds row tid
  if (normed && tid < ROWS) bsq = rsq[tid] + rsq[ROWS + tid] + rsq[2 * ROWS + tid] + rsq[3 * ROWS + tid];

  if (split > 1) {
    // publish this block's slab with write-through (agent-scope) stores, drain them, take a
    // ticket; the last arriver of the column group reduces with agent-scope loads. No L2
    // writeback/invalidate fences (a per-block buffer_wbl2 flushes the whole XCD L2).
    constexpr int SLAB = ROWS * DG_COLS + ROWS;
    float* slab = slabs + ((long)cg * split + sp) * SLAB;
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + 256 * i;
      if (e / DG_COLS < p.M) __hip_atomic_store(slab + e, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (normed && tid < p.M) __hip_atomic_store(slab + ROWS * DG_COLS + tid, bsq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(tickets + cg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      red[0] = (old == (unsigned)(split - 1)) ? 1.f : 0.f;
    }
    __syncthreads();
    const bool last = red[0] != 0.f;
    if (!last) return;
    const float* base = slabs + (long)cg * split * SLAB;
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + 256 * i;
      float t = 0.f;
      if (e / DG_COLS < p.M) {
#pragma unroll 8
        for (int s2 = 0; s2 < split; ++s2)
          t += __hip_atomic_load(base + (long)s2 * SLAB + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      v[i] = t;
    }
    if (normed && tid < p.M) {
      float t = 0.f;
#pragma unroll 8
      for (int s2 = 0; s2 < split; ++s2)
        t += __hip_atomic_load(base + (long)s2 * SLAB + ROWS * DG_COLS + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bsq = t;
    }
    if (tid == 0) __hip_atomic_store(tickets + cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // per-row rstd of the normalised input (rows < ROWS), shared through LDS
  if (normed) {
    __syncthreads();
    if (tid < ROWS) rsq[tid] = rsqrtf(bsq / (float)p.K + p.norm_eps);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NE; ++i) v[i] *= rsq[(tid + 256 * i) / DG_COLS];
  }

  if (pair) {
    // stage the 64 sums of this group (32 gate | 32 up) through LDS, then pair them up
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + 256 * i;
      const int row = e / DG_COLS, col = e % DG_COLS;
      const int wcol = col < 32 ? cg * 32 + col : F + cg * 32 + col - 32;
      float y = v[i];
      if constexpr (W8) y *= p.sb[wcol];
      if (p.bias) y += bf2f(p.bias[wcol]);
      red[row * LDR + col] = y;
    }
    __syncthreads();
    for (int e = tid; e < ROWS * 32; e += 256) {
      const int row = e / 32, c = e % 32;
      if (row >= p.M) continue;
      const float gt = red[row * LDR + c], up = red[row * LDR + c + 32];
      const float y = gt / (1.f + __expf(-gt)) * up;
      if constexpr (OUT_F32) ((float*)p.C)[(long)row * p.ldc + cg * 32 + c] = y;
      else ((bf16_t*)p.C)[(long)row * p.ldc + cg * 32 + c] = f2bf(y);
    }
    return;
  }

  // ---- epilogue: LoRA K-extension (U UB^T), bias, activation, store ----
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = tid + 256 * i;
    const int row = e / DG_COLS, col = e % DG_COLS;
    const int grow = row, gcol = n0 + col;
    if (grow < p.M && gcol < p.N) {
      float y = v[i];
      if (p.Rp > 0) {
        const bf16_t* ur = p.U + (long)grow * p.ldu;
        const bf16_t* br = p.UB + (long)gcol * p.ldub;
        for (int k = 0; k < p.Rp; k += 8) {
          float a8[8], b8[8];
          unpack8(*(const uint4*)(ur + k), a8);
          unpack8(*(const uint4*)(br + k), b8);
#pragma unroll
          for (int q = 0; q < 8; ++q) y += a8[q] * b8[q];
        }
      }
      if constexpr (W8) y *= p.sb[gcol];
      if (p.bias) y += bf2f(p.bias[gcol]);
      y = apply_act(y, p.act);
      if (p.R) y += bf2f(p.R[(long)grow * p.ldr + gcol]);
      if constexpr (OUT_F32) ((float*)p.C)[(long)grow * p.ldc + gcol] = y;
      else ((bf16_t*)p.C)[(long)grow * p.ldc + gcol] = f2bf(y);
    }
  }
}

// CU count of the current device, queried once (thread-safe static initialisation)
static int gemv_cus() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        c <= 0)
      c = 256;
    return c;
  }();
  return n;
}

// ---------------------------------------------------------------------------------------------
// Decode GEMV (M <= 16) without split-K: one workgroup per 16 weight rows of a tile-ordered image
// ---------------------------------------------------------------------------------------------
// The split-K decode kernel above ends in a serial hand-off (write-through slab stores drained,
// an arrival ticket, the last arriver's slab loads): about three dependent device-memory round
// trips after the last weight byte lands. Here a workgroup owns one 16-row group of the
// tile-ordered image (its K chunks are ONE contiguous run of nc x 2 KiB) and its 4 waves split K;
// the partial sums meet in LDS, so the tail is a workgroup barrier. N / 16 workgroups (256 for
// o / down, 384 for qkv) fill the chip without a K split. Each wave keeps DEPTH - 1 k-chunks in
// flight (non-temporal: every weight byte is read once per step). The M <= 16 rows of X are the
// MFMA's 16 A rows. Same epilogue contract as gemm_decode_kernel: in-GEMM RMS norm (folded weight,
// per-row rstd from the X fragments), bias, activation, residual, bf16 / fp32 store; SwiGLU as a
// gate / up row-group pair. Batch 1: 3.28 -> 2.92 ms/token (profiles/decode_b1_gemv16_ab.log).
//
// PAIR (SwiGLU, weight = [gate; up], 2F rows): the workgroup owns output columns [16 grp, 16 grp +
// 16) and streams the gate row group grp and the up row group F / 16 + grp side by side.
//
// W8 (W8A16, config 5): the image is the fp8 tile order of shuffle_decode_weight_fp8 — per 16-row
// group, 2-KiB chunks of 128 k; load h of lane l = 16 g + r holds the 16 e4m3fn bytes of row r at
// k [128 c + 64 h + 16 g, +16), widened in registers to two bf16x8 fragments (k-slot permutation
// shared with the X fragments, so the MFMA sums the same products). Half the bytes per chunk of k
// of the bf16 image; per-column scales sb[col] applied in the epilogue.
template <bool OUT_F32, int DEPTH, bool PAIR, bool W8 = false, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemv16_kernel(GemmArgs p) {
  // M <= 16 rows of X: the MFMA's 16 A rows (row frow of lane (frow, g); rows >= M repeat M - 1)
  // NW waves split the group's K chunks (NW = 8: twice the weight bytes in flight per workgroup)
  __shared__ float red[NW][16][PAIR ? 33 : 17];
  __shared__ float rsq[NW][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, g = lane >> 4;
  const int grp = blockIdx.x;  // 16-row group (of the gate rows when PAIR)
  constexpr int KC = W8 ? 128 : 64;  // k per 2-KiB chunk
  const int nc = p.K / KC;
  const int c_begin = wid * nc / NW, c_end = (wid + 1) * nc / NW;
  const char* wbase = (const char*)p.B + (long)grp * nc * 2048 + lane * 16;
  const char* ubase = PAIR ? (const char*)p.B + ((long)(p.N / 32) + grp) * nc * 2048 + lane * 16 : wbase;
  const bf16_t* xrow = p.A + (long)min(frow, p.M - 1) * p.lda + g * (W8 ? 16 : 8);
  struct Regs { uint4 w0, w1, u0, u1, x0, x1, x2, x3; };
  auto ld = [&](Regs& r, int c) {
    r.w0 = load_nt16(wbase + (long)c * 2048);
    r.w1 = load_nt16(wbase + (long)c * 2048 + 1024);
    if constexpr (PAIR) {
      r.u0 = load_nt16(ubase + (long)c * 2048);
      r.u1 = load_nt16(ubase + (long)c * 2048 + 1024);
    }
    if constexpr (W8) {  // k [128 c + 64 h + 16 g, +16) as two 8-element halves, h = 0, 1
      r.x0 = *(const uint4*)(xrow + c * 128);
      r.x1 = *(const uint4*)(xrow + c * 128 + 8);
      r.x2 = *(const uint4*)(xrow + c * 128 + 64);
      r.x3 = *(const uint4*)(xrow + c * 128 + 72);
    } else {
      r.x0 = *(const uint4*)(xrow + c * 64);
      r.x1 = *(const uint4*)(xrow + c * 64 + 32);
    }
  };
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f}, accu = acc;
  float sq = 0.f;
  const bool normed = p.norm_eps > 0.f;
  auto mma = [&](const Regs& r) {
    if constexpr (W8) {
      const bf16x8 x0 = __builtin_bit_cast(bf16x8, r.x0), x1 = __builtin_bit_cast(bf16x8, r.x1);
      const bf16x8 x2 = __builtin_bit_cast(bf16x8, r.x2), x3 = __builtin_bit_cast(bf16x8, r.x3);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, fp8x8_to_bf16(r.w0.x, r.w0.y), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, fp8x8_to_bf16(r.w0.z, r.w0.w), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, fp8x8_to_bf16(r.w1.x, r.w1.y), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x3, fp8x8_to_bf16(r.w1.z, r.w1.w), acc, 0, 0, 0);
      if constexpr (PAIR) {
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, fp8x8_to_bf16(r.u0.x, r.u0.y), accu, 0, 0, 0);
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, fp8x8_to_bf16(r.u0.z, r.u0.w), accu, 0, 0, 0);
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, fp8x8_to_bf16(r.u1.x, r.u1.y), accu, 0, 0, 0);
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x3, fp8x8_to_bf16(r.u1.z, r.u1.w), accu, 0, 0, 0);
      }
    } else {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x0), __builtin_bit_cast(bf16x8, r.w0), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x1), __builtin_bit_cast(bf16x8, r.w1), acc, 0, 0, 0);
      if constexpr (PAIR) {
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x0), __builtin_bit_cast(bf16x8, r.u0), accu, 0, 0, 0);
        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r.x1), __builtin_bit_cast(bf16x8, r.u1), accu, 0, 0, 0);
      }
    }
    if (normed) {
      float f[8];
      unpack8(r.x0, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) sq += f[e] * f[e];
      unpack8(r.x1, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) sq += f[e] * f[e];
      if constexpr (W8) {
        unpack8(r.x2, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) sq += f[e] * f[e];
        unpack8(r.x3, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) sq += f[e] * f[e];
      }
    }
  };
  Regs r[DEPTH];
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i)
    if (c_begin + i < c_end) ld(r[i], c_begin + i);
  int c = c_begin;
  for (; c + DEPTH <= c_end; c += DEPTH) {
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
      if (c + i + DEPTH - 1 < c_end) ld(r[(i + DEPTH - 1) % DEPTH], c + i + DEPTH - 1);
      mma(r[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < DEPTH - 1; ++i)
    if (c + i < c_end) mma(r[i]);
  // acc[r] of lane (frow, g) = C[row 4 g + r][16 grp + frow] over this wave's k range; the X row
  // sum of squares of row frow is spread over its 4 g lanes
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    red[wid][4 * g + rr][frow] = acc[rr];
    if constexpr (PAIR) red[wid][4 * g + rr][16 + frow] = accu[rr];
  }
  if (normed) {
    float t = sq;
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (g == 0) rsq[wid][frow] = t;
  }
  __syncthreads();
  const int row = tid >> 4, ci = tid & 15;
  if (row < p.M) {
    const int col = grp * 16 + ci;
    // wave partials summed in wave order (NW = 4: the association of the original four-term sum)
    float ss = 0.f, yy = 0.f, uu = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      ss += rsq[w][row];
      yy += red[w][row][ci];
      if constexpr (PAIR) uu += red[w][row][16 + ci];
    }
    const float rs = normed ? rsqrtf(ss / (float)p.K + p.norm_eps) : 1.f;
    float y = yy * rs;
    if constexpr (PAIR) {
      const int F = p.N / 2;
      float up = uu * rs;
      if constexpr (W8) { y *= p.sb[col]; up *= p.sb[F + col]; }
      if (p.bias) { y += bf2f(p.bias[col]); up += bf2f(p.bias[F + col]); }
      y = y / (1.f + __expf(-y)) * up;
    } else {
      if constexpr (W8) y *= p.sb[col];
      if (p.bias) y += bf2f(p.bias[col]);
      y = apply_act(y, p.act);
      if (p.R) y += bf2f(p.R[(long)row * p.ldr + col]);
    }
    if constexpr (OUT_F32) ((float*)p.C)[(long)row * p.ldc + col] = y;
    else ((bf16_t*)p.C)[(long)row * p.ldc + col] = f2bf(y);
  }
}

// Shared tail of the M <= 64 kernels: split-K hand-off (write-through slabs + ticket, last arriver
// reduces), in-GEMM RMS-norm scaling, SwiGLU pair / bias + activation + residual epilogues.
// acc[j][r] = C[16 wid + 4 fq + r][16 j + frow] of the block's 64 columns; sq = sum of squares of
// X row (16 wid + frow) over this block's K range (norm only).
template <bool OUT_F32, bool W8 = false>
__device__ __forceinline__ void m64_finish(const GemmArgs& p, f32x4 (&acc)[4], float sq, float* __restrict__ slabs,
                                           unsigned* __restrict__ tickets, int split, int cg, int sp, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const int n0 = cg * 64;
  const bool normed = p.norm_eps > 0.f;
  const bool pair = p.act == ACT_SWIGLU;
  const int F = p.N / 2;
  // lane holds C[16 wid + 4 fq + r][16 j + frow]
  if (split > 1) {
    constexpr int SLAB = 64 * 64 + 64;
    float* slab = slabs + ((long)cg * split + sp) * SLAB;
    if (normed && fq == 0 && wid * 16 + frow < p.M)
      __hip_atomic_store(slab + 4096 + wid * 16 + frow, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wid * 16 + fq * 4 + r;
        if (row < p.M)
          __hip_atomic_store(slab + row * 64 + j * 16 + frow, acc[j][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(tickets + cg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (old == (unsigned)(split - 1));
    }
    __syncthreads();
    if (!*flag) return;
    const float* base = slabs + (long)cg * split * SLAB;
    if (normed) {
      float t = 0.f;
      if (wid * 16 + frow < p.M) {
#pragma unroll 8
        for (int s2 = 0; s2 < split; ++s2)
          t += __hip_atomic_load(base + (long)s2 * SLAB + 4096 + wid * 16 + frow, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      sq = t;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wid * 16 + fq * 4 + r;
        float t = 0.f;
        // unrolled: the partial loads are independent and must all be in flight at once (a
        // rolled loop waits one L2/MALL round trip per split)
        if (row < p.M) {
#pragma unroll 8
          for (int s2 = 0; s2 < split; ++s2)
            t += __hip_atomic_load(base + (long)s2 * SLAB + row * 64 + j * 16 + frow, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        acc[j][r] = t;
      }
    if (tid == 0) __hip_atomic_store(tickets + cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (normed) {
    // lane holds rows 16 wid + 4 fq + r; their sums of squares sit in lanes 4 fq + r of this wave
    const float rs = rsqrtf(sq / (float)p.K + p.norm_eps);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float rr = __shfl(rs, fq * 4 + r, 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j][r] *= rr;
    }
  }
  if (pair) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = cg * 32 + j * 16 + frow;
      const float bg = p.bias ? bf2f(p.bias[col]) : 0.f, bu = p.bias ? bf2f(p.bias[F + col]) : 0.f;
      const float sg = W8 ? p.sb[col] : 1.f, su = W8 ? p.sb[F + col] : 1.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wid * 16 + fq * 4 + r;
        if (row >= p.M) continue;
        const float gt = acc[j][r] * sg + bg, up = acc[j + 2][r] * su + bu;
        const float y = gt / (1.f + __expf(-gt)) * up;
        if constexpr (OUT_F32) ((float*)p.C)[(long)row * p.ldc + col] = y;
        else ((bf16_t*)p.C)[(long)row * p.ldc + col] = f2bf(y);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + j * 16 + frow;
    if (col >= p.N) continue;
    const float bv = p.bias ? bf2f(p.bias[col]) : 0.f;
    const float sc = W8 ? p.sb[col] : 1.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wid * 16 + fq * 4 + r;
      if (row >= p.M) continue;
      float y = apply_act(acc[j][r] * sc + bv, p.act);
      if (p.R) y += bf2f(p.R[(long)row * p.ldr + col]);
      if constexpr (OUT_F32) ((float*)p.C)[(long)row * p.ldc + col] = y;
      else ((bf16_t*)p.C)[(long)row * p.ldc + col] = f2bf(y);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// M in (16, 64]: LDS-DMA ring GEMM (rollout decode at batch 64)
// ---------------------------------------------------------------------------------------------
// Block = 4 waves, 64 output columns x all (<= 64) rows x a K range (split-K over workgroups).
// Each 64-deep K-step stages X[64 x 64] and W[64 x 64] (8 KiB each, 2 x 16-B global_load_lds
// per lane per operand) into one slot of a 4-slot ring; three steps stay in flight (counted
// vmcnt, raw s_barrier — never __syncthreads inside the loop, which would drain the DMA queue),
// so ~96 KiB per CU of loads are outstanding at 2 blocks/CU without costing VGPRs. Wave w owns
// rows [16w, 16w+16) x 64 columns (4 MFMA fragments). Split-K partials use the write-through
// ticket hand-off of gemm_decode_kernel.
constexpr int R64_SLOTS = 4;
constexpr int R64_SLOT = 2 * 64 * 128;  // X + W, 64 rows x 128 B each
//
// W8 (W8A16, config 5): B is the fp8 tile-ordered image of shuffle_decode_weight_fp8 (16-row
// groups, 2-KiB chunks of 128 k; lane l = 16 g + r of half h holds row r, k [64 h + 16 g, +16)).
// A 64-deep K-step of one 16-row group is ONE contiguous 1-KiB run: each wave stages one group
// with one 16-B LDS-DMA per lane (half the weight bytes of the bf16 ring, and 1-KiB DRAM runs
// instead of 64-B row pieces — the row-major fp8 form of this ring measured slower than bf16).
// The fragment of lane (frow, fq) for MFMA step kk is k [32 kk + 8 fq, +8) of row frow = the
// 8-B half (fq & 1) of unit g = 2 kk + (fq >> 1): conflict-free ds_read_b64 (4 r + 2 fq + e),
// widened to bf16 in registers; per-column scales in the epilogue.
template <bool OUT_F32, bool W8 = false>
__global__ __launch_bounds__(256, 2) void gemm_m64_kernel(GemmArgs p, float* __restrict__ slabs,
                                                          unsigned* __restrict__ tickets, int split) {
  __shared__ __attribute__((aligned(16))) char smem[R64_SLOTS * R64_SLOT];  // the only __shared__ object
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cg = blockIdx.x / split, sp = blockIdx.x % split;
  const int n0 = cg * 64;
  const int frow = lane & 15, fq = lane >> 4;
  const int nk = p.K / 64;
  const int t0 = (int)((long)sp * nk / split), t1 = (int)((long)(sp + 1) * nk / split);
  const int nt = t1 - t0;
  const bool pair = p.act == ACT_SWIGLU;
  const int F = p.N / 2;

  // staging: lane -> (row within an 8-row piece, 16-B slot); 2 pieces per operand per wave
  const int srow = lane >> 3;
  auto stage = [&](int t) {  // K-step t (absolute) -> slot (t - t0) % R64_SLOTS
    char* slot = smem + ((t - t0) % R64_SLOTS) * R64_SLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lr = (wid * 2 + j) * 8 + srow;  // 0..63
      const int ck = (lane & 7) ^ lds_swz(lr);
      const bf16_t* xa = p.A + (long)min(lr, p.M - 1) * p.lda + (long)t * 64 + ck * 8;
      __builtin_amdgcn_global_load_lds((const void*)xa, (lds_void*)(slot + (wid * 2 + j) * 1024), 16, 0, 0);
      if constexpr (!W8) {
        const int wrow_ = pair ? (lr < 32 ? cg * 32 + lr : F + cg * 32 + lr - 32) : min(n0 + lr, p.N - 1);
        const bf16_t* wb = p.B + (long)wrow_ * p.ldb + (long)t * 64 + ck * 8;
        __builtin_amdgcn_global_load_lds((const void*)wb, (lds_void*)(slot + 8192 + (wid * 2 + j) * 1024), 16, 0, 0);
      }
    }
    if constexpr (W8) {  // wave wid stages 16-row group G, k-half t & 1 of chunk t >> 1: one 1-KiB run
      const int G = pair ? (wid < 2 ? 2 * cg + wid : F / 16 + 2 * cg + wid - 2) : min(4 * cg + wid, p.N / 16 - 1);
      const char* wb = (const char*)p.B + ((long)G * (p.K / 128) + (t >> 1)) * 2048 + (t & 1) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)wb, (lds_void*)(slot + 8192 + wid * 1024), 16, 0, 0);
    }
  };
  constexpr int PER = W8 ? 3 : 4;  // LDS-DMAs per lane per K-step

  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool normed = p.norm_eps > 0.f;
  float sq = 0.f;

  // prologue: steps t0 .. t0+2 in flight
#pragma unroll
  for (int i = 0; i < R64_SLOTS - 1; ++i)
    if (i < nt) stage(t0 + i);

  for (int i = 0; i < nt; ++i) {
    // retire step i (PER DMAs per lane per step); later steps stay in flight
    const int ahead = min(R64_SLOTS - 2, nt - 1 - i);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    // refill the slot read in the previous iteration (every wave is past it: barrier above)
    if (i + R64_SLOTS - 1 < nt) stage(t0 + i + R64_SLOTS - 1);
    const char* slot = smem + (i % R64_SLOTS) * R64_SLOT;
    bf16x8 a[2], b[4][2];
    const int ar = wid * 16 + frow;
    if constexpr (W8) {
      // fp8 bytes of row frow, k [8c, 8c + 8) = [32 kk + 8 fq, +8) (c = 4 kk + fq): unit 2 kk +
      // (fq >> 1), half fq & 1 of fragment j's 1-KiB piece -> offsets j * 1024 + kk * 512
      rt_u32x2 w8[8];
      ds_read_b64_x8_512(lds_addr(slot + 8192 + ((fq >> 1) * 16 + frow) * 16 + (fq & 1) * 8), w8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) b[j][kk] = fp8x8_to_bf16(w8[2 * j + kk][0], w8[2 * j + kk][1]);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + fq;
      a[kk] = *(const bf16x8*)(slot + ar * 128 + ((c ^ lds_swz(ar)) << 4));
      if constexpr (!W8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int br = j * 16 + frow;
          b[j][kk] = *(const bf16x8*)(slot + 8192 + br * 128 + ((c ^ lds_swz(br)) << 4));
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], b[j][kk], acc[j], 0, 0, 0);
    if (normed) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = (float)a[kk][e];
          sq += f * f;
        }
    }
  }
  // lanes of row (16 wid + frow) differ in fq: the row's sum of squares over this block's K range
  if (normed) {
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
  }
  m64_finish<OUT_F32, W8>(p, acc, sq, slabs, tickets, split, cg, sp, smem);
}

// ---------------------------------------------------------------------------------------------
// W8A16 decode GEMM for 16 < M <= 64 (config-5 rollouts at batch 64): 64 rows x 256 columns
// ---------------------------------------------------------------------------------------------
// The 64-column ring above re-reads all of X for every 64 weight columns: at M = 64 that is
// 2 x the fp8 weight bytes again from L2 (and each of its 4 waves widens the whole fp8 tile).
// Here a workgroup of 8 waves owns 256 weight rows (16 groups of the tile-ordered fp8 image) x a
// K range (split-K over workgroups): per 64-deep K-step one 3-slot LDS ring receives X (64 rows x
// 128 B, one 16-B LDS-DMA per lane) and 16 KiB of fp8 weights (two contiguous 1-KiB image runs
// per wave). Wave w owns 32 columns (image groups 2w, 2w+1; SwiGLU: the gate group and the
// matching up group, so silu(g) * u pairs in registers) x all 64 rows: it widens only its own
// weight bytes (4 ds_read_b64 + 16 cvt per step) and runs 16 MFMAs per step on 4 X fragments.
// X is read from L2 N / 256 times instead of N / 64. Split-K partials: the write-through slab /
// ticket hand-off of the kernels above; epilogue = in-GEMM RMS norm (rstd from the X fragments),
// per-column fp8 scale, bias, activation / SwiGLU, residual.
constexpr int WD_SLOTS = 5;             // 4 K-steps (96 KiB) in flight per workgroup, one workgroup per CU
constexpr int WD_SLOT = 8192 + 16384;  // X (64 x 128 B) + 16 fp8 image groups (1 KiB each)
constexpr int WD_SLAB = 64 * 256 + 64;  // split-K partial tile + row sums of squares
// W8 = false: the same workgroup over ROW-MAJOR bf16 weights (serving / rollout decode at 16 < M <=
// 64): each wave stages its 32 weight rows x 128 B per K-step with four 16-B LDS-DMAs per lane
// (swizzled like X), one 40-KiB slot per K-step, 4 slots = the whole 160 KiB (3 K-steps, 120 KiB,
// in flight). X is read from L2 N / 256 times — the 64-column ring (gemm_m64_kernel) reads it
// N / 64 times, as many bytes again as the weights at M = 64.
constexpr int WB_SLOTS = 4;
constexpr int WB_SLOT = 8192 + 32768;  // X (64 x 128 B) + 256 weight rows x 128 B

template <bool OUT_F32, bool W8 = true>
__global__ __launch_bounds__(512, 1) void gemm_w8_wide_kernel(GemmArgs p, float* __restrict__ slabs, int split) {
  constexpr int SLOTS = W8 ? WD_SLOTS : WB_SLOTS, SLOT = W8 ? WD_SLOT : WB_SLOT;
  constexpr int PER = W8 ? 3 : 5;  // LDS-DMAs per lane per K-step
  __shared__ __attribute__((aligned(16))) char smem[SLOTS * SLOT];  // the only __shared__ object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int cg = blockIdx.x / split, sp = blockIdx.x % split;
  const int nk = p.K / 64;
  const int t0 = (int)((long)sp * nk / split), t1 = (int)((long)(sp + 1) * nk / split);
  const int nt = t1 - t0;
  const bool pair = p.act == ACT_SWIGLU;
  const int F = p.N / 2;
  const int ngroups = p.N / 16;
  // image group of this wave's fragment j (0, 1)
  auto group_of = [&](int j) -> int {
    if (pair) return j == 0 ? 8 * cg + wid : F / 16 + 8 * cg + wid;
    return min(16 * cg + 2 * wid + j, ngroups - 1);
  };
  const long gstride = (long)(p.K / 128) * 2048;  // bytes per image group
  const char* wsrc0 = (const char*)p.B + (long)group_of(0) * gstride + lane * 16;
  const char* wsrc1 = (const char*)p.B + (long)group_of(1) * gstride + lane * 16;
  // bf16 row-major: instruction q stages local weight rows 32 wid + 16 (q >> 1) + 8 (q & 1) + lane / 8
  // (group group_of(q >> 1)), 16-B slot lane % 8 holding k-chunk slot ^ lds_swz(local row)
  const bf16_t* wrow[4];
  if constexpr (!W8) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 8 * (q & 1) + (lane >> 3);
      const int lr = 32 * wid + 16 * (q >> 1) + r;
      wrow[q] = p.B + (long)(group_of(q >> 1) * 16 + r) * p.ldb + ((lane & 7) ^ lds_swz(lr)) * 8;
    }
  }
  const int xr = wid * 8 + (lane >> 3);  // X row this lane stages
  const int xck = (lane & 7) ^ lds_swz(xr);
  const bf16_t* xsrc = p.A + (long)min(xr, p.M - 1) * p.lda + xck * 8;

  auto stage = [&](int t) {
    char* slot = smem + ((t - t0) % SLOTS) * SLOT;
    __builtin_amdgcn_global_load_lds((const void*)(xsrc + (long)t * 64), (lds_void*)(slot + wid * 1024), 16, 0, 0);
    if constexpr (W8) {
      const long woff = (long)(t >> 1) * 2048 + (t & 1) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)(wsrc0 + woff), (lds_void*)(slot + 8192 + (2 * wid) * 1024), 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void*)(wsrc1 + woff), (lds_void*)(slot + 8192 + (2 * wid + 1) * 1024), 16, 0, 2);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds((const void*)(wrow[q] + (long)t * 64),
                                         (lds_void*)(slot + 8192 + (32 * wid + 8 * q) * 128), 16, 0, 0);
    }
  };

  // SWAP: the weight fragment is the MFMA's A operand, so acc[rr][j][r] = C[X row 16 rr + frow]
  // [column 16 g_j + 4 fq + r]: every lane owns 4 CONSECUTIVE output columns of one row (16-B slab
  // stores / loads, 8-B bf16 stores), and a row's sum of squares is in the lanes of that row
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool normed = p.norm_eps > 0.f;
  float sq[4] = {0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < SLOTS - 1; ++i)
    if (i < nt) stage(t0 + i);
  for (int i = 0; i < nt; ++i) {
    // retire step i (PER LDS-DMAs per lane per step); the later staged steps stay in flight
    const int ahead = min(SLOTS - 2, nt - 1 - i);
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * PER) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (i + SLOTS - 1 < nt) stage(t0 + i + SLOTS - 1);  // the slot every wave finished reading
    const char* slot = smem + (i % SLOTS) * SLOT;
    bf16x8 b[2][2], a[4][2];
    if constexpr (W8) {
      rt_u32x2 w8[4];  // [j * 2 + kk]: row frow, k [32 kk + 8 fq, +8) of group 2 wid + j
      ds_read_b64_x4_512(lds_addr(slot + 8192 + (2 * wid) * 1024 + ((fq >> 1) * 16 + frow) * 16 + (fq & 1) * 8), w8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) b[j][kk] = fp8x8_to_bf16(w8[2 * j + kk][0], w8[2 * j + kk][1]);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int lr = 32 * wid + 16 * j + frow;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          b[j][kk] = *(const bf16x8*)(slot + 8192 + lr * 128 + (((kk * 4 + fq) ^ lds_swz(lr)) << 4));
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rr * 16 + frow;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + fq;
        a[rr][kk] = *(const bf16x8*)(slot + row * 128 + ((c ^ lds_swz(row)) << 4));
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[rr][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][kk], a[rr][kk], acc[rr][j], 0, 0, 0);
    if (normed) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)a[rr][kk][e];
            sq[rr] += f * f;
          }
    }
  }
  // row sums of squares: the 4 fq lanes of row 16 rr + frow each hold a quarter
  if (normed) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      sq[rr] += __shfl_xor(sq[rr], 16, 64);
      sq[rr] += __shfl_xor(sq[rr], 32, 64);
    }
  }
  const int lc = 32 * wid + 4 * fq;  // local column of fragment j: lc + 16 j
  if (split > 1) {
    // partial tile -> slab (plain 16-B stores); wide_reduce_kernel (the next launch) sums the
    // splits and runs the epilogue over every (row, 4 columns) in parallel — a last-arriver
    // reduction would stream split x 64 KiB through ONE workgroup
    float* slab = slabs + ((long)cg * split + sp) * WD_SLAB;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rr * 16 + frow;
      if (row < p.M) {
#pragma unroll
        for (int j = 0; j < 2; ++j) *(f32x4*)(slab + row * 256 + lc + 16 * j) = acc[rr][j];
      }
    }
    if (normed && wid == 0 && fq == 0) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        if (rr * 16 + frow < p.M) slab[64 * 256 + rr * 16 + frow] = sq[rr];
    }
    return;
  }
  // ---- epilogue from registers: row 16 rr + frow, 4 consecutive columns per fragment ----
  if (pair) {
    const int col = 16 * (8 * cg + wid) + 4 * fq;  // first of 4 F-columns
    const float4 one4 = make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 sg = W8 ? *(const float4*)(p.sb + col) : one4, su = W8 ? *(const float4*)(p.sb + F + col) : one4;
    const float sgv[4] = {sg.x, sg.y, sg.z, sg.w}, suv[4] = {su.x, su.y, su.z, su.w};
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rr * 16 + frow;
      if (row >= p.M) continue;
      const float rs = normed ? rsqrtf(sq[rr] / (float)p.K + p.norm_eps) : 1.f;
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gt = acc[rr][0][r] * rs * sgv[r], up = acc[rr][1][r] * rs * suv[r];
        if (p.bias) { gt += bf2f(p.bias[col + r]); up += bf2f(p.bias[F + col + r]); }
        y[r] = gt / (1.f + __expf(-gt)) * up;
      }
      if constexpr (OUT_F32) *(float4*)((float*)p.C + (long)row * p.ldc + col) = make_float4(y[0], y[1], y[2], y[3]);
      else *(uint2*)((bf16_t*)p.C + (long)row * p.ldc + col) = make_uint2(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]));
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 16 * (16 * cg + 2 * wid + j) + 4 * fq;
    if (col >= p.N) continue;
    const float4 sc4 = W8 ? *(const float4*)(p.sb + col) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float scv[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rr * 16 + frow;
      if (row >= p.M) continue;
      const float rs = normed ? rsqrtf(sq[rr] / (float)p.K + p.norm_eps) : 1.f;
      float res[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.R) {
        const uint2 rv = *(const uint2*)(p.R + (long)row * p.ldr + col);
        res[0] = bf2f((bf16_t)(rv.x & 0xffff)); res[1] = bf2f((bf16_t)(rv.x >> 16));
        res[2] = bf2f((bf16_t)(rv.y & 0xffff)); res[3] = bf2f((bf16_t)(rv.y >> 16));
      }
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[rr][j][r] * rs * scv[r];
        if (p.bias) v += bf2f(p.bias[col + r]);
        y[r] = apply_act(v, p.act) + res[r];
      }
      if constexpr (OUT_F32) *(float4*)((float*)p.C + (long)row * p.ldc + col) = make_float4(y[0], y[1], y[2], y[3]);
      else *(uint2*)((bf16_t*)p.C + (long)row * p.ldc + col) = make_uint2(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]));
    }
  }
}

// Split-K epilogue of the wide W8A16 kernel: one thread per (row, 4 output columns) sums the
// split partials (16-B loads), applies the in-GEMM RMS norm (row sums of squares from the slabs),
// per-column fp8 scales, bias, activation / SwiGLU pair, residual, and stores. Column c of the
// output lives in slab group c / 256 (SwiGLU: F-column c in group c / 128, gate at local column
// 32 w + (c % 16), up 16 further, w = (c % 128) / 16).
template <bool OUT_F32>
__global__ __launch_bounds__(256) void wide_reduce_kernel(GemmArgs p, const float* __restrict__ slabs, int split) {
  const bool pair = p.act == ACT_SWIGLU;
  const int F = p.N / 2;
  const int ncol4 = (pair ? F : p.N) / 4;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)p.M * ncol4) return;
  const int row = (int)(e / ncol4), col = (int)(e % ncol4) * 4;
  const int cg = pair ? col / 128 : col / 256;
  const int lcol = pair ? 32 * ((col % 128) / 16) + (col % 16) : col % 256;
  const float* base = slabs + (long)cg * split * WD_SLAB;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), u = g;
  float sq = 0.f;
  const bool normed = p.norm_eps > 0.f;
#pragma unroll 8
  for (int s2 = 0; s2 < split; ++s2) {
    const float* sl = base + (long)s2 * WD_SLAB;
    const float4 a = *(const float4*)(sl + row * 256 + lcol);
    g.x += a.x; g.y += a.y; g.z += a.z; g.w += a.w;
    if (pair) {
      const float4 b = *(const float4*)(sl + row * 256 + lcol + 16);
      u.x += b.x; u.y += b.y; u.z += b.z; u.w += b.w;
    }
    if (normed) sq += sl[64 * 256 + row];
  }
  const float rs = normed ? rsqrtf(sq / (float)p.K + p.norm_eps) : 1.f;
  const float gv[4] = {g.x, g.y, g.z, g.w}, uv[4] = {u.x, u.y, u.z, u.w};
  float y[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (pair) {
      float gt = gv[r] * rs * (p.sb ? p.sb[col + r] : 1.f), up = uv[r] * rs * (p.sb ? p.sb[F + col + r] : 1.f);
      if (p.bias) { gt += bf2f(p.bias[col + r]); up += bf2f(p.bias[F + col + r]); }
      y[r] = gt / (1.f + __expf(-gt)) * up;
    } else {
      float v = gv[r] * rs * (p.sb ? p.sb[col + r] : 1.f);
      if (p.bias) v += bf2f(p.bias[col + r]);
      y[r] = apply_act(v, p.act);
      if (p.R) y[r] += bf2f(p.R[(long)row * p.ldr + col + r]);
    }
  }
  if constexpr (OUT_F32) *(float4*)((float*)p.C + (long)row * p.ldc + col) = make_float4(y[0], y[1], y[2], y[3]);
  else *(uint2*)((bf16_t*)p.C + (long)row * p.ldc + col) = make_uint2(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]));
}

// split-K of the wide W8A16 kernel (one workgroup per CU, 4 K-steps in flight each): the largest
// power of two that keeps the grid <= 256 workgroups with >= 8 K-steps each (the partials go
// through one parallel reduce launch). From the cold-weight sweep (profiles/r3/fp8_decode_table_*,
// M = 24 .. 64): gate_up 108-112 groups -> 2, qkv 24 / 60 groups -> 8 / 4, o 16-20 -> 8, down
// (K 13824 / 14336) 16 / 20 groups -> 16 / 8.
static int wide_split(int N, int K) {
  if (tuning().wide_split > 0) return tuning().wide_split;
  const int groups = N / 256, nk = K / 64;
  int split = 1;
  while (groups * split * 2 <= 256 && nk / (split * 2) >= 8 && split < 16) split *= 2;
  return split;
}

// split-K for the ring kernel, from a cold-weight sweep on MI355X (profiles/kernels_m64_split.log,
// M = 64): wide outputs (>= 256 column groups) stream best unsplit, long K / narrow N want 8-way
// split, mid shapes 2-way.

static int m64_split(int N, int K) {
  if (tuning().m64_split > 0) return tuning().m64_split;
  const int groups = (N + 63) / 64, nk = K / 64;
  int split;
  if (groups >= 256) split = 1;
  else if (nk >= 128 || groups <= 64) split = 8;
  else split = 2;
  while (split > 1 && nk / split < 4) split >>= 1;
  return split;
}

// split-K of the M <= 16 kernel, from a hipGraph-replayed sweep over distinct (cold) weights
// (tools/sweep_decode.py, profiles/kernels_decode_split_sweep.log): wide outputs (>= 256 column
// groups: gate_up, lm_head) stream best unsplit — a second round of workgroups costs more than it
// hides; narrower ones split until ~2 workgroups per CU are resident, keeping >= 2 k-chunks per wave
// (M = 1: qkv 16.5 -> 13.7 us, o 11.8 -> 10.9, down 29.4 -> 28.4 at split 8 vs 4).

// Tile-ordered (shuffled) weights stream best with ~8 blocks per column group at every width
// (gate_up 52.0 -> 43.2 us, lm_head 52.2 -> 47.7 at split 8 vs unsplit row-major; qkv / o / down
// as the row-major heuristic), keeping >= 2 k-chunks per wave (profiles/kernels_decode_depth_shuffle.log).
static int decode_split_shuf(int K) {
  if (tuning().decode_split > 0) return tuning().decode_split;
  const int nc = K / 64;
  int split = 8;
  while (split > 1 && nc / (4 * split) < 2) split >>= 1;
  return split;
}

static int decode_split(int N, int K) {
  if (tuning().decode_split > 0) return tuning().decode_split;
  const int groups = (N + DG_COLS - 1) / DG_COLS;
  const int nc = K / 64;
  if (groups >= 256) return 1;
  int split = 1;
  while (groups * split < 512 && nc / (4 * split * 2) >= 2 && split < 16) split *= 2;
  return split;
}

}  // namespace rt

using namespace rt;

// never let a split-K launch write past the workspace (slabs: groups x split x slab floats;
// tickets: one per column group)
static int fit_split(int split, int groups, long slab_floats) {
  if (groups > RT_SPLITK_TICKETS) return 1;
  while (split > 1 && (long)groups * split * slab_floats > RT_SPLITK_SLAB_FLOATS) split >>= 1;
  return split;
}


// register sets of the M <= 16 kernel's weight pipeline (DEPTH - 1 k-chunks in flight per wave).
// 4 sets cost ~85 VGPRs at MT = 1 (occupancy 3 -> 2 blocks per CU; MT = 2 would spill) and
// measured no faster even on the unsplit wide GEMMs (gate_up 48.9 vs 48.7 us, lm_head 52.8 vs
// 52.6; profiles/kernels_decode_depth_shuffle.log): the default stays 2. 2 / 4 force (tuning).
// batch-1 GEMVs on the 16-row no-split kernel: narrow outputs (qkv, o, down) whose split-K tail
// costs more than a second round of workgroups; tuning gemv16 = 0 keeps them on gemm_decode_kernel
// tuning gemv16: 0 off, 1 narrow outputs only (N <= 8192: qkv, o, down), 2 also wide ones (SwiGLU
// gate_up, lm_head)
// rows of X on the no-split kernel (1..16; tuning gemv16_maxm)
static int gemv16_max_m() {
  const int m = tuning().gemv16_maxm;
  return m < 1 ? 1 : (m > 16 ? 16 : m);
}
static bool use_gemv16(int N, int K, int act) {
  const int env = tuning().gemv16;
  if (!env || K % 64 || K < 1024) return false;
  if (act == ACT_SWIGLU) return env >= 2 && N % 32 == 0 && N / 32 >= 256;
  return N % 16 == 0 && N / 16 >= 256 && (N <= 8192 || env >= 2);
}

static int decode_depth(int MT, long blocks) {
  if (MT > 1) return 2;
  const int dd = tuning().decode_depth;
  if (dd == 2 || dd == 4) return dd;
  (void)blocks;
  return 2;
}


extern "C" int rt_gemm_nt(const void* A, long lda, const void* B, long ldb, const void* U, long ldu,
                          const void* UB, long ldub, int Rp, const void* bias, void* C, long ldc, int M,
                          int N, int K, int act, int out_f32, float* slabs, unsigned* tickets,
                          const void* R, long ldr, float norm_eps, int wshuf, hipStream_t stream) {
  GemmArgs p;
  p.A = (const bf16_t*)A; p.lda = lda;
  p.B = (const bf16_t*)B; p.ldb = ldb;
  p.U = (const bf16_t*)U; p.ldu = ldu;
  p.UB = (const bf16_t*)UB; p.ldub = ldub;
  p.Rp = (U && UB) ? Rp : 0;
  p.bias = (const bf16_t*)bias;
  p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = act;
  p.sa = nullptr; p.sb = nullptr;
  p.R = (const bf16_t*)R; p.ldr = ldr; p.norm_eps = norm_eps; p.wshuf = wshuf;
  if (M <= 0 || N <= 0) return 0;
  if (wshuf && (M > 64 || N % 16 != 0 || K % 64 != 0)) return -4;  // shuffled weights: decode kernel only
  if (act == ACT_SWIGLU && (M > 64 || N % 64 != 0 || (U && UB))) return -2;
  if (M > 64) return -5;  // token-parallel GEMMs: rt_gemm_big
  if (M > 16 && M <= 64 && p.Rp == 0 && !wshuf && tuning().m64_wide && act != ACT_SWIGLU && N % 256 == 0 &&
      N <= 16384 && K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 && (!R || ldr % 4 == 0)) {
    // 256 weight rows per workgroup over the row-major weights (X from L2 N / 256 times). Cold-weight
    // probe at M = 24..64 (profiles/r6/m64_wide_probe.log): qkv 24 -> 17-19 us, o 18-19 -> 13-15,
    // down 32-37 -> 28-31 vs the 64-column ring. Wide outputs (>= 64 groups: split 2 + a reduce) stay
    // on the ring: SwiGLU gate / up 51-54 vs 58-65 us, the LM head (N 32000) 58-60 vs 77-80 us
    int split = slabs ? fit_split(wide_split(N, K), N / 256, WD_SLAB) : 1;
    split = std::min(split, std::max(1, K / 64));
    dim3 grid((N / 256) * split), block(512);
    if (out_f32) hipLaunchKernelGGL((gemm_w8_wide_kernel<true, false>), grid, block, 0, stream, p, slabs, split);
    else hipLaunchKernelGGL((gemm_w8_wide_kernel<false, false>), grid, block, 0, stream, p, slabs, split);
    if (split > 1) {
      const long work = (long)M * (act == ACT_SWIGLU ? N / 2 : N) / 4;
      if (out_f32) hipLaunchKernelGGL((wide_reduce_kernel<true>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream,
                                      p, slabs, split);
      else hipLaunchKernelGGL((wide_reduce_kernel<false>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream,
                              p, slabs, split);
    }
  } else if (M > 16 && M <= 64 && p.Rp == 0 && !wshuf) {
    const int split = (slabs && tickets) ? fit_split(m64_split(N, K), (N + 63) / 64, 64 * 64 + 64) : 1;
    dim3 grid(((N + 63) / 64) * split), block(256);
    if (out_f32) hipLaunchKernelGGL((gemm_m64_kernel<true>), grid, block, 0, stream, p, slabs, tickets, split);
    else hipLaunchKernelGGL((gemm_m64_kernel<false>), grid, block, 0, stream, p, slabs, tickets, split);
  } else if (M <= gemv16_max_m() && wshuf && tuning().decode_split == 0 && use_gemv16(N, K, act) && p.Rp == 0) {
    const bool pair = act == ACT_SWIGLU;
    dim3 grid(pair ? N / 32 : N / 16), block(256);
    const int gd = tuning().gemv16_depth;
#define G16(D, P) if (out_f32) hipLaunchKernelGGL((gemv16_kernel<true, D, P>), grid, block, 0, stream, p); \
                  else hipLaunchKernelGGL((gemv16_kernel<false, D, P>), grid, block, 0, stream, p);
    // waves per row group: 0 = auto — 8 when the grid has at most one workgroup per CU (o / down:
    // N / 16 = 256), so each CU keeps twice the weight bytes in flight; 4 on wider grids (qkv 384,
    // lm_head 2000 workgroups), where 8 measured the same or slower. Batch-1 p50 0.383 -> 0.376 s
    // (profiles/r4/gemv16_waves_ab.log)
    int nw = tuning().gemv16_waves;
    if (nw == 0) nw = (int)grid.x <= gemv_cus() ? 8 : 4;
    if (pair) { G16(4, true) } else if (gd == 6) { G16(6, false) } else if (gd == 8) { G16(8, false) }
    else if (nw == 8) {
      if (out_f32) hipLaunchKernelGGL((gemv16_kernel<true, 4, false, false, 8>), grid, dim3(512), 0, stream, p);
      else hipLaunchKernelGGL((gemv16_kernel<false, 4, false, false, 8>), grid, dim3(512), 0, stream, p);
    } else if (nw == 16) {
      if (out_f32) hipLaunchKernelGGL((gemv16_kernel<true, 4, false, false, 16>), grid, dim3(1024), 0, stream, p);
      else hipLaunchKernelGGL((gemv16_kernel<false, 4, false, false, 16>), grid, dim3(1024), 0, stream, p);
    } else { G16(4, false) }
#undef G16
  } else {
    const int MT = (M + 15) / 16;
    const int want = wshuf ? decode_split_shuf(K) : decode_split(N, K);
    const int split = (slabs && tickets) ? fit_split(want, (N + DG_COLS - 1) / DG_COLS, MT * 16 * (DG_COLS + 1)) : 1;
    dim3 grid(((N + DG_COLS - 1) / DG_COLS) * split), block(256);
    const bool deep = decode_depth(MT, (long)grid.x) == 4;
#define DG_CASE(mt, d)                                                                                     \
  if (out_f32) hipLaunchKernelGGL((gemm_decode_kernel<mt, true, false, d>), grid, block, 0, stream, p, slabs, tickets, split); \
  else hipLaunchKernelGGL((gemm_decode_kernel<mt, false, false, d>), grid, block, 0, stream, p, slabs, tickets, split);
    switch (MT) {
      case 1: if (deep) { DG_CASE(1, 4) } else { DG_CASE(1, 2) } break;
      case 2: DG_CASE(2, 2) break;
      case 3: DG_CASE(3, 2) break;
      case 4: DG_CASE(4, 2) break;
      default: return -1;
    }
#undef DG_CASE
  }
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_gemm_big_fp8(const void*, long, const float*, const void*, long, const float*, const void*, void*,
                               long, int, int, int, int, const void*, long, const void*, long, int, void*, long,
                               const void*, hipStream_t);

// fp8 GEMMs: C[M,N] (bf16) = act( (A_q B_q^T) * sa[row] * sb[col] + bias ), A_q / B_q OCP e4m3fn.
//  * M > 64 : W8A8 on the gemm_big schedule, MX-scaled mfma_16x16x128_f8f6f4 (2x the bf16 rate)
//  * M <= 64: W8A16 (A = bf16 activations, sa ignored): half the weight bytes.
//      - M <= 16 with the tile-ordered fp8 image (wshuf, shuffle_decode_weight_fp8): gemv16_kernel<W8>,
//        one workgroup per 16 weight rows, no split-K;
//      - 16 < M <= 64 with the image: the LDS-DMA ring gemm_m64_kernel<W8> (split-K slabs);
//      - row-major fp8 weights (no image: small / odd shapes): the split-K register-streaming kernel.
extern "C" int rt_gemm_fp8(const void* A, long lda, const float* sa, const void* B, long ldb, const float* sb,
                           const void* bias, void* C, long ldc, int M, int N, int K, int act, int a_is_bf16,
                           float* slabs, unsigned* tickets, const void* R, long ldr, float norm_eps, int wshuf,
                           hipStream_t stream) {
  GemmArgs p;
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.U = nullptr; p.ldu = 0; p.UB = nullptr; p.ldub = 0; p.Rp = 0;
  p.bias = (const bf16_t*)bias; p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K; p.act = act;
  p.sa = sa; p.sb = sb;
  p.R = (const bf16_t*)R; p.ldr = ldr; p.norm_eps = norm_eps; p.wshuf = 0;
  if (M <= 0 || N <= 0) return 0;
  if ((R || norm_eps > 0.f) && !a_is_bf16) return -3;
  if (a_is_bf16) {
    if (M > 64 || K % 64) return -1;
    const bool pair = act == ACT_SWIGLU;
    if (wshuf) {
      // tile-ordered fp8 image: the no-split 16-row kernel up to 16 rows (or RT variant 4), the
      // LDS-DMA ring above
      if (K % 128 || N % 16 || (pair && N % 64)) return -4;
      if (M <= 16 && tuning().gemm_variant != 4) {
        dim3 grid(pair ? N / 32 : N / 16), block(256);
        if (pair) hipLaunchKernelGGL((gemv16_kernel<false, 4, true, true>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((gemv16_kernel<false, 4, false, true>), grid, block, 0, stream, p);
      } else if (N % 256 == 0 && tuning().gemm_variant != 5) {
        // 256 weight rows per workgroup (X read N / 256 times); RT variant 5 = the 64-column ring
        int split = slabs ? fit_split(wide_split(N, K), N / 256, WD_SLAB) : 1;
        split = std::min(split, std::max(1, K / 64));
        dim3 grid((N / 256) * split), block(512);
        hipLaunchKernelGGL((gemm_w8_wide_kernel<false>), grid, block, 0, stream, p, slabs, split);
        if (split > 1) {
          const long work = (long)M * (pair ? N / 2 : N) / 4;
          hipLaunchKernelGGL((wide_reduce_kernel<false>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, p,
                             slabs, split);
        }
      } else {
        const int split = (slabs && tickets) ? fit_split(m64_split(N, K), (N + 63) / 64, 64 * 64 + 64) : 1;
        dim3 grid(((N + 63) / 64) * split), block(256);
        hipLaunchKernelGGL((gemm_m64_kernel<false, true>), grid, block, 0, stream, p, slabs, tickets, split);
      }
    } else {
      const int MT = (M + 15) / 16;
      const int split = (slabs && tickets) ? fit_split(decode_split(N, K), (N + DG_COLS - 1) / DG_COLS, MT * 16 * (DG_COLS + 1)) : 1;
      dim3 grid(((N + DG_COLS - 1) / DG_COLS) * split), block(256);
      switch (MT) {
        case 1:
          if (decode_depth(1, (long)grid.x) == 4) hipLaunchKernelGGL((gemm_decode_kernel<1, false, true, 4>), grid, block, 0, stream, p, slabs, tickets, split);
          else hipLaunchKernelGGL((gemm_decode_kernel<1, false, true, 2>), grid, block, 0, stream, p, slabs, tickets, split);
          break;
        case 2: hipLaunchKernelGGL((gemm_decode_kernel<2, false, true, 2>), grid, block, 0, stream, p, slabs, tickets, split); break;
        case 3: hipLaunchKernelGGL((gemm_decode_kernel<3, false, true, 2>), grid, block, 0, stream, p, slabs, tickets, split); break;
        case 4: hipLaunchKernelGGL((gemm_decode_kernel<4, false, true, 2>), grid, block, 0, stream, p, slabs, tickets, split); break;
        default: return -1;
      }
    }
  } else {
    // W8A8 (M > 64): the gemm_big schedule with the MX fp8 MFMA; SwiGLU pairs [gate; up] in its
    // epilogue
    if (K % 128 || N % 8 || lda % 16 || ldb % 16 || ldc % 8) return -1;
    if (act != 0 && !(act == ACT_SWIGLU && N % 256 == 0)) return -2;
    return rt_gemm_big_fp8(A, lda, sa, B, ldb, sb, bias, C, ldc, M, N, K, act == ACT_SWIGLU ? 5 : 0, nullptr, 0,
                           nullptr, 0, 0, nullptr, 0, nullptr, stream);
  }
  RT_LAUNCH_CHECK();
  return 0;
}

// Decode-weight image for the M <= 64 kernel: W [N, K] row-major -> per (16-row group G, 64-k chunk
// c) one 2-KiB tile in the order the kernel's lanes load it (lane l = 16 g + r of load h reads
// W[16 G + r][64 c + 32 h + 8 g .. +8]), tiles of one row group consecutive in c. Every 16-B load
// instruction of a wave then reads one contiguous 1-KiB run (tools/microbench/hbm_pattern.hip:
// 6.3-6.7 TB/s vs 5.9 for the row-major 16-rows x 128-B pattern). Measured at M = 1 (graph replay,
// cold weights, profiles/kernels_decode_depth_shuffle.log): the split-K launches gain (qkv 14.2 ->
// 12.8 us, o 11.0 -> 10.3, down 28.5 -> 21.9), the unsplit wide ones do not (gate_up 52.7 -> 51.3,
// lm_head 49.7 -> 56.9; rotating each block's k walk made both worse) until they are split 8 ways
// too (decode_split_shuf: gate_up 43.2, lm_head 47.7). At the same split the results are bitwise
// identical to the row-major launch. One thread per 16 B.
__global__ __launch_bounds__(256) void shuffle_decode_weight_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                                     long N, long K) {
  const long nc = K / 64;
  const long total = N * K / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long l = i & 63, h = (i >> 6) & 1, tile = i >> 7;
    const long G = tile / nc, c = tile % nc;
    const long row = G * 16 + (l & 15), k = c * 64 + h * 32 + (l >> 4) * 8;
    dst[i] = src[(row * K + k) / 8];
  }
}

extern "C" int rt_shuffle_decode_weight(const void* src, void* dst, long N, long K, hipStream_t stream) {
  if (N % 16 || K % 64) return -1;
  const long total = N * K / 8;
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(shuffle_decode_weight_kernel, dim3(blocks), dim3(256), 0, stream, (const uint4*)src, (uint4*)dst, N, K);
  RT_LAUNCH_CHECK();
  return 0;
}

// fp8 decode-weight image for gemv16_kernel<W8>: q [N, K] e4m3fn bytes row-major -> per (16-row
// group G, 128-k chunk c) one 2-KiB tile; 16-B unit i of a tile: lane l = i & 63 of load h =
// (i >> 6) & 1 holds row 16 G + (l & 15), k [128 c + 64 h + 16 (l >> 4), +16). Every load
// instruction of a wave then reads one contiguous 1-KiB run. One thread per 16 B.
__global__ __launch_bounds__(256) void shuffle_decode_weight_fp8_kernel(const uint4* __restrict__ src,
                                                                        uint4* __restrict__ dst, long N, long K) {
  const long nc = K / 128;
  const long total = N * K / 16;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long l = i & 63, h = (i >> 6) & 1, tile = i >> 7;
    const long G = tile / nc, c = tile % nc;
    const long row = G * 16 + (l & 15), k = c * 128 + h * 64 + (l >> 4) * 16;
    dst[i] = src[(row * K + k) / 16];
  }
}

extern "C" int rt_shuffle_decode_weight_fp8(const void* src, void* dst, long N, long K, hipStream_t stream) {
  if (N % 16 || K % 128) return -1;
  const long total = N * K / 16;
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(shuffle_decode_weight_fp8_kernel, dim3(blocks), dim3(256), 0, stream, (const uint4*)src,
                     (uint4*)dst, N, K);
  RT_LAUNCH_CHECK();
  return 0;
}
