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
// Two kernels:
//  * gemm_tile_kernel  — M > 64: 128x128x64 block tile, 4 waves (2x2, 64x64 each, 4x4
//    mfma_f32_16x16x32_bf16 accumulators), global_load_lds (16 B/lane) into an XOR-swizzled
//    lane-linear LDS image (source-address swizzle, cdna_hip_programming.md rule 21), two LDS
//    stages, XCD-aware bijective block remap + grouped tile order, LDS-staged coalesced epilogue.
//  * gemm_skinny_kernel — M <= 64 (decode / small batch): weight streaming. One block = 16 output
//    columns x all M rows; its 4 waves split K and stream W straight to VGPRs with a deep
//    unrolled prefetch (LDS would be pure overhead: W is read once, cdna_hip_programming.md §5,
//    'GEMV / M <= 16 decode weights'), cross-wave reduction through LDS.
//
// Replaces every projection GEMM of the reference's HF forward passes (reference
// call sites reinforcement_learning_optimization_after_rag.py:38,200,207,313,318).
#include "rt_common.h"

namespace rt {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_TANH = 3, ACT_SILU = 4 };

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
};

typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------------------------------------
// Large-M tile kernel
// ---------------------------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int STAGE_BYTES = (TBM + TBN) * TBK * 2;  // 32 KiB per stage (A + B)
constexpr int GROUP_M = 8;

template <bool OUT_F32>
__global__ __launch_bounds__(256, 2) void gemm_tile_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_m = (p.M + TBM - 1) / TBM, tiles_n = (p.N + TBN - 1) / TBN;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % gsz);
  const int tn = (bid % (GROUP_M * tiles_n)) / gsz;
  const int m0 = tm * TBM, n0 = tn * TBN;

  const int nk_main = p.K / TBK;
  const int nk = nk_main + p.Rp / TBK;

  // Per-lane staging source rows (4 A chunks + 4 B chunks per wave, 8 rows x 128 B each).
  // LDS image is lane-linear: lane l of chunk c lands at row 8c + (l>>3), 16-B slot (l&7).
  // It must hold k-chunk slot ^ (row&7)  ->  source k-chunk = (l&7) ^ (l>>3).
  const int r_in_chunk = lane >> 3;
  const int src_kc = (lane & 7) ^ r_in_chunk;
  long a_row_off[4], b_row_off[4], u_row_off[4], ub_row_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + r_in_chunk;
    const int ga = min(m0 + row, p.M - 1);
    const int gb = min(n0 + row, p.N - 1);
    a_row_off[i] = (long)ga * p.lda + src_kc * 8;
    b_row_off[i] = (long)gb * p.ldb + src_kc * 8;
    u_row_off[i] = (long)ga * p.ldu + src_kc * 8;
    ub_row_off[i] = (long)gb * p.ldub + src_kc * 8;
  }

  auto stage = [&](int t, int buf) {
    char* sA = smem + buf * STAGE_BYTES;
    char* sB = sA + TBM * TBK * 2;
    const bf16_t *pa, *pb;
    long ka;
    if (t < nk_main) {
      ka = (long)t * TBK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pa = p.A + a_row_off[i] + ka;
        pb = p.B + b_row_off[i] + ka;
        __builtin_amdgcn_global_load_lds((const void*)pa, (lds_void*)(sA + (wid * 4 + i) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)pb, (lds_void*)(sB + (wid * 4 + i) * 1024), 16, 0, 0);
      }
    } else {
      ka = (long)(t - nk_main) * TBK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pa = p.U + u_row_off[i] + ka;
        pb = p.UB + ub_row_off[i] + ka;
        __builtin_amdgcn_global_load_lds((const void*)pa, (lds_void*)(sA + (wid * 4 + i) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)pb, (lds_void*)(sB + (wid * 4 + i) * 1024), 16, 0, 0);
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wr = wid >> 1, wc = wid & 1;
  const int frow = lane & 15, fk = lane >> 4;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage(t + 1, cur ^ 1);
    const char* sA = smem + cur * STAGE_BYTES;
    const char* sB = sA + TBM * TBK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
      const int kc = kk * 4 + fk;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr * 64 + i * 16 + frow;
        af[i] = *(const bf16x8*)(sA + row * 128 + ((kc ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wc * 64 + j * 16 + frow;
        bfr[j] = *(const bf16x8*)(sB + row * 128 + ((kc ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: bias + activation, then store ----
  float bcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wc * 64 + j * 16 + frow;
    bcol[j] = (p.bias && col < p.N) ? bf2f(p.bias[col]) : 0.f;
  }

  if constexpr (OUT_F32) {
    float* C = (float*)p.C;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + frow;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * 64 + i * 16 + fk * 4 + r;
          if (row < p.M && col < p.N) C[(long)row * p.ldc + col] = apply_act(acc[i][j][r] + bcol[j], p.act);
        }
      }
  } else {
    // Stage the bf16 tile through LDS (row stride 136 elems = 272 B) for 16-B coalesced stores.
    bf16_t* tile = (bf16_t*)smem;
    constexpr int LDT = TBN + 8;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc * 64 + j * 16 + frow;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 64 + i * 16 + fk * 4 + r;
          tile[row * LDT + col] = f2bf(apply_act(acc[i][j][r] + bcol[j], p.act));
        }
      }
    __syncthreads();
    bf16_t* C = (bf16_t*)p.C;
    const int cc = tid & 15;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      const int row = pass * 16 + (tid >> 4);
      const int grow = m0 + row, gcol = n0 + cc * 8;
      if (grow < p.M && gcol < p.N) {
        const uint4 v = *(const uint4*)(tile + row * LDT + cc * 8);
        *(uint4*)(C + (long)grow * p.ldc + gcol) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Skinny (M <= 64) weight-streaming kernel
// ---------------------------------------------------------------------------------------------
// Each wave: 16 output columns (one MFMA B fragment), all MT*16 rows, a contiguous range of
// 64-deep K chunks. Per 64-chunk, lane group g = lane>>4 owns k in [16g, 16g+16) (k-slot
// permutation: MFMA step s uses k = 16g + 8s + j, identical for A and B, so the sum is exact) so
// each W row is read as 4 lanes x 32 contiguous bytes = one full 128-B line per k-chunk.
constexpr int SK_PREF = 4;  // 64-chunks in flight per wave

template <int MT, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmArgs p) {
  __shared__ float red[4][MT * 16][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int frow = lane & 15, g = lane >> 4;

  const int nc_main = p.K / 64;
  const int c_begin = (wid * nc_main) / 4, c_end = ((wid + 1) * nc_main) / 4;

  const int wn = min(n0 + frow, p.N - 1);
  const bf16_t* wrow = p.B + (long)wn * p.ldb + g * 16;
  const bf16_t* xrow[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) xrow[m] = p.A + (long)min(m * 16 + frow, p.M - 1) * p.lda + g * 16;

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // software pipeline: W for SK_PREF chunks ahead in registers
  uint4 wbuf[SK_PREF][2];
#pragma unroll
  for (int s = 0; s < SK_PREF; ++s) {
    const int c = c_begin + s;
    if (c < c_end) {
      wbuf[s][0] = *(const uint4*)(wrow + (long)c * 64);
      wbuf[s][1] = *(const uint4*)(wrow + (long)c * 64 + 8);
    }
  }
  for (int c0 = c_begin; c0 < c_end; c0 += SK_PREF) {
#pragma unroll
    for (int s = 0; s < SK_PREF; ++s) {
      const int c = c0 + s;
      if (c < c_end) {
        const uint4 w0 = wbuf[s][0], w1 = wbuf[s][1];
        const int cn = c + SK_PREF;
        if (cn < c_end) {
          wbuf[s][0] = *(const uint4*)(wrow + (long)cn * 64);
          wbuf[s][1] = *(const uint4*)(wrow + (long)cn * 64 + 8);
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const uint4 x0 = *(const uint4*)(xrow[m] + (long)c * 64);
          const uint4 x1 = *(const uint4*)(xrow[m] + (long)c * 64 + 8);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0),
                                                           __builtin_bit_cast(bf16x8, w0), acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1),
                                                           __builtin_bit_cast(bf16x8, w1), acc[m], 0, 0, 0);
        }
      }
    }
  }
  // LoRA extension chunks: handled by wave 3 (its main range is last to start, roughly balanced)
  if (p.Rp > 0 && wid == 3) {
    const bf16_t* ubrow = p.UB + (long)wn * p.ldub + g * 16;
    for (int c = 0; c < p.Rp / 64; ++c) {
      const uint4 w0 = *(const uint4*)(ubrow + c * 64);
      const uint4 w1 = *(const uint4*)(ubrow + c * 64 + 8);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf16_t* urow = p.U + (long)min(m * 16 + frow, p.M - 1) * p.ldu + g * 16;
        const uint4 x0 = *(const uint4*)(urow + c * 64);
        const uint4 x1 = *(const uint4*)(urow + c * 64 + 8);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x0),
                                                         __builtin_bit_cast(bf16x8, w0), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x1),
                                                         __builtin_bit_cast(bf16x8, w1), acc[m], 0, 0, 0);
      }
    }
  }
  // acc[m] lane holds C[row = m*16 + 4g + r][col = frow]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][m * 16 + g * 4 + r][frow] = acc[m][r];
  __syncthreads();
  for (int e = tid; e < MT * 16 * 16; e += 256) {
    const int row = e >> 4, col = e & 15;
    const int grow = row, gcol = n0 + col;
    if (grow < p.M && gcol < p.N) {
      float v = red[0][row][col] + red[1][row][col] + red[2][row][col] + red[3][row][col];
      if (p.bias) v += bf2f(p.bias[gcol]);
      v = apply_act(v, p.act);
      if constexpr (OUT_F32) ((float*)p.C)[(long)grow * p.ldc + gcol] = v;
      else ((bf16_t*)p.C)[(long)grow * p.ldc + gcol] = f2bf(v);
    }
  }
}

}  // namespace rt

using namespace rt;

extern "C" int rt_gemm_nt(const void* A, long lda, const void* B, long ldb, const void* U, long ldu,
                          const void* UB, long ldub, int Rp, const void* bias, void* C, long ldc, int M,
                          int N, int K, int act, int out_f32, hipStream_t stream) {
  GemmArgs p;
  p.A = (const bf16_t*)A; p.lda = lda;
  p.B = (const bf16_t*)B; p.ldb = ldb;
  p.U = (const bf16_t*)U; p.ldu = ldu;
  p.UB = (const bf16_t*)UB; p.ldub = ldub;
  p.Rp = (U && UB) ? Rp : 0;
  p.bias = (const bf16_t*)bias;
  p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = act;
  if (M <= 0 || N <= 0) return 0;
  if (M <= 64) {
    const int MT = (M + 15) / 16;
    dim3 grid((N + 15) / 16), block(256);
#define SK_CASE(mt)                                                                              \
  case mt:                                                                                       \
    if (out_f32) hipLaunchKernelGGL((gemm_skinny_kernel<mt, true>), grid, block, 0, stream, p);  \
    else hipLaunchKernelGGL((gemm_skinny_kernel<mt, false>), grid, block, 0, stream, p);         \
    break;
    switch (MT) { SK_CASE(1) SK_CASE(2) SK_CASE(3) SK_CASE(4) default: return -1; }
#undef SK_CASE
  } else {
    const int tiles = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
    dim3 grid(tiles), block(256);
    if (out_f32) hipLaunchKernelGGL((gemm_tile_kernel<true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((gemm_tile_kernel<false>), grid, block, 0, stream, p);
  }
  RT_LAUNCH_CHECK();
  return 0;
}
