// On-device token sampler: temperature, top-k, top-p (nucleus), greedy, and the
// log-prob of the drawn token under the full tempered distribution (PPO's behaviour log-prob, so
// rollout needs no separate "old log-prob" forward). One workgroup per row.
//
//  * top-k threshold: exact 4-pass 8-bit radix select of the k-th largest logit (ties kept, as the
//    reference's HF TopK warper keeps every logit >= the k-th value).
//  * top-p threshold: the same radix walk but histogramming probability MASS: the smallest set of
//    highest-probability tokens whose mass reaches p (ties at the threshold kept).
//  * draw: Gumbel-max over the kept set with a counter-based Philox stream keyed by
//    (seed, row, offset + token id); `offset` is read from device memory so a hipGraph-captured
//    decode step stays random across replays (the decode epilogue kernel advances it).
// Reference behaviour being replaced: HF generate(do_sample=True, temperature=0.7)
// (reinforcement_learning_optimization_after_rag.py:38-44).
#include "rt_common.h"

namespace rt {

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }

template <typename T>
__global__ __launch_bounds__(256) void sample_kernel(const T* __restrict__ logits, long ld, int V, float inv_temp,
                                                     int top_k, float top_p, int greedy, uint64_t seed,
                                                     const int64_t* __restrict__ offset_ptr,
                                                     const uint8_t* __restrict__ row_active, long* __restrict__ out_tok,
                                                     float* __restrict__ out_logp) {
  __shared__ float hist_f[256];
  __shared__ unsigned hist_c[256];
  __shared__ float redf[8];
  __shared__ int redi[8];
  __shared__ uint32_t sh_key;
  __shared__ float sh_f;

  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // pass 1: max of tempered logits (and argmax for greedy)
  float mx = -INFINITY;
  int amx = 0;
  for (int i = tid; i < V; i += 256) {
    const float f = ld1<T>(x + i) * inv_temp;
    if (f > mx) { mx = f; amx = i; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(mx, off, 64);
    const int oi = __shfl_xor(amx, off, 64);
    if (om > mx || (om == mx && oi < amx)) { mx = om; amx = oi; }
  }
  if (lane == 0) { redf[wid] = mx; redi[wid] = amx; }
  __syncthreads();
  float M = redf[0];
  int AM = redi[0];
  for (int w = 1; w < 4; ++w)
    if (redf[w] > M || (redf[w] == M && redi[w] < AM)) { M = redf[w]; AM = redi[w]; }
  __syncthreads();
  // pass 2: sum of exp
  float s = 0.f;
  for (int i = tid; i < V; i += 256) s += __expf(ld1<T>(x + i) * inv_temp - M);
  const float S = block_sum(s, redf);
  const float lse = M + __logf(S);

  int tok = AM;
  const bool active = row_active ? row_active[row] != 0 : true;
  if (!greedy && active) {
    // ---- top-k threshold (key space of raw logits; order == tempered order for inv_temp > 0) ----
    uint32_t kth = 0;  // keep key >= kth
    if (top_k > 0 && top_k < V) {
      uint32_t prefix = 0, mask = 0;
      unsigned remaining = top_k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        hist_c[tid] = 0;
        __syncthreads();
        for (int i = tid; i < V; i += 256) {
          const uint32_t k = fkey(ld1<T>(x + i));
          if ((k & mask) == prefix) atomicAdd(&hist_c[(k >> shift) & 255], 1u);
        }
        __syncthreads();
        if (tid == 0) {
          unsigned cum = 0;
          int bsel = 0;
          for (int bb = 255; bb >= 0; --bb) {
            if (cum + hist_c[bb] >= remaining) { bsel = bb; break; }
            cum += hist_c[bb];
          }
          remaining -= cum;
          sh_key = bsel;
        }
        __syncthreads();
        prefix |= sh_key << shift;
        mask |= 255u << shift;
        __syncthreads();
      }
      kth = prefix;
    }
    // ---- top-p threshold by probability mass among the top-k survivors ----
    uint32_t pth = kth;
    if (top_p < 1.f) {
      float sk = 0.f;
      for (int i = tid; i < V; i += 256) {
        const float f = ld1<T>(x + i);
        if (fkey(f) >= kth) sk += __expf(f * inv_temp - M);
      }
      const float Sk = block_sum(sk, redf);
      const float target = top_p * Sk;
      uint32_t prefix = 0, mask = 0;
      float above = 0.f;
      for (int shift = 24; shift >= 0; shift -= 8) {
        hist_f[tid] = 0.f;
        __syncthreads();
        for (int i = tid; i < V; i += 256) {
          const float f = ld1<T>(x + i);
          const uint32_t k = fkey(f);
          if (k >= kth && (k & mask) == prefix) atomicAdd(&hist_f[(k >> shift) & 255], __expf(f * inv_temp - M));
        }
        __syncthreads();
        if (tid == 0) {
          int bsel = 0;
          float a = above;
          for (int bb = 255; bb >= 0; --bb) {
            if (a + hist_f[bb] >= target || bb == 0) { bsel = bb; break; }
            a += hist_f[bb];
          }
          sh_key = bsel;
          sh_f = a;
        }
        __syncthreads();
        prefix |= sh_key << shift;
        mask |= 255u << shift;
        above = sh_f;
        __syncthreads();
      }
      pth = prefix > kth ? prefix : kth;
    }
    // ---- Gumbel-max draw over kept tokens ----
    const uint64_t off = offset_ptr ? (uint64_t)offset_ptr[0] : 0ull;
    float best = -INFINITY;
    int bi = AM;
    for (int i = tid; i < V; i += 256) {
      const float f = ld1<T>(x + i);
      if (fkey(f) >= pth) {
        const uint4 r = Philox::gen(seed, (uint64_t)row, off * (uint64_t)V + (uint64_t)i);
        const float u = u32_to_unit(r.x);
        const float gmb = -__logf(-__logf(u));
        const float sc = f * inv_temp + gmb;
        if (sc > best || (sc == best && i < bi)) { best = sc; bi = i; }
      }
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
      const float ob = __shfl_xor(best, o2, 64);
      const int oi = __shfl_xor(bi, o2, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    __syncthreads();
    if (lane == 0) { redf[wid] = best; redi[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      float B = redf[0];
      int BI = redi[0];
      for (int w = 1; w < 4; ++w)
        if (redf[w] > B || (redf[w] == B && redi[w] < BI)) { B = redf[w]; BI = redi[w]; }
      redi[0] = BI;
    }
    __syncthreads();
    tok = redi[0];
  }
  if (tid == 0) {
    out_tok[row] = tok;
    if (out_logp) out_logp[row] = ld1<T>(x + tok) * inv_temp - lse;
  }
}


// ---------------------------------------------------------------------------------------------
// bf16 fast path: the row (<= 80k tokens) is staged ONCE in LDS as 16-bit order-preserving keys;
// top-k / top-p thresholds are 2-pass 8-bit radix selects over those keys with per-wave
// histograms (no cross-wave atomic contention); Philox noise only for surviving tokens.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t key16(uint16_t b) {  // bf16 bits -> ascending unsigned key
  return (b & 0x8000u) ? (uint32_t)(~b & 0xFFFFu) : (uint32_t)(b | 0x8000u);
}
__device__ __forceinline__ float key16_to_f(uint32_t k) {
  const uint16_t b = (k & 0x8000u) ? (uint16_t)(k & 0x7FFFu) : (uint16_t)(~k & 0xFFFFu);
  return bf2f(b);
}

__global__ __launch_bounds__(256) void sample_bf16_lds_kernel(const bf16_t* __restrict__ logits, long ld, int V,
                                                              float inv_temp, int top_k, float top_p, int greedy,
                                                              uint64_t seed, const int64_t* __restrict__ offset_ptr,
                                                              const uint8_t* __restrict__ row_active,
                                                              long* __restrict__ out_tok, float* __restrict__ out_logp) {
  extern __shared__ __attribute__((aligned(16))) uint16_t keys[];   // [V] (+ pad) 16-bit keys
  __shared__ float hist[4][256];
  __shared__ float redf[8];
  __shared__ int redi[8];
  __shared__ uint32_t sh_sel;
  __shared__ float sh_f;
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nv = V / 8;

  // stage + max/argmax (keys are monotone in the logit value)
  uint32_t kmax = 0;
  int amx = 0;
  for (int c = tid; c < nv; c += 256) {
    const uint4 v = *(const uint4*)(x + (long)c * 8);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t k0 = key16((uint16_t)(w[q] & 0xFFFF)), k1 = key16((uint16_t)(w[q] >> 16));
      keys[c * 8 + 2 * q] = (uint16_t)k0;
      keys[c * 8 + 2 * q + 1] = (uint16_t)k1;
      if (k0 > kmax) { kmax = k0; amx = c * 8 + 2 * q; }
      if (k1 > kmax) { kmax = k1; amx = c * 8 + 2 * q + 1; }
    }
  }
  for (int i = nv * 8 + tid; i < V; i += 256) {
    const uint32_t k = key16(x[i]);
    keys[i] = (uint16_t)k;
    if (k > kmax) { kmax = k; amx = i; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t ok = __shfl_xor(kmax, off, 64);
    const int oi = __shfl_xor(amx, off, 64);
    if (ok > kmax || (ok == kmax && oi < amx)) { kmax = ok; amx = oi; }
  }
  if (lane == 0) { redi[wid] = amx; redf[wid] = __uint_as_float(kmax); }
  __syncthreads();
  uint32_t KM = __float_as_uint(redf[0]);
  int AM = redi[0];
  for (int w2 = 1; w2 < 4; ++w2) {
    const uint32_t k = __float_as_uint(redf[w2]);
    if (k > KM || (k == KM && redi[w2] < AM)) { KM = k; AM = redi[w2]; }
  }
  const float M = key16_to_f(KM) * inv_temp;
  __syncthreads();
  float s = 0.f;
  for (int i = tid; i < V; i += 256) s += __expf(key16_to_f(keys[i]) * inv_temp - M);
  const float S = block_sum(s, redf);
  const float lse = M + __logf(S);

  int tok = AM;
  const bool active = row_active ? row_active[row] != 0 : true;
  if (!greedy && active) {
    uint32_t kth = 0;
    if (top_k > 0 && top_k < V) {
      uint32_t prefix = 0;
      unsigned remaining = top_k;
      for (int shift = 8; shift >= 0; shift -= 8) {
        for (int i = tid; i < 1024; i += 256) (&hist[0][0])[i] = 0.f;
        __syncthreads();
        const uint32_t mask = shift == 8 ? 0u : 0xFF00u;
        for (int i = tid; i < V; i += 256) {
          const uint32_t k = keys[i];
          if ((k & mask) == prefix) atomicAdd(&hist[wid][(k >> shift) & 255], 1.f);
        }
        __syncthreads();
        if (tid == 0) {
          unsigned cum = 0;
          int bsel = 0;
          for (int bb = 255; bb >= 0; --bb) {
            const unsigned h = (unsigned)(hist[0][bb] + hist[1][bb] + hist[2][bb] + hist[3][bb]);
            if (cum + h >= remaining) { bsel = bb; break; }
            cum += h;
          }
          remaining -= cum;
          sh_sel = bsel;
        }
        __syncthreads();
        prefix |= sh_sel << shift;
        __syncthreads();
      }
      kth = prefix;
    }
    uint32_t pth = kth;
    if (top_p < 1.f) {
      float sk = 0.f;
      for (int i = tid; i < V; i += 256) {
        const uint32_t k = keys[i];
        if (k >= kth) sk += __expf(key16_to_f(k) * inv_temp - M);
      }
      const float target = top_p * block_sum(sk, redf);
      uint32_t prefix = 0;
      float above = 0.f;
      for (int shift = 8; shift >= 0; shift -= 8) {
        for (int i = tid; i < 1024; i += 256) (&hist[0][0])[i] = 0.f;
        __syncthreads();
        const uint32_t mask = shift == 8 ? 0u : 0xFF00u;
        for (int i = tid; i < V; i += 256) {
          const uint32_t k = keys[i];
          if (k >= kth && (k & mask) == prefix)
            atomicAdd(&hist[wid][(k >> shift) & 255], __expf(key16_to_f(k) * inv_temp - M));
        }
        __syncthreads();
        if (tid == 0) {
          int bsel = 0;
          float a = above;
          for (int bb = 255; bb >= 0; --bb) {
            const float h = hist[0][bb] + hist[1][bb] + hist[2][bb] + hist[3][bb];
            if (a + h >= target || bb == 0) { bsel = bb; break; }
            a += h;
          }
          sh_sel = bsel;
          sh_f = a;
        }
        __syncthreads();
        prefix |= sh_sel << shift;
        above = sh_f;
        __syncthreads();
      }
      pth = prefix > kth ? prefix : kth;
    }
    const uint64_t off = offset_ptr ? (uint64_t)offset_ptr[0] : 0ull;
    float best = -INFINITY;
    int bi = AM;
    for (int i = tid; i < V; i += 256) {
      const uint32_t k = keys[i];
      if (k >= pth) {
        const uint4 r = Philox::gen(seed, (uint64_t)row, off * (uint64_t)V + (uint64_t)i);
        const float gmb = -__logf(-__logf(u32_to_unit(r.x)));
        const float sc = key16_to_f(k) * inv_temp + gmb;
        if (sc > best || (sc == best && i < bi)) { best = sc; bi = i; }
      }
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
      const float ob = __shfl_xor(best, o2, 64);
      const int oi = __shfl_xor(bi, o2, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    __syncthreads();
    if (lane == 0) { redf[wid] = best; redi[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      float Bv = redf[0];
      int BI = redi[0];
      for (int w2 = 1; w2 < 4; ++w2)
        if (redf[w2] > Bv || (redf[w2] == Bv && redi[w2] < BI)) { Bv = redf[w2]; BI = redi[w2]; }
      redi[0] = BI;
    }
    __syncthreads();
    tok = redi[0];
  }
  if (tid == 0) {
    out_tok[row] = tok;
    if (out_logp) out_logp[row] = key16_to_f(keys[tok]) * inv_temp - lse;
  }
}

// ---------------------------------------------------------------------------------------------
// top-k (+ top-p) sampler for bf16 logits, one 1024-thread workgroup per row
// ---------------------------------------------------------------------------------------------
// The radix-histogram select above serialises on LDS atomics: bf16 logits share a handful of
// exponent values, so most lanes of a wave hit the same few high-byte bins (~100 us per row at
// V = 32000). Here the k-th largest key is found by a 16-step bitwise binary search over the
// LDS-resident keys (count >= candidate: a block reduction, no atomics), the <= CAP survivors are
// compacted, and top-p / the Gumbel draw run on the survivors only. Same kept set and the same
// Philox stream (seed, row, offset * V + token) as sample_bf16_lds_kernel, so the same token wins.
constexpr int TK_CAP = 2048;

// In-row (16-lane) all-reduce steps by DPP (xor 1, xor 2, half-mirror, mirror: afterwards every
// lane of a row holds the row's total) — register crossbar moves, where __shfl_xor is an LDS
// ds_bpermute round trip per step. A wave total is then the four row totals (v_readlane, scalar).
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ int row_sum_i(int v) {
  v += dpp_i<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_i<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_i<0x141>(v);  // row_half_mirror
  v += dpp_i<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
  v = row_sum_i(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ float wave_sum_f(float v) {
  auto step = [](float x, int sel) -> float {
    const int xi = __float_as_int(x);
    const int o = sel == 0 ? dpp_i<0xB1>(xi) : sel == 1 ? dpp_i<0x4E>(xi) : sel == 2 ? dpp_i<0x141>(xi) : dpp_i<0x140>(xi);
    return x + __int_as_float(o);
  };
  v = step(v, 0);
  v = step(v, 1);
  v = step(v, 2);
  v = step(v, 3);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}
// (key desc, index asc) argmax over the wave, result in every lane
__device__ __forceinline__ void wave_argmax(uint32_t& k, int& i) {
  auto step = [&](int sel) {
    const int ok = sel == 0 ? dpp_i<0xB1>((int)k) : sel == 1 ? dpp_i<0x4E>((int)k) : sel == 2 ? dpp_i<0x141>((int)k) : dpp_i<0x140>((int)k);
    const int oi = sel == 0 ? dpp_i<0xB1>(i) : sel == 1 ? dpp_i<0x4E>(i) : sel == 2 ? dpp_i<0x141>(i) : dpp_i<0x140>(i);
    if ((uint32_t)ok > k || ((uint32_t)ok == k && oi < i)) { k = (uint32_t)ok; i = oi; }
  };
  step(0);
  step(1);
  step(2);
  step(3);
  // the four row results (scalar), folded in row order
  uint32_t kb = (uint32_t)__builtin_amdgcn_readlane((int)k, 0);
  int ib = __builtin_amdgcn_readlane(i, 0);
  uint32_t kr_[3];
  int ir_[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    kr_[r] = (uint32_t)__builtin_amdgcn_readlane((int)k, 16 * (r + 1));
    ir_[r] = __builtin_amdgcn_readlane(i, 16 * (r + 1));
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
    if (kr_[r] > kb || (kr_[r] == kb && ir_[r] < ib)) { kb = kr_[r]; ib = ir_[r]; }
  k = kb;
  i = ib;
}
// candidate windows below the row maximum, in key steps (bf16 ulps): 8, 12, 16, 24, ... 1536
// (x sqrt 2), counted on a 1-in-8 subsample of the keys (element 0 of every 8-key chunk), two 16-bit
// counts per int
constexpr int NWIN = 16;
__device__ __forceinline__ constexpr uint32_t kwin(int q) { return (q & 1 ? 12u : 8u) << (q >> 1); }

__device__ __forceinline__ int block_sum_int1024(int v, int* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(1024) void sample_topk_search_kernel(
    const bf16_t* __restrict__ logits, long ld, int V, float inv_temp, int top_k, float top_p, uint64_t seed,
    const int64_t* __restrict__ offset_ptr, const uint8_t* __restrict__ row_active, long* __restrict__ out_tok,
    float* __restrict__ out_logp, int flags) {
  // flags bit 0: candidate window (tuning sample_window); bit 1: the <= 64-survivor wave-0 fast
  // path (tuning sample_fast64; 0 sends those rows through the block-wide sort / top-p / Gumbel
  // path, the same arithmetic — tests pin the two bitwise)
  const bool use_window = flags & 1, fast64 = flags & 2;
  extern __shared__ __attribute__((aligned(16))) uint16_t keys[];  // [V]
  __shared__ int lidx[TK_CAP];
  __shared__ float lval[TK_CAP];   // tempered logit of each survivor
  __shared__ uint16_t lkey[TK_CAP];  // window path: key of each candidate
  __shared__ int redi[16][NWIN / 2 + 1];
  __shared__ float redf[16];
  __shared__ int cnt;
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nv = V / 8;

  // pass 1: stage keys (the first RC chunks of every thread stay in registers, raw bf16 words and
  // keys), row max. All of a thread's register-chunk loads are issued before the first is used (one
  // round trip); keys are built two per 32-bit word and maxed with packed 16-bit ops (the kernel is
  // VALU-bound on its one CU at batch 1). The argmax index (smallest index of the max key) is found
  // in pass 2 by the few threads that hold the max.
  constexpr int RC = 4;
  typedef __attribute__((ext_vector_type(2))) unsigned short u16x2_t;
  uint4 rr[RC], kr[RC];
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = tid + i * 1024;
    rr[i] = c < nv ? *(const uint4*)(x + (long)c * 8) : make_uint4(0, 0, 0, 0);
  }
  // key of each bf16 half: negatives bit-flipped, positives with the sign bit set (= key16)
  auto keyw = [](uint32_t w) -> uint32_t { return w ^ (((w & 0x80008000u) >> 15) * 0x7FFFu | 0x80008000u); };
  auto pmax = [](uint32_t a, uint32_t b) -> uint32_t {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, a), __builtin_bit_cast(u16x2_t, b)));
  };
  auto keys_of = [&](const uint4& v) -> uint4 { return make_uint4(keyw(v.x), keyw(v.y), keyw(v.z), keyw(v.w)); };
  auto cmax_of = [&](const uint4& k) -> uint32_t {  // max key of a chunk
    const uint32_t m = pmax(pmax(k.x, k.y), pmax(k.z, k.w));
    return max(m & 0xFFFFu, m >> 16);
  };
  uint32_t kmax = 0;
#pragma unroll
  for (int i = 0; i < RC; ++i) {
    const int c = tid + i * 1024;
    if (c < nv) {
      kr[i] = keys_of(rr[i]);
      *(uint4*)(keys + c * 8) = kr[i];
      kmax = max(kmax, cmax_of(kr[i]));
    } else {
      kr[i] = make_uint4(0, 0, 0, 0);
    }
  }
  for (int c = tid + RC * 1024; c < nv; c += 1024) {
    const uint4 kv = keys_of(*(const uint4*)(x + (long)c * 8));
    *(uint4*)(keys + c * 8) = kv;
    kmax = max(kmax, cmax_of(kv));
  }
  const uint32_t kmax_own = kmax;
  {
    int ki = (int)kmax, dummy = 0;
    // wave max (index unused: every lane passes 0)
    uint32_t ku = (uint32_t)ki;
    wave_argmax(ku, dummy);
    kmax = ku;
  }
  __shared__ int amin;
  if (tid == 0) { cnt = 0; amin = 0x7fffffff; }
  if (lane == 0) redf[wid] = __uint_as_float(kmax);
  __syncthreads();
  uint32_t KM = __float_as_uint(redf[0]);
  for (int w2 = 1; w2 < 16; ++w2) KM = max(KM, __float_as_uint(redf[w2]));
  const float M = key16_to_f(KM) * inv_temp;
  // pass 2: normaliser of the full tempered distribution (behaviour log-prob); for the window path,
  // how many subsample keys lie within kwin(q) key steps (bf16 ulps) below the maximum; and the
  // argmax index (threads holding a max key: first match in index order, LDS atomicMin)
  float s = 0.f;
  int wc[NWIN / 2] = {};  // field q & 1 (16 bits) of wc[q / 2]
  auto pass2 = [&](const uint4& raw, const uint4& kv) {
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = __uint_as_float(e & 1 ? (w[e >> 1] & 0xFFFF0000u) : (w[e >> 1] << 16));
      s += __expf(f * inv_temp - M);
    }
    const uint32_t d = KM - (kv.x & 0xFFFFu);
#pragma unroll
    for (int q = 0; q < NWIN; ++q) wc[q >> 1] += (d < kwin(q)) ? (1 << (16 * (q & 1))) : 0;
  };
#pragma unroll
  for (int i = 0; i < RC; ++i)
    if (tid + i * 1024 < nv) pass2(rr[i], kr[i]);
  for (int c = tid + RC * 1024; c < nv; c += 1024) pass2(*(const uint4*)(x + (long)c * 8), *(const uint4*)(keys + c * 8));
  if (kmax_own == KM) {
    int idx = 0x7fffffff;
    for (int c = tid; c < nv && idx == 0x7fffffff; c += 1024) {
      const uint4 kv = *(const uint4*)(keys + c * 8);
      const uint16_t* k8 = (const uint16_t*)&kv;
      for (int e = 0; e < 8; ++e)
        if (k8[e] == KM) { idx = c * 8 + e; break; }
    }
    atomicMin(&amin, idx);
  }
  s = wave_sum_f(s);
#pragma unroll
  for (int q = 0; q < NWIN / 2; ++q) wc[q] = wave_sum_i(wc[q]);
  __syncthreads();
  if (lane == 0) {
    redf[wid] = s;
#pragma unroll
    for (int q = 0; q < NWIN / 2; ++q) redi[wid][q] = wc[q];
  }
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int w2 = 0; w2 < 16; ++w2) S += redf[w2];
  const float lse = M + __logf(S);
  const int AM = amin;

  int tok = AM;
  const bool active = row_active ? row_active[row] != 0 : true;
  if (active) {
    const int K = min(top_k, V);
    // window path: a window below the maximum holding >= K keys and at most TK_CAP (typically
    // 2-3 K) — every key >= the k-th largest is in it, so the k-th largest over the window's
    // candidates IS the k-th largest over the row. The window is sized from the subsample counts
    // (the narrowest with >= K / 4 + 2 subsample keys: ~2 K candidates); its exact count is known
    // after the compaction, and a window holding < K or > TK_CAP keys falls back to the full-row
    // search.
    // The candidates go to LDS (wave-aggregated slots) and ONE wave finds the k-th key with wave
    // reductions only, instead of 16 block-wide passes.
    uint32_t win = 0;
    if (use_window) {
      // every wave: lane l < 16 holds wave l's packed counts, a row reduce sums them (no barrier)
      const int need = K / 4 + 2;
      int tot[NWIN / 2];
#pragma unroll
      for (int q = 0; q < NWIN / 2; ++q)
        tot[q] = __builtin_amdgcn_readlane(row_sum_i(redi[lane & 15][q]), 0);
#pragma unroll
      for (int q = NWIN - 1; q >= 0; --q)
        if (((tot[q >> 1] >> (16 * (q & 1))) & 0xFFFF) >= need) win = kwin(q);
    }
    uint32_t kth = 0;
    bool done = false;
    if (win) {
      // chunks with a key in the window (chunk max vs the window floor, packed) place their
      // candidates through an LDS slot counter — a few hundred of 32000 keys
      auto cand = [&](const uint4& kv, int c) {
        if (c < nv && KM - cmax_of(kv) < win) {
          const uint16_t* k8 = (const uint16_t*)&kv;
          for (int e = 0; e < 8; ++e)
            if (KM - k8[e] < win) {
              const int pos = atomicAdd(&cnt, 1);
              if (pos < TK_CAP) { lidx[pos] = c * 8 + e; lkey[pos] = k8[e]; }
            }
        }
      };
#pragma unroll
      for (int i = 0; i < RC; ++i) cand(kr[i], tid + i * 1024);
      for (int c = tid + RC * 1024; c < nv; c += 1024) cand(*(const uint4*)(keys + c * 8), c);
      __syncthreads();
      const int n = cnt;
      // every thread has read cnt before wave 0 (compaction below) or thread 0 (retry) rewrites it
      __syncthreads();
      if (n >= K && n <= TK_CAP) {
        done = true;
        if (wid == 0) {
          // k-th largest key: largest t with count(keys >= t) >= K, bit by bit from the top; the
          // lane's first 8 candidates in registers
          constexpr int CR = 8;
          uint32_t ck[CR];
#pragma unroll
          for (int i = 0; i < CR; ++i) ck[i] = lane + 64 * i < n ? lkey[lane + 64 * i] : 0u;
          uint32_t prefix = 0;
          for (int b = 15; b >= 0; --b) {
            const uint32_t cnd = prefix | (1u << b);
            int c = 0;  // wave-uniform: ballot popcounts
#pragma unroll
            for (int i = 0; i < CR; ++i) c += (int)__popcll(__ballot(ck[i] >= cnd && lane + 64 * i < n));
            for (int j0 = 64 * CR; j0 < n; j0 += 64)
              c += (int)__popcll(__ballot(j0 + lane < n && lkey[min(j0 + lane, n - 1)] >= cnd));
            if (c >= K) prefix = cnd;
          }
          kth = prefix;
          // survivors (key >= kth, ties kept) compacted in place, in candidate order
          int ns = 0;
          for (int j0 = 0; j0 < n; j0 += 64) {
            const int j = j0 + lane;
            const bool in = j < n;
            const int idx = in ? lidx[j] : 0;
            const uint32_t key = in ? lkey[j] : 0u;
            const bool keep = in && key >= kth;
            const unsigned long long bal = __ballot(keep);
            const int pos = ns + (int)__popcll(bal & ((1ull << lane) - 1ull));
            if (keep) { lidx[pos] = idx; lval[pos] = key16_to_f(key) * inv_temp; }
            ns += (int)__popcll(bal);
          }
          if (lane == 0) cnt = ns;
        }
      } else {
        if (tid == 0) cnt = 0;
        __syncthreads();
      }
    }
    if (!done) {
      // k-th largest key over the LDS-resident keys: 16 block-wide counting passes
      uint32_t prefix = 0;
      for (int b = 15; b >= 0; --b) {
        const uint32_t cnd = prefix | (1u << b);
        int c = 0;
        for (int cc = tid; cc < nv; cc += 1024) {
          const uint4 kv = *(const uint4*)(keys + cc * 8);
          const uint16_t* k8 = (const uint16_t*)&kv;
#pragma unroll
          for (int e = 0; e < 8; ++e) c += k8[e] >= cnd;
        }
        if (block_sum_int1024(c, &redi[0][0]) >= K) prefix = cnd;
      }
      kth = prefix;
      // compact the survivors (ties at the threshold kept)
      for (int cc = tid; cc < nv; cc += 1024) {
        const uint4 kv = *(const uint4*)(keys + cc * 8);
        const uint16_t* k8 = (const uint16_t*)&kv;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (k8[e] >= kth) {
            const int pos = atomicAdd(&cnt, 1);
            if (pos < TK_CAP) { lidx[pos] = cc * 8 + e; lval[pos] = key16_to_f(k8[e]) * inv_temp; }
          }
      }
    }
    __syncthreads();
    const bool overflow = cnt > TK_CAP;  // > TK_CAP - top_k ties at the k-th value: draw from the keys
    const int n = min(cnt, TK_CAP);
    if (!overflow && n <= 64 && fast64) {
      // <= 64 survivors (top-k 50): sort, nucleus cut and Gumbel draw in wave 0's registers, no
      // block barrier — the same arithmetic, lane assignment and reduction order as the general
      // path below, so the same token
      if (wid != 0) return;
      float v = lane < n ? lval[lane] : -INFINITY;
      int ix = lane < n ? lidx[lane] : 0x7fffffff;
      float vthr = -INFINITY;
      if (top_p < 1.f && n > 1) {
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
          for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const float ov = __shfl_xor(v, stride, 64);
            const int oi = __shfl_xor(ix, stride, 64);
            const bool i_lo = (lane & stride) == 0;
            const bool desc = ((lane & ~stride) & size) == 0;
            const bool mine_first = v > ov || (v == ov && ix < oi);
            if (!((i_lo == desc) ? mine_first : !mine_first)) { v = ov; ix = oi; }
          }
        // one survivor per lane (per = 1): the general path's chunked prefix with a chunk of one
        const float part = lane < n ? __expf(v - M) : 0.f;
        float incl = part;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        const float total = __shfl(incl, 63, 64);
        const float target = top_p * total;
        float run = incl - part;
        bool found = false;
        if (lane < n) {
          run += __expf(v - M);
          found = run >= target;
        }
        const unsigned long long m = __ballot(found);
        const int src = m ? __ffsll((long long)m) - 1 : n - 1;
        vthr = __shfl(v, src, 64);
      }
      const uint64_t off = offset_ptr ? (uint64_t)offset_ptr[0] : 0ull;
      float best = -INFINITY;
      int bi = AM;
      if (lane < n && v >= vthr) {
        const uint4 r = Philox::gen(seed, (uint64_t)row, off * (uint64_t)V + (uint64_t)ix);
        best = v - __logf(-__logf(u32_to_unit(r.x)));
        bi = ix;
      }
#pragma unroll
      for (int o2 = 32; o2 > 0; o2 >>= 1) {
        const float ob = __shfl_xor(best, o2, 64);
        const int oi = __shfl_xor(bi, o2, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      if (lane == 0) {
        out_tok[row] = bi;
        if (out_logp) out_logp[row] = key16_to_f(keys[bi]) * inv_temp - lse;
      }
      return;
    }
    float vthr = -INFINITY;  // kept: lval >= vthr
    if (top_p < 1.f && n > 1 && !overflow) {
      // sort survivors by (value desc, token asc) — a total order, so every sorting network gives
      // the same sequence. n <= 64 (top-k 50): one wave, in registers, no barriers
      if (n <= 64) {
        if (wid == 0) {
          float v = lane < n ? lval[lane] : -INFINITY;
          int ix = lane < n ? lidx[lane] : 0x7fffffff;
#pragma unroll
          for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
              const float ov = __shfl_xor(v, stride, 64);
              const int oi = __shfl_xor(ix, stride, 64);
              const bool i_lo = (lane & stride) == 0;
              const bool desc = ((lane & ~stride) & size) == 0;
              const bool mine_first = v > ov || (v == ov && ix < oi);
              if (!((i_lo == desc) ? mine_first : !mine_first)) { v = ov; ix = oi; }
            }
          lval[lane] = v;
          lidx[lane] = ix;
        }
        __syncthreads();
      } else {
      // bitonic over the next power of two, block-wide
      int P = 1;
      while (P < n) P <<= 1;
      for (int i = n + tid; i < P; i += 1024) { lval[i] = -INFINITY; lidx[i] = 0x7fffffff; }
      __syncthreads();
      for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = tid; i < P / 2; i += 1024) {
            const int lo = 2 * i - (i & (stride - 1));
            const int hi = lo + stride;
            const bool desc = ((lo & size) == 0);
            const float a = lval[lo], bv = lval[hi];
            const int ia = lidx[lo], ib = lidx[hi];
            const bool a_first = a > bv || (a == bv && ia < ib);
            if (a_first != desc) { lval[lo] = bv; lval[hi] = a; lidx[lo] = ib; lidx[hi] = ia; }
          }
          __syncthreads();
        }
      }
      // smallest prefix whose mass reaches top_p of the survivors' mass (one wave, serial chunks)
      if (wid == 0) {
        const int per = (n + 63) / 64;
        float part = 0.f;
        for (int j = lane * per; j < min(n, (lane + 1) * per); ++j) part += __expf(lval[j] - M);
        float incl = part;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        const float total = __shfl(incl, 63, 64);
        const float target = top_p * total;
        float run = incl - part;  // exclusive prefix of this lane's chunk
        int jcut = n - 1;
        bool found = false;
        for (int j = lane * per; j < min(n, (lane + 1) * per); ++j) {
          run += __expf(lval[j] - M);
          if (run >= target) { jcut = j; found = true; break; }
        }
        // first lane (lowest index) that reached the target
        const unsigned long long m = __ballot(found);
        const int src = m ? __ffsll((long long)m) - 1 : 63;
        jcut = __shfl(jcut, src, 64);
        if (lane == 0) redf[0] = lval[jcut];
      }
      __syncthreads();
      vthr = redf[0];
      __syncthreads();
    }
    // Gumbel-max over the kept survivors
    const uint64_t off = offset_ptr ? (uint64_t)offset_ptr[0] : 0ull;
    float best = -INFINITY;
    int bi = AM;
    if (!overflow) {
      for (int j = tid; j < n; j += 1024) {
        const float v = lval[j];
        if (v >= vthr) {
          const int i = lidx[j];
          const uint4 r = Philox::gen(seed, (uint64_t)row, off * (uint64_t)V + (uint64_t)i);
          const float sc = v - __logf(-__logf(u32_to_unit(r.x)));
          if (sc > best || (sc == best && i < bi)) { best = sc; bi = i; }
        }
      }
    } else {  // degenerate tie plateau: top-k set only (top-p not applied), straight from the keys
      for (int i = tid; i < V; i += 1024) {
        const uint32_t k = keys[i];
        if (k >= kth) {
          const uint4 r = Philox::gen(seed, (uint64_t)row, off * (uint64_t)V + (uint64_t)i);
          const float sc = key16_to_f(k) * inv_temp - __logf(-__logf(u32_to_unit(r.x)));
          if (sc > best || (sc == best && i < bi)) { best = sc; bi = i; }
        }
      }
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
      const float ob = __shfl_xor(best, o2, 64);
      const int oi = __shfl_xor(bi, o2, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    __syncthreads();
    if (lane == 0) { redf[wid] = best; redi[wid][0] = bi; }
    __syncthreads();
    if (tid == 0) {
      float Bv = redf[0];
      int BI = redi[0][0];
      for (int w2 = 1; w2 < 16; ++w2)
        if (redf[w2] > Bv || (redf[w2] == Bv && redi[w2][0] < BI)) { Bv = redf[w2]; BI = redi[w2][0]; }
      redi[0][0] = BI;
    }
    __syncthreads();
    tok = redi[0][0];
  }
  if (tid == 0) {
    out_tok[row] = tok;
    if (out_logp) out_logp[row] = key16_to_f(keys[tok]) * inv_temp - lse;
  }
}

}  // namespace rt

using namespace rt;

extern "C" int rt_sample(const void* logits, int is_f32, long ld, long B, int V, float inv_temp, int top_k, float top_p,
                         int greedy, uint64_t seed, const int64_t* offset_ptr, const uint8_t* row_active, long* out_tok,
                         float* out_logp, hipStream_t stream) {
  if (B == 0) return 0;
  if (!is_f32 && !greedy && top_k > 0 && top_k <= 1024 && V % 8 == 0 && ld % 8 == 0 && (size_t)V * 2 <= 96 * 1024) {
    const size_t shm = ((size_t)V * 2 + 15) / 16 * 16;
    hipLaunchKernelGGL(sample_topk_search_kernel, dim3(B), dim3(1024), shm, stream, (const bf16_t*)logits, ld, V,
                       inv_temp, top_k, top_p, seed, offset_ptr, row_active, out_tok, out_logp,
                       (tuning().sample_window ? 1 : 0) | (tuning().sample_fast64 ? 2 : 0));
    RT_LAUNCH_CHECK();
    return 0;
  }
  if (!is_f32 && V % 8 == 0 && ld % 8 == 0 && (size_t)V * 2 <= 96 * 1024) {
    const size_t shm = ((size_t)V * 2 + 15) / 16 * 16;
    hipLaunchKernelGGL(sample_bf16_lds_kernel, dim3(B), dim3(256), shm, stream, (const bf16_t*)logits, ld, V, inv_temp,
                       top_k, top_p, greedy, seed, offset_ptr, row_active, out_tok, out_logp);
    RT_LAUNCH_CHECK();
    return 0;
  }
  if (is_f32)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(256), 0, stream, (const float*)logits, ld, V, inv_temp,
                       top_k, top_p, greedy, seed, offset_ptr, row_active, out_tok, out_logp);
  else
    hipLaunchKernelGGL(sample_kernel<bf16_t>, dim3(B), dim3(256), 0, stream, (const bf16_t*)logits, ld, V, inv_temp,
                       top_k, top_p, greedy, seed, offset_ptr, row_active, out_tok, out_logp);
  RT_LAUNCH_CHECK();
  return 0;
}
