// Dense-retrieval kernels (SURVEY K12 pool+normalise, K13 flat top-k, K14 IVF list scan).
//
// The bi-encoder's sentence embedding is a masked mean over tokens followed by L2 normalisation
// (sentence-transformers pooling). Search scores are inner products of normalised vectors
// (= cosine), produced by the MFMA GEMM for flat search or by the IVF list scan below; the top-k
// of a row is an exact 4-pass radix select of the k-th largest score followed by an LDS bitonic
// sort of the survivors (no full sort of N = 100k scores).
#include "rt_common.h"

namespace rt {

// x [B, S, H] bf16, lengths [B] -> out [B, H] fp32 (L2-normalised if norm != 0)
__global__ __launch_bounds__(256) void pool_norm_kernel(const bf16_t* __restrict__ x, const int* __restrict__ lengths,
                                                        int S, int H, int normalize, float* __restrict__ out) {
  extern __shared__ float acc[];  // [H]
  __shared__ float sb[4];
  const int b = blockIdx.x;
  const int len = lengths ? lengths[b] : S;
  for (int h = threadIdx.x; h < H; h += 256) {
    float s = 0.f;
    for (int t = 0; t < len; ++t) s += bf2f(x[((long)b * S + t) * H + h]);
    acc[h] = s / (float)max(len, 1);
  }
  __syncthreads();
  float ss = 0.f;
  for (int h = threadIdx.x; h < H; h += 256) ss += acc[h] * acc[h];
  const float tot = block_sum(ss, sb);
  const float inv = normalize ? 1.f / fmaxf(sqrtf(tot), 1e-12f) : 1.f;
  for (int h = threadIdx.x; h < H; h += 256) out[(long)b * H + h] = acc[h] * inv;
}

__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int TOPK_CAND = 1024;  // max survivors sorted in LDS (k + ties)

// scores [nq, N] fp32 (row stride ld) -> vals/ids [nq, k] sorted descending; ids optionally mapped
// through idmap (IVF candidate slot -> document id). Scores of -inf are never returned as hits
// unless fewer than k finite scores exist.
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ scores, long ld, int N, int k,
                                                   const long* __restrict__ idmap, long ldmap,
                                                   float* __restrict__ out_v, long* __restrict__ out_i) {
  __shared__ unsigned hist[256];
  __shared__ uint32_t sh_sel;
  __shared__ unsigned sh_cnt;
  __shared__ float cv[TOPK_CAND];
  __shared__ int ci[TOPK_CAND];
  const long row = blockIdx.x;
  const float* s = scores + row * ld;
  const int tid = threadIdx.x;
  uint32_t prefix = 0, mask = 0;
  unsigned remaining = (unsigned)min(k, N);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += 256) {
      const uint32_t key = okey(s[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned cum = 0;
      int sel = 0;
      for (int b = 255; b >= 0; --b) {
        if (cum + hist[b] >= remaining) { sel = b; break; }
        cum += hist[b];
      }
      remaining -= cum;
      sh_sel = sel;
    }
    __syncthreads();
    prefix |= sh_sel << shift;
    mask |= 255u << shift;
    __syncthreads();
  }
  // gather survivors (key >= prefix): strictly-greater first guaranteed < k, ties fill the rest
  if (tid == 0) sh_cnt = 0;
  for (int i = tid; i < TOPK_CAND; i += 256) { cv[i] = -INFINITY; ci[i] = 0x7fffffff; }
  __syncthreads();
  for (int i = tid; i < N; i += 256) {
    const float v = s[i];
    if (okey(v) >= prefix) {
      const unsigned slot = atomicAdd(&sh_cnt, 1u);
      if (slot < TOPK_CAND) { cv[slot] = v; ci[slot] = i; }
    }
  }
  __syncthreads();
  // bitonic sort descending by value, ascending index on ties
  for (int size = 2; size <= TOPK_CAND; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < TOPK_CAND; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const float vi = cv[i], vj = cv[j];
          const int ii = ci[i], ij = ci[j];
          const bool i_first = vi > vj || (vi == vj && ii < ij);
          if (desc != i_first) { cv[i] = vj; cv[j] = vi; ci[i] = ij; ci[j] = ii; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += 256) {
    out_v[row * k + i] = cv[i];
    const int idx = ci[i];
    long id = idx == 0x7fffffff ? -1 : idx;
    if (idmap && id >= 0) id = idmap[row * ldmap + id];
    out_i[row * k + i] = id;
  }
}

// IVF list scan: for query qi and its probe p (list L = probes[qi, p]), score every vector of the
// list (vectors stored contiguously per list from lstart[L], lsize[L] of them; lists may carry
// spare capacity for incremental adds) and write into cand[qi, p*maxlen + j] (+ ids).
// Metric: inner product, or (l2) the negated squared distance 2 q.x - |x|^2 - |q|^2 with |x|^2
// stored per slot — both "higher is better" for the shared top-k. Unused slots get -inf.
// One workgroup per (probe, query); one thread per vector, query in LDS.
__global__ __launch_bounds__(256) void ivf_scan_kernel(const bf16_t* __restrict__ q, int d, const int* __restrict__ probes,
                                                       int nprobe, const int* __restrict__ lstart,
                                                       const int* __restrict__ lsize, const bf16_t* __restrict__ vecs,
                                                       const long* __restrict__ ids, const float* __restrict__ sqnorm,
                                                       int l2, int maxlen, float* __restrict__ cand,
                                                       long* __restrict__ cand_ids) {
  extern __shared__ float qs[];
  __shared__ float sb[4];
  const int p = blockIdx.x, qi = blockIdx.y;
  float qq = 0.f;
  for (int i = threadIdx.x; i < d; i += 256) {
    const float v = bf2f(q[(long)qi * d + i]);
    qs[i] = v;
    qq += v * v;
  }
  const float qn = l2 ? block_sum(qq, sb) : 0.f;  // block_sum synchronises
  __syncthreads();
  const int L = probes[(long)qi * nprobe + p];
  const int b0 = L >= 0 ? lstart[L] : 0;
  const int len = L >= 0 ? min(lsize[L], maxlen) : 0;
  float* out = cand + ((long)qi * nprobe + p) * maxlen;
  long* oid = cand_ids + ((long)qi * nprobe + p) * maxlen;
  for (int j = threadIdx.x; j < maxlen; j += 256) {
    if (j < len) {
      const bf16_t* vr = vecs + (long)(b0 + j) * d;
      float s = 0.f;
      for (int c = 0; c < d; c += 8) {
        float f[8];
        unpack8(*(const uint4*)(vr + c), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += f[e] * qs[c + e];
      }
      out[j] = l2 ? 2.f * s - sqnorm[b0 + j] - qn : s;
      oid[j] = ids[b0 + j];
    } else {
      out[j] = -INFINITY;
      oid[j] = -1;
    }
  }
}

// k-means update: centroid c = mean of the rows order[seg[c] .. seg[c+1]) of x (rows sorted by
// assigned centroid), L2-normalised for the inner-product metric. One workgroup per centroid, a
// column per thread, rows summed in a fixed order (deterministic, no atomics). Empty clusters are
// left untouched (the caller reseeds them). mode bit 0: L2-normalise; bit 1: the plain segment sum
// (the deterministic embedding-table gradient, ops.misc._EmbedFn).
__global__ __launch_bounds__(256) void segment_mean_kernel(const float* __restrict__ x, int d,
                                                           const long* __restrict__ order, const int* __restrict__ seg,
                                                           int mode, float* __restrict__ out) {
  extern __shared__ float col[];  // [d]
  __shared__ float sb[4];
  const int c = blockIdx.x;
  const int r0 = seg[c], r1 = seg[c + 1];
  if (r1 <= r0) return;  // uniform over the block
  const bool normalize = mode & 1;
  const float inv = (mode & 2) ? 1.f : 1.f / (float)(r1 - r0);  // bit 1: plain sum
  float ss = 0.f;
  for (int j = threadIdx.x; j < d; j += 256) {
    float a = 0.f;
    for (int r = r0; r < r1; ++r) a += x[order[r] * (long)d + j];
    a *= inv;
    col[j] = a;
    ss += a * a;
  }
  const float tot = normalize ? block_sum(ss, sb) : 1.f;
  const float scale = normalize ? 1.f / fmaxf(sqrtf(tot), 1e-12f) : 1.f;
  __syncthreads();
  for (int j = threadIdx.x; j < d; j += 256) out[(long)c * d + j] = col[j] * scale;
}

}  // namespace rt

using namespace rt;

extern "C" int rt_pool_norm(const void* x, const int* lengths, int B, int S, int H, int normalize, float* out,
                            hipStream_t stream) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(pool_norm_kernel, dim3(B), dim3(256), H * sizeof(float), stream, (const bf16_t*)x, lengths, S, H,
                     normalize, out);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_topk(const float* scores, long ld, long nq, int N, int k, const long* idmap, long ldmap, float* out_v,
                       long* out_i, hipStream_t stream) {
  if (k > TOPK_CAND / 2) return -1;
  if (nq == 0) return 0;
  hipLaunchKernelGGL(topk_kernel, dim3(nq), dim3(256), 0, stream, scores, ld, N, k, idmap, ldmap, out_v, out_i);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_ivf_scan(const void* q, int nq, int d, const int* probes, int nprobe, const int* lstart,
                           const int* lsize, const void* vecs, const long* ids, const float* sqnorm, int l2,
                           int maxlen, float* cand, long* cand_ids, hipStream_t stream) {
  if (d % 8 != 0 || (l2 && !sqnorm)) return -1;
  if (nq == 0) return 0;
  hipLaunchKernelGGL(ivf_scan_kernel, dim3(nprobe, nq), dim3(256), d * sizeof(float), stream, (const bf16_t*)q, d,
                     probes, nprobe, lstart, lsize, (const bf16_t*)vecs, ids, sqnorm, l2, maxlen, cand, cand_ids);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_segment_mean(const float* x, int d, const long* order, const int* seg, int k, int mode,
                               float* out, hipStream_t stream) {
  if (k == 0) return 0;
  hipLaunchKernelGGL(segment_mean_kernel, dim3(k), dim3(256), d * sizeof(float), stream, x, d, order, seg, mode, out);
  RT_LAUNCH_CHECK();
  return 0;
}
