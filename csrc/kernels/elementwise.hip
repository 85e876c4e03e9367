// Memory-bound elementwise kernels (SURVEY K3 RoPE, K6 SwiGLU, K15 embedding gather / KV append).
// All bf16 traffic is 16-B vectorised (cdna_hip_programming.md Guideline 13); RoPE reads a host
// precomputed fp32 cos/sin table instead of evaluating trig on device (Appendix B, element-wise).
#include "rt_common.h"

namespace rt {

// ---------------------------------------------------------------------------------------------
// RoPE (HF rotate_half convention: pairs (i, i + D/2)) on a fused qkv buffer, fused with the
// KV-cache append. One thread = 8 rotation pairs of one (token, head).
//   qkv   [T, ld]   q heads at [0, Hq*D), k heads at [Hq*D, (Hq+Hkv)*D), v after
//   pos   [T]       rotary position of each token
//   cos/sin [P, D/2] fp32
//   caches [B, Hkv, Smax, D] (optional): token t = b*S + s goes to slot slot_base[b] + s
//   sign = +1 forward, -1 backward (inverse rotation of the incoming gradient)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_qkv_kernel(bf16_t* __restrict__ qkv, long ld, const int* __restrict__ pos,
                                                       const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                       int T, int S, int Hq, int Hkv, int D, float sign,
                                                       bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                       const int* __restrict__ slot_base, int Smax, int do_rope_q) {
  const int per_head = D / 16;
  const int nheads = Hq + 2 * Hkv;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)T * nheads * per_head;
  if (gid >= total) return;
  const int c = gid % per_head;
  const int head = (gid / per_head) % nheads;
  const long t = gid / ((long)per_head * nheads);
  const int half = D / 2;
  bf16_t* row = qkv + t * ld + (long)head * D;
  const int e1 = c * 8, e2 = half + c * 8;
  float a[8], b[8];
  unpack8(*(const uint4*)(row + e1), a);
  unpack8(*(const uint4*)(row + e2), b);
  const bool is_q = head < Hq, is_k = !is_q && head < Hq + Hkv;
  if (cosT && (is_k || (is_q && do_rope_q))) {
    const int p = pos[t];
    const float* cr = cosT + (long)p * half + e1;
    const float* sr = sinT + (long)p * half + e1;
    const float4 c0 = *(const float4*)cr, c1 = *(const float4*)(cr + 4);
    const float4 s0 = *(const float4*)sr, s1 = *(const float4*)(sr + 4);
    const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x1 = a[k], x2 = b[k], s = sign * sn[k];
      // explicit fma order (the fused decode kernels round identically: bitwise-equal cache appends)
      a[k] = fmaf(x1, cs[k], -(x2 * s));
      b[k] = fmaf(x2, cs[k], x1 * s);
    }
    *(uint4*)(row + e1) = pack8(a);
    *(uint4*)(row + e2) = pack8(b);
  }
  if (kc && !is_q) {
    const int bidx = t / S, s = t % S;
    const int hk = is_k ? head - Hq : head - Hq - Hkv;
    bf16_t* cache = is_k ? kc : vc;
    RT_ASSERT((slot_base ? slot_base[bidx] : 0) + s < Smax);
    bf16_t* dst = cache + (((long)bidx * Hkv + hk) * Smax + (slot_base ? slot_base[bidx] : 0) + s) * D;
    *(uint4*)(dst + e1) = pack8(a);
    *(uint4*)(dst + e2) = pack8(b);
  }
}

// ---------------------------------------------------------------------------------------------
// SwiGLU: gu [T, 2F] (gate | up) -> y [T, F] = silu(gate) * up ; backward to dgu [T, 2F].
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ y, long T,
                                                         int F) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nv = F / 8;
  if (gid >= T * nv) return;
  const long t = gid / nv;
  const int c = gid % nv;
  float g[8], u[8], o[8];
  unpack8(*(const uint4*)(gu + t * 2 * F + c * 8), g);
  unpack8(*(const uint4*)(gu + t * 2 * F + F + c * 8), u);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = g[k] / (1.f + __expf(-g[k])) * u[k];
  *(uint4*)(y + t * F + c * 8) = pack8(o);
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dy,
                                                         bf16_t* __restrict__ dgu, long T, int F) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nv = F / 8;
  if (gid >= T * nv) return;
  const long t = gid / nv;
  const int c = gid % nv;
  float g[8], u[8], d[8], dg[8], du[8];
  unpack8(*(const uint4*)(gu + t * 2 * F + c * 8), g);
  unpack8(*(const uint4*)(gu + t * 2 * F + F + c * 8), u);
  unpack8(*(const uint4*)(dy + t * F + c * 8), d);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float sg = 1.f / (1.f + __expf(-g[k]));
    const float si = g[k] * sg;
    du[k] = d[k] * si;
    dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
  }
  *(uint4*)(dgu + t * 2 * F + c * 8) = pack8(dg);
  *(uint4*)(dgu + t * 2 * F + F + c * 8) = pack8(du);
}

// ---------------------------------------------------------------------------------------------
// Embedding gather: out[t] = table[ids[t]] (+ pos_table[pos_ids[t]]) ; rows of H bf16.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed_kernel(const bf16_t* __restrict__ table, const long* __restrict__ ids,
                                                    const bf16_t* __restrict__ ptable, const long* __restrict__ pids,
                                                    bf16_t* __restrict__ out, long T, int H) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nv = H / 8;
  if (gid >= T * nv) return;
  const long t = gid / nv;
  const int c = gid % nv;
  RT_ASSERT(ids[t] >= 0);
  uint4 v = *(const uint4*)(table + ids[t] * H + c * 8);
  if (ptable) {
    float a[8], b[8];
    unpack8(v, a);
    unpack8(*(const uint4*)(ptable + pids[t] * H + c * 8), b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += b[k];
    v = pack8(a);
  }
  *(uint4*)(out + t * H + c * 8) = v;
}

// ---------------------------------------------------------------------------------------------
// Varlen scatter: out[r] = inv[r] >= 0 ? src[inv[r]] : 0 for every row r of the [B*S] grid the
// attention kernels tile (inv = inverse of the packed row index). One pass writes the whole grid,
// pad rows included: replaces a zero fill + index_copy (two launches, the generic index_copy runs
// at ~1 TB/s). Rows of H bf16, 16 B per thread.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rows_scatter_kernel(const bf16_t* __restrict__ src, long lds,
                                                           const int* __restrict__ inv, bf16_t* __restrict__ out,
                                                           long R, int H, long N) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nv = H / 8;
  if (gid >= R * nv) return;
  const long r = gid / nv;
  const int c = gid % nv;
  const int j = inv[r];
  RT_ASSERT(j < N);
  uint4 v = make_uint4(0, 0, 0, 0);
  if (j >= 0) v = *(const uint4*)(src + (long)j * lds + c * 8);
  *(uint4*)(out + r * H + c * 8) = v;
}

}  // namespace rt

using namespace rt;

static inline unsigned nblocks(long total) { return (unsigned)((total + 255) / 256); }

extern "C" int rt_rows_scatter(const void* src, long lds, const int* inv, void* out, long R, int H, long N,
                               hipStream_t stream) {
  if (H % 8 != 0 || lds % 8 != 0) return -1;
  const long total = R * (H / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(rows_scatter_kernel, dim3(nblocks(total)), dim3(256), 0, stream, (const bf16_t*)src, lds, inv,
                     (bf16_t*)out, R, H, N);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_rope_qkv(void* qkv, long ld, const int* pos, const float* cosT, const float* sinT, int T, int S,
                           int Hq, int Hkv, int D, float sign, void* kc, void* vc, const int* slot_base, int Smax,
                           int do_rope_q, hipStream_t stream) {
  if (D % 16 != 0 || ld % 8 != 0) return -1;
  const long total = (long)T * (Hq + 2 * Hkv) * (D / 16);
  if (total == 0) return 0;
  hipLaunchKernelGGL(rope_qkv_kernel, dim3(nblocks(total)), dim3(256), 0, stream, (bf16_t*)qkv, ld, pos, cosT, sinT,
                     T, S, Hq, Hkv, D, sign, (bf16_t*)kc, (bf16_t*)vc, slot_base, Smax, do_rope_q);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_swiglu_fwd(const void* gu, void* y, long T, int F, hipStream_t stream) {
  if (F % 8 != 0) return -1;
  const long total = T * (F / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(nblocks(total)), dim3(256), 0, stream, (const bf16_t*)gu, (bf16_t*)y, T, F);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_swiglu_bwd(const void* gu, const void* dy, void* dgu, long T, int F, hipStream_t stream) {
  if (F % 8 != 0) return -1;
  const long total = T * (F / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(nblocks(total)), dim3(256), 0, stream, (const bf16_t*)gu,
                     (const bf16_t*)dy, (bf16_t*)dgu, T, F);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_embed(const void* table, const long* ids, const void* ptable, const long* pids, void* out, long T,
                        int H, hipStream_t stream) {
  if (H % 8 != 0) return -1;
  const long total = T * (H / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(embed_kernel, dim3(nblocks(total)), dim3(256), 0, stream, (const bf16_t*)table, ids,
                     (const bf16_t*)ptable, pids, (bf16_t*)out, T, H);
  RT_LAUNCH_CHECK();
  return 0;
}
