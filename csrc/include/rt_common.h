// Common device helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
//
// Everything here is written for wave64: lane ids are threadIdx.x & 63, cross-lane
// reductions walk offsets 32..1, block sizes are multiples of 64.
#pragma once
#include "rt_tuning.h"
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define RT_WAVE 64

#define RT_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) return (int)_e;                                         \
  } while (0)

#define RT_LAUNCH_CHECK() RT_HIP_CHECK(hipGetLastError())

// Device-side bounds checks of the debug build (python -m rag_tl_domainllm_optimizer_amd._build
// --debug): a failed check prints the condition and traps the wave, which surfaces as
// a launch error on the next synchronisation instead of a silent out-of-bounds access.
#ifndef RAGTL_DEBUG
#define RAGTL_DEBUG 0
#endif
#define RT_ASSERT(cond)                                                                 \
  do {                                                                                  \
    if (RAGTL_DEBUG && !(cond)) {                                                       \
      printf("RT_ASSERT failed %s:%d: %s\n", __FILE__, __LINE__, #cond);               \
      __builtin_trap();                                                                 \
    }                                                                                   \
  } while (0)

namespace rt {

typedef uint16_t bf16_t;  // raw bf16 bits; storage type for every bf16 tensor

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;   // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;     // 16x16 accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16;   // 32x32 accumulator
typedef __attribute__((ext_vector_type(8))) uint16_t u16x8;
typedef __attribute__((ext_vector_type(4))) uint16_t u16x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// 16-B non-temporal load (global_load_dwordx4 ... nt): for data read once per launch (weights)
__device__ __forceinline__ uint4 load_nt16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 8-B non-temporal load (fp8 K/V cache rows: read once per decode step)
__device__ __forceinline__ uint2 load_nt8(const void* p) {
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
  const u32x2_t v = __builtin_nontemporal_load((const u32x2_t*)p);
  return make_uint2(v.x, v.y);
}

// ---- transposed LDS reads that do not drain LDS-DMA ----
// hipcc places `s_waitcnt vmcnt(0)` in front of every __builtin_amdgcn_ds_read_tr16_b64 while a
// global_load_lds is in flight (the intrinsic carries no alias information, so every pending
// LDS-DMA is assumed to write what it reads), which empties a kernel's prefetch pipeline at each
// transposed read. These helpers issue the reads in inline asm and end with their own
// `s_waitcnt lgkmcnt(0)`, so the outputs are complete at ASMEND (cdna_hip_programming.md §5.7:
// the compiler neither counts nor waits for asm memory operations). The caller orders them behind
// the LDS-DMA that filled the image (counted vmcnt, + barrier for other waves' DMA). EXEC must be
// all ones (ISA requirement of ds_read_b64_tr_b16).
typedef __attribute__((ext_vector_type(4))) short rt_s16x4;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// 4 reads at a + {0, O1, O2, O3} (byte offsets, compile-time)
template <int O1, int O2, int O3>
__device__ __forceinline__ void ds_tr16_x4(uint32_t a, rt_s16x4& r0, rt_s16x4& r1, rt_s16x4& r2, rt_s16x4& r3) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4\n\t"
      "ds_read_b64_tr_b16 %1, %4 offset:%5\n\t"
      "ds_read_b64_tr_b16 %2, %4 offset:%6\n\t"
      "ds_read_b64_tr_b16 %3, %4 offset:%7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(a), "i"(O1), "i"(O2), "i"(O3)
      : "memory");
}
// F fragments x 4 reads at a_f + {0, O1, O2, O3}: r[4 f + h]
template <int O1, int O2, int O3>
__device__ __forceinline__ void ds_tr16_frag2(uint32_t a0, uint32_t a1, rt_s16x4 (&r)[8]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\t"
      "ds_read_b64_tr_b16 %1, %8 offset:%10\n\t"
      "ds_read_b64_tr_b16 %2, %8 offset:%11\n\t"
      "ds_read_b64_tr_b16 %3, %8 offset:%12\n\t"
      "ds_read_b64_tr_b16 %4, %9\n\t"
      "ds_read_b64_tr_b16 %5, %9 offset:%10\n\t"
      "ds_read_b64_tr_b16 %6, %9 offset:%11\n\t"
      "ds_read_b64_tr_b16 %7, %9 offset:%12\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
      : "v"(a0), "v"(a1), "i"(O1), "i"(O2), "i"(O3)
      : "memory");
}
template <int O1, int O2, int O3>
__device__ __forceinline__ void ds_tr16_frag4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, rt_s16x4 (&r)[16]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %16\n\t"
      "ds_read_b64_tr_b16 %1, %16 offset:%20\n\t"
      "ds_read_b64_tr_b16 %2, %16 offset:%21\n\t"
      "ds_read_b64_tr_b16 %3, %16 offset:%22\n\t"
      "ds_read_b64_tr_b16 %4, %17\n\t"
      "ds_read_b64_tr_b16 %5, %17 offset:%20\n\t"
      "ds_read_b64_tr_b16 %6, %17 offset:%21\n\t"
      "ds_read_b64_tr_b16 %7, %17 offset:%22\n\t"
      "ds_read_b64_tr_b16 %8, %18\n\t"
      "ds_read_b64_tr_b16 %9, %18 offset:%20\n\t"
      "ds_read_b64_tr_b16 %10, %18 offset:%21\n\t"
      "ds_read_b64_tr_b16 %11, %18 offset:%22\n\t"
      "ds_read_b64_tr_b16 %12, %19\n\t"
      "ds_read_b64_tr_b16 %13, %19 offset:%20\n\t"
      "ds_read_b64_tr_b16 %14, %19 offset:%21\n\t"
      "ds_read_b64_tr_b16 %15, %19 offset:%22\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]),
        "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "i"(O1), "i"(O2), "i"(O3)
      : "memory");
}

// 8 plain 8-B LDS reads at a + {0, 512, ..., 3584} (the fp8 W fragments of the W8A16 LDS-DMA ring:
// 4 column fragments x 2 MFMA k-steps), issued from asm like the transposed reads above: hipcc
// otherwise drains every LDS-DMA in flight (s_waitcnt vmcnt(0)) in front of them
typedef __attribute__((ext_vector_type(2))) unsigned rt_u32x2;
__device__ __forceinline__ void ds_read_b64_x8_512(uint32_t a, rt_u32x2 (&r)[8]) {
  asm volatile(
      "ds_read_b64 %0, %8\n\t"
      "ds_read_b64 %1, %8 offset:512\n\t"
      "ds_read_b64 %2, %8 offset:1024\n\t"
      "ds_read_b64 %3, %8 offset:1536\n\t"
      "ds_read_b64 %4, %8 offset:2048\n\t"
      "ds_read_b64 %5, %8 offset:2560\n\t"
      "ds_read_b64 %6, %8 offset:3072\n\t"
      "ds_read_b64 %7, %8 offset:3584\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
      : "v"(a)
      : "memory");
}

// 4 plain 8-B LDS reads at a + {0, 512, 1024, 1536} (fp8 W fragments of the wide W8A16 kernel:
// 2 column fragments x 2 MFMA k-steps)
__device__ __forceinline__ void ds_read_b64_x4_512(uint32_t a, rt_u32x2 (&r)[4]) {
  asm volatile(
      "ds_read_b64 %0, %4\n\t"
      "ds_read_b64 %1, %4 offset:512\n\t"
      "ds_read_b64 %2, %4 offset:1024\n\t"
      "ds_read_b64 %3, %4 offset:1536\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(a)
      : "memory");
}

// 2 x (2 reads at a_i + {0, O1})
template <int O1>
__device__ __forceinline__ void ds_tr16_2x2(uint32_t a0, uint32_t a1, rt_s16x4& r0, rt_s16x4& r1, rt_s16x4& r2,
                                            rt_s16x4& r3) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4\n\t"
      "ds_read_b64_tr_b16 %1, %4 offset:%6\n\t"
      "ds_read_b64_tr_b16 %2, %5\n\t"
      "ds_read_b64_tr_b16 %3, %5 offset:%6\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(a0), "v"(a1), "i"(O1)
      : "memory");
}

// D = A.B + D on a 16x16x32 bf16 MFMA with D tied to AGPRs ("+a") and a "memory" clobber that pins
// surrounding loads / LDS-DMA issues to their source position (gemm_big.hip's 4-wave kernels).
// The x86 host pass parses kernel bodies too and has no AGPR constraint: the asm is device-pass only.
// PAD: lead with `s_nop 1`, the 2 wait states a VALU write of an A/B operand register needs before
// the MFMA reads it (cdna_hip_programming.md §5.7 item 2: hipcc pads nothing inside asm) — for
// call sites where hipcc may place a register copy of a fragment right in front of the MFMA.
typedef __attribute__((ext_vector_type(4))) int rt_i32x4;
template <bool PAD>
__device__ __forceinline__ void mfma_16x16x32_bf16_agpr(f32x4& d, const rt_i32x4& a, const rt_i32x4& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (PAD)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b) : "memory");
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b) : "memory");
#endif
}

// Scheduling fence for an AGPR accumulator: the compiler treats the value as redefined here, so
// reads of it cannot move above this point (it does not know the latency of an asm MFMA and would
// otherwise read a result that is still in flight) and its initialisation cannot sink below it.
__device__ __forceinline__ void agpr_fence(f32x4& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+a"(d));
#endif
}

__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(((uint32_t)x) << 16);
}

// Round-to-nearest-even f32 -> bf16 through the compiler's cast (lowers to
// v_cvt_pk_bf16_f32 on gfx950 and keeps NaN a NaN).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 16-byte vector of 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

// 8 OCP e4m3fn bytes (lo = bytes 0-3, hi = 4-7) -> 8 bf16 (exact: every e4m3fn value is a bf16)
__device__ __forceinline__ bf16x8 fp8x8_to_bf16(unsigned lo, unsigned hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.f, false);
  const bf16x2_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.f, true);
  const bf16x2_t c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.f, false);
  const bf16x2_t d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.f, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// 8 floats * inv -> 8 OCP e4m3fn bytes (round to nearest even; |x * inv| <= 448 by the caller's scale)
__device__ __forceinline__ uint2 f32x8_to_fp8(const float* v, float inv) {
  unsigned lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
  return make_uint2(lo, hi);
}

// Sum of `ns` fp32 split-K slabs of 8 consecutive floats (slab q at p + q * stride), added in
// slab order from slab 0 (bitwise equal to a rolled `for q` loop). The loads of the first 8 slabs
// are issued unconditionally (indices clamped to ns - 1, the surplus ones hit cache) before the
// first add: ONE L2/MALL round trip, where a rolled loop with a runtime trip count waits for every
// slab's loads in turn (docs/DESIGN.md 'A rolled reduction loop ... Unroll it').
__device__ __forceinline__ void sum_slabs8(const float* p, long stride, int ns, float (&out)[8]) {
  float4 lo[8], hi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float* sp = p + (long)min(q, ns - 1) * stride;
    lo[q] = *(const float4*)sp;
    hi[q] = *(const float4*)(sp + 4);
  }
  out[0] = lo[0].x; out[1] = lo[0].y; out[2] = lo[0].z; out[3] = lo[0].w;
  out[4] = hi[0].x; out[5] = hi[0].y; out[6] = hi[0].z; out[7] = hi[0].w;
#pragma unroll
  for (int q = 1; q < 8; ++q)
    if (q < ns) {
      out[0] += lo[q].x; out[1] += lo[q].y; out[2] += lo[q].z; out[3] += lo[q].w;
      out[4] += hi[q].x; out[5] += hi[q].y; out[6] += hi[q].z; out[7] += hi[q].w;
    }
  for (int q = 8; q < ns; ++q) {
    const float4 a = *(const float4*)(p + (long)q * stride), b = *(const float4*)(p + (long)q * stride + 4);
    out[0] += a.x; out[1] += a.y; out[2] += a.z; out[3] += a.w;
    out[4] += b.x; out[5] += b.y; out[6] += b.z; out[7] += b.w;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `sbuf` must hold blockDim.x/64 floats. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* sbuf) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sbuf[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += sbuf[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* sbuf) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) sbuf[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, sbuf[i]);
  return r;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, T1):
// blocks dealt round-robin over 8 XCDs are renumbered so each XCD gets a contiguous
// chunk of the tile grid (neighbouring tiles share operand panels in that XCD's L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// Philox4x32-10 counter-based RNG (graph-replay safe: state = (seed, offset) in memory).
struct Philox {
  __device__ static inline uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ static inline uint4 gen(uint64_t seed, uint64_t subseq, uint64_t offset) {
    uint4 c = make_uint4((uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)subseq,
                         (uint32_t)(subseq >> 32));
    uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

__device__ __forceinline__ float u32_to_unit(uint32_t x) {
  // uniform in (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

}  // namespace rt
