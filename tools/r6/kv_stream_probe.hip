// Round-6 probe: is the batch-256 decode attention (attn_decode_mfma_kernel<4, 1>: 53 us per layer
// for ~248 MB of K/V = 4.7 TB/s) bound by its K/V access pattern or by its per-tile compute chain?
// Load-only kernels with the production pattern — one wave per (batch row, kv head), 16-key tiles,
// lane (g, r16) loading K[key r16][32 s + 8 g ..] (4 x 16 B) and V[key 4 i + g][8 r16 ..] (4 x 16 B),
// non-temporal, DEPTH tiles in flight — over the production cache layout [B, Hkv, Smax, D] (K and V
// in separate tensors), and the same over an interleaved layout [B, Hkv, Smax, 2, D] (a key's K and
// V rows adjacent: one 8-KiB contiguous run per tile). Context 173..300 keys (the decode steps of
// the headline rollout), Smax 456, B 256, Hkv 8, D 128, bf16.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/r6/kv_stream_probe.hip -o tools/r6/bin/kv_stream_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int D = 128, HKV = 8, B = 256, SMAX = 456;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const void* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

struct Tile { uint4 k[4]; uint4 v[4]; };

// INTER: 0 = separate K / V tensors, 1 = [.., Smax, 2, D]
template <int INTER, int DEPTH>
__global__ __launch_bounds__(64) void kv_load_kernel(const unsigned short* kc, const unsigned short* vc, int len,
                                                     unsigned* sink) {
  const int lane = threadIdx.x, g = lane >> 4, r16 = lane & 15;
  const int bh = blockIdx.x;
  const long kvrow = INTER ? 2 * D : D;  // elements per key slot of one tensor
  const unsigned short* kb = kc + (long)bh * SMAX * kvrow;
  const unsigned short* vb = INTER ? kb + D : vc + (long)bh * SMAX * D;
  auto load = [&](Tile& T, int c0) {
    const long key = min(c0 + r16, len - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) T.k[s] = ld_nt(kb + key * kvrow + 32 * s + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) T.v[i] = ld_nt(vb + (long)min(c0 + 4 * i + g, len - 1) * kvrow + 8 * r16);
  };
  unsigned acc = 0;
  auto consume = [&](const Tile& T) {
#pragma unroll
    for (int s = 0; s < 4; ++s) acc ^= T.k[s].x ^ T.k[s].w ^ T.v[s].y ^ T.v[s].z;
  };
  Tile t[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (16 * d < len) load(t[d], 16 * d);
  for (int c0 = 0; c0 < len; c0 += 16 * DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int c = c0 + 16 * d;
      if (c < len) {
        consume(t[d]);
        if (c + 16 * DEPTH < len) load(t[d], c + 16 * DEPTH);
      }
    }
  }
  if (acc == 0x12345678u) sink[bh * 64 + lane] = acc;
}

int main() {
  const long n = (long)B * HKV * SMAX * D;
  unsigned short *K, *V, *KV;
  unsigned* sink;
  CK(hipMalloc(&K, n * 2));
  CK(hipMalloc(&V, n * 2));
  CK(hipMalloc(&KV, 2 * n * 2));
  CK(hipMalloc(&sink, (long)B * HKV * 64 * 4));
  CK(hipMemset(K, 1, n * 2));
  CK(hipMemset(V, 2, n * 2));
  CK(hipMemset(KV, 3, 2 * n * 2));
  // a 1 GiB buffer swept between launches so every launch starts from cold caches
  char* junk;
  const long JB = 1L << 30;
  CK(hipMalloc(&junk, JB));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](auto kern, const char* name) {
    double tot_us = 0, tot_bytes = 0;
    for (int len = 173; len <= 300; len += 16) {
      std::vector<float> ts;
      for (int r = 0; r < 7; ++r) {
        CK(hipMemsetAsync(junk, r, JB, 0));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(B * HKV), dim3(64), 0, 0, K, V, len, sink);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f);
      }
      std::sort(ts.begin(), ts.end());
      const double bytes = (double)B * HKV * len * D * 2 * 2;
      tot_us += ts[3];
      tot_bytes += bytes;
    }
    printf("%-34s %7.1f us per launch (mean over len 173..300), %.2f TB/s\n", name, tot_us / 8, tot_bytes / tot_us * 1e-6);
    fflush(stdout);
  };
  auto run_i = [&](auto kern, const char* name) {
    double tot_us = 0, tot_bytes = 0;
    for (int len = 173; len <= 300; len += 16) {
      std::vector<float> ts;
      for (int r = 0; r < 7; ++r) {
        CK(hipMemsetAsync(junk, r, JB, 0));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(B * HKV), dim3(64), 0, 0, KV, (const unsigned short*)nullptr, len, sink);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f);
      }
      std::sort(ts.begin(), ts.end());
      const double bytes = (double)B * HKV * len * D * 2 * 2;
      tot_us += ts[3];
      tot_bytes += bytes;
    }
    printf("%-34s %7.1f us per launch (mean over len 173..300), %.2f TB/s\n", name, tot_us / 8, tot_bytes / tot_us * 1e-6);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run(kv_load_kernel<0, 2>, "separate K/V, 2 tiles in flight");
    run(kv_load_kernel<0, 3>, "separate K/V, 3 tiles in flight");
    run(kv_load_kernel<0, 4>, "separate K/V, 4 tiles in flight");
    run_i(kv_load_kernel<1, 2>, "interleaved K|V, 2 tiles in flight");
    run_i(kv_load_kernel<1, 4>, "interleaved K|V, 4 tiles in flight");
  }
  return 0;
}
