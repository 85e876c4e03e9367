// Batch-256 decode GEMMs on gemm_big (production 256x128 split-K / SwiGLU forms): row stride of the
// activations (lda) and of the weights (ldb) = K or K + 64 elements (8 KiB power-of-two strides vs
// padded ones), plus the linked rt_gemm_m256 variant (stream-isolation builds of gemm_m256ws.hip).
// Cold weights (4 copies, back-to-back), median of 7 runs of 40 launches.
//
//   ./gemm_m256_pad [M]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" int rt_gemm_big(int layout_a, int layout_b, const void* A, long lda, const void* B, long ldb,
                           const void* A2, long lda2, const void* B2, long ldb2, int K2, const void* bias,
                           void* C, long ldc, void* C2, long ldc2, const void* R, long ldr, int M, int N, int K,
                           int act, int out, int nsplit, const void* zpage, int bn, float* sk_part,
                           unsigned* sk_tickets, hipStream_t stream);
extern "C" int rt_gemm_m256(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int nsplit, int epi, hipStream_t stream);

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_bf16(uint16_t* p, long n, uint32_t seed, float amp) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((int)(h & 0xFFFF) - 32768) * (1.f / 32768.f) * amp;
    uint32_t u = __float_as_uint(f);
    p[i] = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
  }
}

struct Shape { const char* name; int N, K, split, swiglu; };

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 256;
  const Shape shapes[] = {{"qkv", 6144, 4096, 5, 0}, {"o", 4096, 4096, 8, 0}, {"down", 4096, 14336, 8, 0},
                          {"gate_up", 28672, 4096, 1, 1}};
  const long maxW = 28672L * (4096 + 64);
  uint16_t *A, *W, *Z;
  CK(hipMalloc(&A, 256L * (14336 + 64) * 2));
  CK(hipMalloc(&W, 4 * maxW * 2));
  CK(hipMalloc(&Z, 4096));
  CK(hipMemset(Z, 0, 4096));
  fill_bf16<<<4096, 256>>>(A, 256L * (14336 + 64), 17u, 1.f);
  for (int c = 0; c < 4; ++c) fill_bf16<<<4096, 256>>>(W + c * maxW, maxW, 91u + c, 1.f / 64);
  float* S0;
  CK(hipMalloc(&S0, 16L * 256 * 28672 * 4));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto fn) {
    for (int c = 0; c < 4; ++c) fn(c);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; ++it)
        for (int c = 0; c < 4; ++c) fn(c);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f / 40.f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[3];
  };
  for (const Shape& s : shapes) {
    const long ldc = s.swiglu ? s.N / 2 : s.N;
    printf("M=%d %-8s N=%5d K=%5d split %d:", M, s.name, s.N, s.K, s.split);
    for (int pa = 0; pa < 2; ++pa)
      for (int pb = 0; pb < 2; ++pb) {
        const long lda = s.K + 64 * pa, ldb = s.K + 64 * pb;
        auto prod = [&](int c) {
          const uint16_t* w = W + c * maxW;
          const int rc = rt_gemm_big(0, 0, A, lda, w, ldb, nullptr, 0, nullptr, 0, 0, nullptr, S0, ldc, nullptr, 0,
                                     nullptr, 0, M, s.N, s.K, s.swiglu ? 5 : 0, s.swiglu ? 0 : 3, s.split, Z, 128,
                                     nullptr, nullptr, 0);
          if (rc) { fprintf(stderr, "rt_gemm_big rc=%d (%s)\n", rc, s.name); exit(1); }
        };
        printf("  A%s B%s %6.1f", pa ? "+64" : "   ", pb ? "+64" : "   ", timeit(prod));
      }
    auto mine = [&](int c) {
      const int rc = rt_gemm_m256(A, s.K, W + c * maxW, s.K, S0, ldc, M, s.N, s.K, s.split, s.swiglu, 0);
      if (rc) { fprintf(stderr, "rt_gemm_m256 rc=%d (%s)\n", rc, s.name); exit(1); }
    };
    printf("  | variant %6.1f us\n", timeit(mine));
    fflush(stdout);
  }
  return 0;
}
