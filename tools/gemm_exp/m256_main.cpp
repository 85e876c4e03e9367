// Batch-256 decode GEMMs: gemm_m256_kernel (csrc/kernels/gemm_m256.hip, one section per K-step)
// vs the production form on gemm_big_kernel (256 x 128 tiles, four barrier-bracketed phases per
// K-step). Per shape: both results compared bitwise (fp32 slabs / bf16 SwiGLU output), then
// back-to-back launches over 4 weight copies (cold weights, as in a decode step), median of 7 runs.
//
//   ./gemm_m256_exp [M]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
  const long maxW = 28672L * 4096;
  uint16_t *A, *W, *Z;
  CK(hipMalloc(&A, 256L * 14336 * 2));
  CK(hipMalloc(&W, 4 * maxW * 2));
  CK(hipMalloc(&Z, 4096));
  CK(hipMemset(Z, 0, 4096));
  fill_bf16<<<4096, 256>>>(A, 256L * 14336, 17u, 1.f);
  for (int c = 0; c < 4; ++c) fill_bf16<<<4096, 256>>>(W + c * maxW, maxW, 91u + c, 1.f / 64);
  float *S0, *S1;
  const long slab = 16L * 256 * 28672;
  CK(hipMalloc(&S0, slab * 4));
  CK(hipMalloc(&S1, slab * 4));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    const long n_out = s.swiglu ? (long)M * (s.N / 2) : (long)s.split * M * s.N;
    const long ldc = s.swiglu ? s.N / 2 : s.N;
    auto prod = [&](int c, void* C) {
      const uint16_t* w = W + c * maxW;
      const int rc = s.swiglu ? rt_gemm_big(0, 0, A, s.K, w, s.K, nullptr, 0, nullptr, 0, 0, nullptr, C, ldc, nullptr, 0,
                                            nullptr, 0, M, s.N, s.K, 5, 0, 1, Z, 128, nullptr, nullptr, 0)
                              : rt_gemm_big(0, 0, A, s.K, w, s.K, nullptr, 0, nullptr, 0, 0, nullptr, C, ldc, nullptr, 0,
                                            nullptr, 0, M, s.N, s.K, 0, 3, s.split, Z, 128, nullptr, nullptr, 0);
      if (rc) { fprintf(stderr, "rt_gemm_big rc=%d (%s)\n", rc, s.name); exit(1); }
    };
    auto mine = [&](int c, void* C) {
      const int rc = rt_gemm_m256(A, s.K, W + c * maxW, s.K, C, ldc, M, s.N, s.K, s.split, s.swiglu, 0);
      if (rc) { fprintf(stderr, "rt_gemm_m256 rc=%d (%s)\n", rc, s.name); exit(1); }
    };
    // bitwise check on weight copy 0
    const size_t bytes = n_out * (s.swiglu ? 2 : 4);
    CK(hipMemset(S0, 0xFF, bytes));
    CK(hipMemset(S1, 0xEE, bytes));
    prod(0, S0);
    mine(0, S1);
    CK(hipDeviceSynchronize());
    std::vector<char> h0(bytes), h1(bytes);
    CK(hipMemcpy(h0.data(), S0, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), S1, bytes, hipMemcpyDeviceToHost));
    long diff = 0;
    const int es = s.swiglu ? 2 : 4;
    for (long i = 0; i < n_out; ++i) diff += memcmp(h0.data() + i * es, h1.data() + i * es, es) != 0;
    auto timeit = [&](auto fn) {
      for (int c = 0; c < 4; ++c) fn(c, S0);
      CK(hipDeviceSynchronize());
      std::vector<float> ts;
      for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < 10; ++it)
          for (int c = 0; c < 4; ++c) fn(c, S0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f / 40.f);
      }
      std::sort(ts.begin(), ts.end());
      return ts[3];
    };
    const float tp = timeit(prod), tm = timeit(mine), tp2 = timeit(prod), tm2 = timeit(mine);
    printf("M=%d %-8s N=%5d K=%5d split %d: gemm_big 256x128 %6.1f / %6.1f us | gemm_m256 %6.1f / %6.1f us | "
           "%ld of %ld outputs differ\n",
           M, s.name, s.N, s.K, s.split, tp, tp2, tm, tm2, diff, n_out);
    fflush(stdout);
  }
  return 0;
}
