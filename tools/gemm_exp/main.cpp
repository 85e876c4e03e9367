// Standalone timing harness for the token-parallel GEMM (gemm_big) and experimental variants of it.
// No torch: the kernel source (csrc/kernels/gemm_big.hip, or an experiment copy compiled with
// -DEXP_* switches, tools/gemm_exp/build.sh) is linked straight into this program, so a variant is
// one hipcc line and one run. Prints one line per shape: us per launch, PF/s, and a checksum of C
// (variants that skip waits produce wrong C on purpose; the checksum shows which ones are exact).
//
//   ./gemm_exp [reps] [ring | w4]   (ring: tuning gemm_ring = 1; w4: NT shapes on the 4-wave kernel)
#include <hip/hip_runtime.h>

#include "rt_tuning.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>

extern "C" int rt_gemm_big(int layout_a, int layout_b, const void* A, long lda, const void* B, long ldb,
                           const void* A2, long lda2, const void* B2, long ldb2, int K2, const void* bias,
                           void* C, long ldc, void* C2, long ldc2, const void* R, long ldr, int M, int N, int K,
                           int act, int out, int nsplit, const void* zpage, int bn, float* sk_part,
                           unsigned* sk_tickets, hipStream_t stream);

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ void fill_bf16(uint16_t* p, long n, uint32_t seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((int)(h & 0xFFFF) - 32768) * (1.f / 32768.f) * 0.05f;  // |x| < 0.05
    uint32_t u = __float_as_uint(f);
    p[i] = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
  }
}

__global__ void checksum(const uint16_t* c, long n, double* out) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += (double)__uint_as_float((uint32_t)c[i] << 16) * (double)((i % 7) + 1);
  atomicAdd(out, s);
}

struct Shape { const char* name; int la, lb, M, N, K, act, bn; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  // w4: the NT shapes on the 4-wave 128 x 128-per-wave kernel (bn = 4), NN skipped
  const bool w4 = argc > 2 && std::string(argv[2]) == "w4";
  if (argc > 2 && std::string(argv[2]) == "ring") {
    rt::Tuning t = *rt_tuning();
    t.gemm_ring = 1;
    rt_set_tuning(&t);
    printf("tuning: gemm_ring = 1\n");
  }
  const Shape shapes[] = {
      {"nt_1024tiles_8192x8192x4096", 0, 0, 8192, 8192, 4096, 0, 256},
      {"nt_qkv_9632x6144x4096", 0, 0, 9632, 6144, 4096, 0, 0},
      {"nt_gateup_swiglu_9632x28672x4096", 0, 0, 9632, 28672, 4096, 5, 0},
      {"nt_down_9632x4096x14336", 0, 0, 9632, 4096, 14336, 0, 0},
      {"nn_qkv_dx_9632x4096x6144", 0, 1, 9632, 4096, 6144, 0, 0},
  };
  long maxA = 0, maxB = 0, maxC = 0;
  for (const Shape& s : shapes) {
    maxA = std::max(maxA, (long)s.M * s.K);
    maxB = std::max(maxB, (long)s.N * s.K);
    maxC = std::max(maxC, (long)s.M * s.N);
  }
  uint16_t *A, *B, *C, *Z;
  double* cs;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxB * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&Z, 4096));
  CK(hipMalloc(&cs, sizeof(double)));
  CK(hipMemset(Z, 0, 4096));
  fill_bf16<<<4096, 256>>>(A, maxA, 17u);
  fill_bf16<<<4096, 256>>>(B, maxB, 91u);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (Shape s : shapes) {
    if (w4) {
      if (s.lb != 0) continue;
      s.bn = 4;
    }
    // NT: A [M, K], B [N, K]; NN: A [M, K] (= dY), B [K, N] (= W, KMAJ)
    const long lda = s.K, ldb = s.lb == 0 ? s.K : s.N;
    const int nout = s.act == 5 ? s.N / 2 : s.N;
    auto run = [&]() {
      const int rc = rt_gemm_big(s.la, s.lb, A, lda, B, ldb, nullptr, 0, nullptr, 0, 0, nullptr, C, nout, nullptr, 0,
                                 nullptr, 0, s.M, s.N, s.K, s.act, 0, 1, Z, s.bn, nullptr, nullptr, 0);
      if (rc) { fprintf(stderr, "rt_gemm_big rc=%d on %s\n", rc, s.name); exit(1); }
    };
    for (int i = 0; i < 3; ++i) run();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, 0));
      run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2] * 1e3;
    CK(hipMemset(cs, 0, sizeof(double)));
    checksum<<<1024, 256>>>(C, (long)s.M * nout, cs);
    double h = 0.0;
    CK(hipMemcpy(&h, cs, sizeof(double), hipMemcpyDeviceToHost));
    const double fl = 2.0 * s.M * (double)s.N * s.K;
    printf("%-36s med %8.1f us  min %8.1f us  %.3f PF/s  checksum %.6e\n", s.name, med, ts[0] * 1e3,
           fl / (med * 1e-6) / 1e15, h);
  }
  return 0;
}
