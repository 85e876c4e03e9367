// Standalone timing harness for the token-parallel GEMM (gemm_big) and experimental variants of it.
// No torch: the kernel source (csrc/kernels/gemm_big.hip, or an experiment copy compiled with
// -DEXP_* switches, tools/gemm_exp/build.sh) is linked straight into this program, so a variant is
// one hipcc line and one run. Prints one line per shape: us per launch, PF/s, and a checksum of C
// (variants that skip waits produce wrong C on purpose; the checksum shows which ones are exact).
//
//   ./gemm_exp [reps] [-] [cus,...]   (cus: run every shape again on a stream restricted to that many
//   CUs by a CU mask, spread evenly over the 256 mask bits)
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
                           int act, int out, int nsplit, const void* zpage, int bn, hipStream_t stream);

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ void fill_bf16(uint16_t* p, long n, uint32_t seed, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((int)(h & 0xFFFF) - 32768) * (1.f / 32768.f) * scale;  // uniform in (-scale, scale)
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
  std::vector<int> cus_list = {0};  // 0 = default stream (all CUs)
  if (argc > 3) {
    cus_list.clear();
    std::string a = argv[3];
    size_t pos = 0;
    while (pos < a.size()) {
      size_t q = a.find(',', pos);
      if (q == std::string::npos) q = a.size();
      cus_list.push_back(atoi(a.substr(pos, q - pos).c_str()));
      pos = q + 1;
    }
  }
  const Shape shapes[] = {
      {"nt_1024tiles_8192x8192x4096", 0, 0, 8192, 8192, 4096, 0, 256},
      {"nt_qkv_9632x6144x4096", 0, 0, 9632, 6144, 4096, 0, 0},
      {"nt_o_9632x4096x4096", 0, 0, 9632, 4096, 4096, 0, 0},
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
  // activations uniform in (-1, 1), weights in (-1/64, 1/64): the operand statistics of
  // tools/gemm_big_probe.py (the chip's clock under load depends on the operands' switching)
  fill_bf16<<<4096, 256>>>(A, maxA, 17u, 1.f);
  fill_bf16<<<4096, 256>>>(B, maxB, 91u, 1.f / 64.f);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int ncu : cus_list) {
  hipStream_t st = 0;
  if (ncu > 0 && ncu < 256) {
    uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < ncu; ++i) {
      const int b = (int)((long)i * 256 / ncu);  // evenly spread enabled bits
      mask[b >> 5] |= 1u << (b & 31);
    }
    CK(hipExtStreamCreateWithCUMask(&st, 8, mask));
  }
  printf("# cus %d\n", ncu > 0 ? ncu : 256);
  for (const Shape& s : shapes) {
    // NT: A [M, K], B [N, K]; NN: A [M, K] (= dY), B [K, N] (= W, KMAJ)
    const long lda = s.K, ldb = s.lb == 0 ? s.K : s.N;
    const int nout = s.act == 5 ? s.N / 2 : s.N;
    auto run = [&]() {
      const int rc = rt_gemm_big(s.la, s.lb, A, lda, B, ldb, nullptr, 0, nullptr, 0, 0, nullptr, C, nout, nullptr, 0,
                                 nullptr, 0, s.M, s.N, s.K, s.act, 0, 1, Z, s.bn, st);
      if (rc) { fprintf(stderr, "rt_gemm_big rc=%d on %s\n", rc, s.name); exit(1); }
    };
    for (int i = 0; i < 3; ++i) run();
    CK(hipStreamSynchronize(st));
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, st));
      run();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2] * 1e3;
    CK(hipStreamSynchronize(st));
    CK(hipMemset(cs, 0, sizeof(double)));
    checksum<<<1024, 256>>>(C, (long)s.M * nout, cs);
    double h = 0.0;
    CK(hipMemcpy(&h, cs, sizeof(double), hipMemcpyDeviceToHost));
    const double fl = 2.0 * s.M * (double)s.N * s.K;
    printf("%-36s med %8.1f us  min %8.1f us  %.3f PF/s  checksum %.6e\n", s.name, med, ts[0] * 1e3,
           fl / (med * 1e-6) / 1e15, h);
  }
  if (st) CK(hipStreamDestroy(st));
  }
  return 0;
}
