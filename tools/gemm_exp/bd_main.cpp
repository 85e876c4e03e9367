// Timing + exactness harness for tools/gemm_exp/gemm_bdirect.hip (B operand straight from a
// fragment-ordered weight image into VGPRs) against gemm_big (csrc/kernels/gemm_big.hip) on the
// Mistral-7B update shapes (M = 9632). Prints per shape: gemm_big (planner), gemm_big (256x256
// tiles only), bdirect, and the number of output elements that differ from gemm_big.
//   ./bd_exp [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

extern "C" int rt_gemm_big(int layout_a, int layout_b, const void* A, long lda, const void* B, long ldb,
                           const void* A2, long lda2, const void* B2, long ldb2, int K2, const void* bias,
                           void* C, long ldc, void* C2, long ldc2, const void* R, long ldr, int M, int N, int K,
                           int act, int out, int nsplit, const void* zpage, int bn, hipStream_t stream);
extern "C" int bd_gemm(const void* A, long lda, const void* Bimg, void* C, long ldc, int M, int N, int K,
                       hipStream_t st);
extern "C" int bd_shuffle(const void* W, long ldw, void* img, int N, int K, hipStream_t st);

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_bf16(uint16_t* p, long n, uint32_t seed, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((int)(h & 0xFFFF) - 32768) * (1.f / 32768.f) * scale;
    uint32_t u = __float_as_uint(f);
    p[i] = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
  }
}

__global__ void count_diff(const uint16_t* a, const uint16_t* b, long n, unsigned long long* out) {
  unsigned long long c = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) c += a[i] != b[i];
  atomicAdd(out, c);
}

struct Shape { const char* name; int M, N, K; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const Shape shapes[] = {
      {"qkv_9632x6144x4096", 9632, 6144, 4096},
      {"o_9632x4096x4096", 9632, 4096, 4096},
      {"gateup_9632x28672x4096", 9632, 28672, 4096},
      {"down_9632x4096x14336", 9632, 4096, 14336},
  };
  long maxA = 0, maxB = 0, maxC = 0;
  for (const Shape& s : shapes) {
    maxA = std::max(maxA, (long)s.M * s.K);
    maxB = std::max(maxB, (long)s.N * s.K);
    maxC = std::max(maxC, (long)s.M * s.N);
  }
  uint16_t *A, *B, *Bi, *C0, *C1, *Z;
  unsigned long long* dc;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxB * 2));
  CK(hipMalloc(&Bi, maxB * 2));
  CK(hipMalloc(&C0, maxC * 2));
  CK(hipMalloc(&C1, maxC * 2));
  CK(hipMalloc(&Z, 4096));
  CK(hipMalloc(&dc, 8));
  CK(hipMemset(Z, 0, 4096));
  fill_bf16<<<4096, 256>>>(A, maxA, 17u, 1.f);
  fill_bf16<<<4096, 256>>>(B, maxB, 91u, 1.f / 64.f);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto&& fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, 0));
      fn();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
  };
  for (const Shape& s : shapes) {
    CK(hipMemset(C0, 0, (long)s.M * s.N * 2));
    CK(hipMemset(C1, 0xFF, (long)s.M * s.N * 2));
    if (bd_shuffle(B, s.K, Bi, s.N, s.K, 0)) { fprintf(stderr, "bd_shuffle rc\n"); return 1; }
    auto gb = [&](int bn) {
      return [&, bn]() {
        if (rt_gemm_big(0, 0, A, s.K, B, s.K, nullptr, 0, nullptr, 0, 0, nullptr, C0, s.N, nullptr, 0, nullptr, 0, s.M,
                        s.N, s.K, 0, 0, 1, Z, bn, 0)) { fprintf(stderr, "rt_gemm_big rc\n"); exit(1); }
      };
    };
    auto bdr = [&]() {
      if (bd_gemm(A, s.K, Bi, C1, s.N, s.M, s.N, s.K, 0)) { fprintf(stderr, "bd_gemm rc\n"); exit(1); }
    };
    const float t_bd = timeit(bdr);
    const float t_256 = timeit(gb(256));
    const float t_plan = timeit(gb(0));
    CK(hipMemset(dc, 0, 8));
    count_diff<<<1024, 256>>>(C0, C1, (long)s.M * s.N, dc);
    unsigned long long nd = 0;
    CK(hipMemcpy(&nd, dc, 8, hipMemcpyDeviceToHost));
    const double fl = 2.0 * s.M * (double)s.N * s.K;
    printf("%-24s gemm_big %7.1f us (%.3f PF/s)  gemm_big bn256 %7.1f us  bdirect %7.1f us (%.3f PF/s)  diff %llu\n",
           s.name, t_plan, fl / t_plan * 1e-9, t_256, t_bd, fl / t_bd * 1e-9, nd);
    fflush(stdout);
  }
  return 0;
}
