// Phase timing of the batch-1 top-k sampler (tools/sampler_exp/make_variants.py builds copies of
// sampling.hip that stop after pass 1 / pass 2 / the k-th key search; use_window >= 100 arms the
// early exit): 100 launches captured in one hipGraph, replayed, GPU time per launch.
//   ./sampler_exp_<variant> [window 0|1] [scale]
#include <hip/hip_runtime.h>

#include "rt_tuning.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <random>
#include <vector>

extern "C" int rt_sample(const void* logits, int is_f32, long ld, long B, int V, float inv_temp, int top_k, float top_p,
                         int greedy, uint64_t seed, const int64_t* offset_ptr, const uint8_t* row_active, long* out_tok,
                         float* out_logp, hipStream_t stream);

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int win = argc > 1 ? atoi(argv[1]) : 1;
  const float scale = argc > 2 ? (float)atof(argv[2]) : 1.3f;
  const int V = 32000;
  std::vector<uint16_t> h(V);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, scale);
  for (int i = 0; i < V; ++i) {
    float f = nd(rng);
    uint32_t u;
    std::memcpy(&u, &f, 4);
    h[i] = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
  }
  void* d;
  long* tok;
  float* lp;
  int64_t* off;
  CK(hipMalloc(&d, V * 2));
  CK(hipMalloc(&tok, 8));
  CK(hipMalloc(&lp, 4));
  CK(hipMalloc(&off, 8));
  CK(hipMemcpy(d, h.data(), V * 2, hipMemcpyHostToDevice));
  CK(hipMemset(off, 0, 8));
  rt::Tuning t = *rt_tuning();
  t.sample_window = win;  // + 100 arms the early exit of the phase variants
  rt_set_tuning(&t);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto launch = [&]() {
    if (rt_sample(d, 0, V, 1, V, 1.f / 0.7f, 50, 0.9f, 0, 3, off, nullptr, tok, lp, st)) exit(2);
  };
  launch();
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 100; ++i) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  long ht = 0;
  CK(hipMemcpy(&ht, tok, 8, hipMemcpyDeviceToHost));
  printf("window=%d scale=%.2f: %.2f us per launch (token %ld)\n", win, scale, ms * 1e3f / 1000.f, ht);
  return 0;
}
