// See ivf_host.h.
#include "ivf_host.h"

#include <algorithm>
#include <random>
#include <vector>

namespace ragtl {
namespace {

// assign [N] int64 (list id per vector) -> (offsets [nlist+1] int32, order [N] int64): order lists
// the vector indices grouped by list, stable within a list.
std::vector<at::Tensor> build_lists(const at::Tensor& assign_in, int64_t nlist) {
  TORCH_CHECK(assign_in.device().is_cpu(), "build_lists expects a CPU tensor");
  auto assign = assign_in.to(at::kLong).contiguous();
  const int64_t N = assign.numel();
  const int64_t* a = assign.data_ptr<int64_t>();
  auto offsets = at::zeros({nlist + 1}, at::kInt);
  auto order = at::empty({N}, at::kLong);
  int* off = offsets.data_ptr<int>();
  int64_t* ord = order.data_ptr<int64_t>();
  std::vector<int64_t> cnt(nlist, 0);
  for (int64_t i = 0; i < N; ++i) {
    TORCH_CHECK(a[i] >= 0 && a[i] < nlist, "build_lists: assignment out of range");
    ++cnt[a[i]];
  }
  off[0] = 0;
  for (int64_t l = 0; l < nlist; ++l) off[l + 1] = off[l] + (int)cnt[l];
  std::vector<int64_t> cur(off, off + nlist);
  for (int64_t i = 0; i < N; ++i) ord[cur[a[i]]++] = i;
  return {offsets, order};
}

// k-means++ seeding on (a sample of) float32 vectors [N, d]; returns k row indices.
at::Tensor kmeanspp(const at::Tensor& x_in, int64_t k, int64_t seed) {
  TORCH_CHECK(x_in.device().is_cpu(), "kmeanspp expects a CPU tensor");
  auto x = x_in.to(at::kFloat).contiguous();
  const int64_t N = x.size(0), d = x.size(1);
  TORCH_CHECK(k <= N, "kmeanspp: k > N");
  const float* X = x.data_ptr<float>();
  std::mt19937_64 rng((uint64_t)seed);
  std::vector<double> dist(N, std::numeric_limits<double>::infinity());
  auto out = at::empty({k}, at::kLong);
  int64_t* o = out.data_ptr<int64_t>();
  o[0] = (int64_t)(rng() % (uint64_t)N);
  for (int64_t c = 1; c < k; ++c) {
    const float* cv = X + o[c - 1] * d;
    double tot = 0.0;
    at::parallel_for(0, N, 2048, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        const float* xi = X + i * d;
        double s = 0.0;
        for (int64_t j = 0; j < d; ++j) { const double t = (double)xi[j] - cv[j]; s += t * t; }
        if (s < dist[i]) dist[i] = s;
      }
    });
    for (int64_t i = 0; i < N; ++i) tot += dist[i];
    std::uniform_real_distribution<double> U(0.0, tot);
    double r = U(rng), acc = 0.0;
    int64_t pick = N - 1;
    for (int64_t i = 0; i < N; ++i) {
      acc += dist[i];
      if (acc >= r) { pick = i; break; }
    }
    o[c] = pick;
  }
  return out;
}

}  // namespace

void bind_ivf_host(pybind11::module& m) {
  m.def("ivf_build_lists", &build_lists, "counting-sort inverted lists from coarse assignments");
  m.def("kmeanspp_init", &kmeanspp, "k-means++ seeding (host)");
}

}  // namespace ragtl
