// Native host helpers for the IVF vector index: inverted-list construction by a
// parallel counting sort of coarse assignments, and k-means++ seeding. The heavy k-means
// iterations (GEMM + argmax + segment mean) and list scans run on the GPU; these pieces are
// branchy, sequential-by-nature host work kept out of Python loops.
#pragma once
#include <torch/extension.h>

namespace ragtl {
void bind_ivf_host(pybind11::module& m);
}
