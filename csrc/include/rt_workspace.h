// Sizes of the per-(device, stream) split-K workspace shared by the skinny GEMM kernels and the
// bindings that allocate it. Launchers clamp their split-K so the partial slabs always fit.
#pragma once
constexpr long RT_SPLITK_SLAB_FLOATS = 1L << 24;  // fp32 partial slabs (64 MiB)
constexpr int RT_SPLITK_TICKETS = 1 << 16;        // one arrival counter per column group
