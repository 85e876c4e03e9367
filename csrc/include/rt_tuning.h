// Kernel-selection knobs of the native launchers, in ONE explicit struct.
//
// Every launch-path heuristic that has a measured alternative (A/B switches kept for the probes
// in tools/, forced split-K factors for tests) reads its value from here. The struct is process
// configuration, not a per-call channel: it is written only by rt_set_tuning (Python:
// ops.set_tuning / ops.tuning(...) context), never by a launcher, and per-call operands (split-K
// slabs, fp8 K/V scales, debug stamps) are ordinary launch arguments. Defaults are the measured
// best choices (docs/DESIGN.md); 0 in a "force" field means "use the heuristic".
#pragma once

namespace rt {

struct Tuning {
  // ---- decode attention (attention.hip) ----
  int decode_mw = 1;          // small-batch 8-wave MFMA kernel (0: VALU split kernel)
  int decode_mw_kpp = 512;    // keys per partition of the 8-wave kernel past 1024 cache slots
  int decode_mfma = 1;        // large-batch MFMA kernel (0: VALU kernel)
  int attn_kv_nt = 1;         // non-temporal K/V cache loads
  int decode_fp8_mw = 0;      // fp8 cache: the 8-wave kernel at every batch
  int decode_g1_valu = 1;     // fp8 cache, MHA at large batch: the VALU kernel
  int decode_g1_nw = 2;       // waves per row of that kernel (1, 2, 4)
  int decode_nk = 4;          // VALU split kernel: keys per lane per chunk (2, 4, 8)
  int attn_bwd_atomic_dq = 0; // attention backward: fp32-atomic dQ (round-1 form)
  int attn_fwd_w8 = 0;        // training / prefill attention forward: 8 waves x 16 query rows (else 4 x 32)
  // ---- norms (norm.hip) ----
  // threads per row of the split-K-slab norm (256, or 512 at H = 4096: 6.76 -> 6.56 us at batch 256,
  // profiles/r4/norm_slab_threads.log)
  int norm_slab_threads = 512;
  // ---- decode / skinny GEMMs (gemm_bf16.hip) ----
  int gemm_variant = 0;       // M > 64 library-shaped kernel: 0 auto, 1 128x128, 2 256x256, 4/5 fp8 forms
  int gemv16 = 2;             // 16-row no-split GEMV at M <= 16: 0 off, 1 narrow outputs, 2 all
  int gemv16_maxm = 16;       // rows handled by it (1..16)
  int gemv16_depth = 4;       // its weight-pipeline depth (4, 6, 8)
  int gemv16_waves = 0;       // waves per 16-row group: 0 auto (8 on grids <= 1 workgroup per CU, else 4), 4, 8, 16
  int decode_split = 0;       // force split-K of the M <= 16 decode kernel
  int decode_depth = 0;       // force weight-pipeline depth (2 / 4) of the M <= 16 decode kernel
  int m64_split = 0;          // force split-K of the 16 < M <= 64 ring kernel
  int wide_split = 0;         // force split-K of the wide W8A16 kernel
  int gemm_fp8_256 = 0;       // W8A8: the round-1 256x256 kernel instead of the gemm_big schedule
  // ---- token-parallel GEMMs (gemm_big.hip) ----
  int gemm_tr_builtin = 0;    // NN / TN transposed reads through the compiler builtin
  int gemm_b_nt = 0;          // non-temporal weight stream when one row tile covers M
  float gemm_bn128_cost = 0.55f;  // planner: time of a 256x128 tile / a 256x256 tile
  int gemm_group_m = 4;       // rows of 256x256 tiles per L2-reuse group in the tile order
  // stream-K tail for the partial last wave of 256x256 tiles: 0 off, 1 when the planner's cost
  // model prefers it, 2 always (tests). Off by default: measured SLOWER than the wave planner at the
  // update / reference shapes (M = 9632 qkv 422 vs 387 us, o 277 vs 260 us; the chip-wide burst of
  // partial-tile hand-offs at the end of the launch costs more than the tail it removes;
  // profiles/r4/gemm_streamk_vs_planner.log)
  int gemm_streamk = 0;
  // NT 256x256 tiles (no activation / SwiGLU / RoPE epilogue) on the 10-slot granule ring (160 KiB
  // LDS, granules issued ~2 K-steps ahead) instead of two K-step buffers
  int gemm_ring = 0;
};

}  // namespace rt

extern "C" const rt::Tuning* rt_tuning();
extern "C" void rt_set_tuning(const rt::Tuning* t);

namespace rt {
inline const Tuning& tuning() { return *rt_tuning(); }
}  // namespace rt
