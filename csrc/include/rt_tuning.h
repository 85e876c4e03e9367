// Kernel-selection knobs of the native launchers, in ONE explicit struct.
//
// Every launch-path heuristic that has a live measured alternative (forced split-K factors and
// depths for tests, planner costs, A/B between kernels that are used elsewhere anyway) reads its
// value from here; alternatives measured slower and used nowhere else are not kept in the product
// kernels (docs/DESIGN.md "Round 5": tools/gemm_exp holds the experiment copies). The struct is process
// configuration, not a per-call channel: it is written only by rt_set_tuning (Python:
// ops.set_tuning / ops.tuning(...) context), never by a launcher, and per-call operands (split-K
// slabs, fp8 K/V scales, debug stamps) are ordinary launch arguments. Defaults are the measured
// best choices (docs/DESIGN.md); 0 in a "force" field means "use the heuristic".
#pragma once

namespace rt {

struct Tuning {
  // ---- decode attention (attention.hip) ----
  int decode_mw_bh = 320;     // (batch x kv heads) below which decode attention runs multi-wave workgroups:
                              // 8 waves per (row, kv head) below 256, 4 waves from 256 up to this bound
                              // (decode step at batch 32 4.35 -> 4.20 ms; at 48 / 64 / 96 the one-wave
                              // kernel is 2-9 % faster: profiles/r6/decode_attn_4wave_ab.log)
  int decode_mw_kpp = 512;    // keys per partition of the 8-wave small-batch kernel past decode_mw_smax cache slots
  int decode_mw_smax = 1024;  // cache slots up to which it runs one partition per kv head (fewer: measured slower
                              // at 456 slots, profiles/r5/decode_b1_deferred_partition_merge.log)
  // ---- training / prefill attention (attention.hip) ----
  int attn_fwd_hp_maxs = 1024;  // causal D = 128 forwards up to this many query positions use the head-packed
                                // 32-position tiles (GQA-4) or 64-position tiles of one head (other
                                // groupings); 0: always the 128-position tiles of one head
  int attn_dq_hp_maxs = 1024;   // causal GQA-4 backward dQ up to this many positions on head-packed 16-position
                                // workgroups (0: 64 positions of one head)
  int attn_lpt = 8192;          // causal forward / backward grids of at most this many workgroups dispatch their
                                // heaviest tiles first within each XCD (attention.hip attn_block_xyz); 0: tile order
  // ---- norms (norm.hip) ----
  // threads per row of the split-K-slab norm (256, or 512 at H = 4096: 6.76 -> 6.56 us at batch 256,
  // profiles/r4/norm_slab_threads.log)
  int norm_slab_threads = 512;
  // ---- decode / skinny GEMMs (gemm_bf16.hip) ----
  int gemm_variant = 0;       // W8A16 decode with fp8 images: 4 = no 16-row kernel at M <= 16, 5 = the
                              // 64-column ring instead of the 256-row wide kernel (A/B of live kernels)
  int gemv16 = 2;             // 16-row no-split GEMV at M <= 16: 0 off, 1 narrow outputs, 2 all
  int gemv16_maxm = 16;       // rows handled by it (1..16)
  int gemv16_depth = 4;       // its weight-pipeline depth (4, 6, 8)
  int gemv16_waves = 0;       // waves per 16-row group: 0 auto (8 on grids <= 1 workgroup per CU, else 4), 4, 8, 16
  int decode_split = 0;       // force split-K of the M <= 16 decode kernel
  int decode_depth = 0;       // force weight-pipeline depth (2 / 4) of the M <= 16 decode kernel
  int m64_split = 0;          // force split-K of the 16 < M <= 64 ring kernel
  int wide_split = 0;         // force split-K of the wide W8A16 kernel
  int m64_wide = 1;           // bf16 16 < M <= 64, N % 256 == 0, N <= 16384, no SwiGLU: 256 weight rows per workgroup
                              // (the wide kernel over row-major weights); 0: the 64-column ring gemm_m64_kernel
  // ---- token-parallel GEMMs (gemm_big.hip) ----
  float gemm_bn128_cost = 0.55f;  // planner: time of a 256x128 tile / a 256x256 tile
  int gemm_group_m = 4;       // rows of 256x256 tiles per L2-reuse group in the tile order
  // ---- sampler (sampling.hip) ----
  int sample_window = 1;      // top-k: candidates from a window below the row max, k-th key in one
                              // wave (0: 16 block-wide counting passes over the whole row; same draw)
  int sample_fast64 = 1;      // <= 64 survivors: sort / top-p / draw in wave 0's registers without a block
                              // barrier (0: the block-wide path; same draw)
};

}  // namespace rt

extern "C" const rt::Tuning* rt_tuning();
extern "C" void rt_set_tuning(const rt::Tuning* t);

namespace rt {
inline const Tuning& tuning() { return *rt_tuning(); }
}  // namespace rt
