// Python bindings of the gfx950 kernel library (module `_C` of the framework package).
//
// Thin, checked wrappers: validate device/dtype/shape/alignment, allocate outputs, launch on the
// current HIP stream. The kernels themselves live in csrc/kernels/*.hip and are built with
// hipcc --offload-arch=gfx950; this translation unit is host-only C++ against libtorch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "host/tokenizer.h"
#include "host/ivf_host.h"
#include "rt_workspace.h"
#include "rt_tuning.h"

extern "C" {
int rt_gemm_nt(const void*, long, const void*, long, const void*, long, const void*, long, int, const void*, void*,
               long, int, int, int, int, int, float*, unsigned*, const void*, long, float, int, hipStream_t);
int rt_shuffle_decode_weight(const void*, void*, long, long, hipStream_t);
int rt_shuffle_decode_weight_fp8(const void*, void*, long, long, hipStream_t);
int rt_gemm_big(int, int, const void*, long, const void*, long, const void*, long, const void*, long, int,
                const void*, void*, long, void*, long, const void*, long, int, int, int, int, int, int, const void*,
                int, hipStream_t);
int rt_gemm_small(int, int, const void*, long, const void*, long, void*, long, int, int, int, int, int, const void*,
                  int, hipStream_t);
int rt_gemm_big_rope(const void*, long, const void*, long, const void*, long, const void*, long, int, const void*,
                     void*, long, int, int, int, const int*, const float*, const float*, int, int, const void*, int,
                     hipStream_t);
int rt_gemm_splitk_reduce(const float*, int, int, int, const void*, int, const void*, long, void*, long, hipStream_t);
int rt_gemm_big_fp8_slabs(const void*, long, const float*, const void*, long, const float*, float*, int, int, int, int,
                          int, hipStream_t);
int rt_gemm_big_fp8(const void*, long, const float*, const void*, long, const float*, const void*, void*, long, int,
                    int, int, int, const void*, long, const void*, long, int, void*, long, const void*, hipStream_t);
int rt_gemm_fp8(const void*, long, const float*, const void*, long, const float*, const void*, void*, long, int, int,
                int, int, int, float*, unsigned*, const void*, long, float, int, hipStream_t);
int rt_quant_fp8_rows(const void*, long, void*, long, float*, long, int, hipStream_t);
int rt_norm_fwd(int, const void*, const void*, const void*, const void*, void*, void*, float*, float*, int, int, float,
                const float*, int, hipStream_t);
int rt_norm_bwd(int, const void*, const void*, const void*, const float*, const float*, const void*, void*, float*,
                float*, int, int, hipStream_t);
int rt_norm_bwd_blocks(int);
int rt_rope_qkv(void*, long, const int*, const float*, const float*, int, int, int, int, int, float, void*, void*,
                const int*, int, int, hipStream_t);
int rt_swiglu_fwd(const void*, void*, long, int, hipStream_t);
int rt_swiglu_bwd(const void*, const void*, void*, long, int, hipStream_t);
int rt_embed(const void*, const long*, const void*, const long*, void*, long, int, hipStream_t);
int rt_rows_scatter(const void*, long, const int*, void*, long, int, long, hipStream_t);
int rt_attn_fwd(const void*, long, const void*, long, const void*, long, void*, long, float*, const int*, const int*,
                const float*, int, int, int, int, int, int, int, int, int, float, hipStream_t);
int rt_attn_decode(const void*, long, const void*, const void*, int, const int*, const int*, int, float*, int, int,
                   void*, long, int, int, int, int, float, hipStream_t);
int rt_attn_decode_fused(const void*, long, void*, void*, int, const int*, const int*, const int*, const int*,
                         const float*, const float*, float, int, float*, unsigned*, int, int, void*, long, int, int, int,
                         int, float, const float*, int, float*, float*, int, long long*, hipStream_t);
int rt_attn_decode_fused_ps(int, int);
int rt_kv_store_fp8(const void*, long, void*, void*, float*, float*, int, int, int, int, int, int, int, hipStream_t);
int rt_attn_decode_mfma_ok(int, int, int, int, int);
int rt_attn_bwd(const void*, long, const void*, long, const void*, long, const void*, long, const void*, long,
                const float*, float*, float*, void*, long, void*, long, void*, long, const int*, int, int, int, int,
                int, int, int, float, const int*, const float*, const float*, hipStream_t);
int rt_logprob_fwd(const void*, int, long, const long*, float, long, int, float*, float*, float*, float*, hipStream_t);
int rt_logprob_bwd(const void*, int, long, const long*, float, long, int, const float*, const float*, const float*,
                   const float*, void*, long, hipStream_t);
int rt_sample(const void*, int, long, long, int, float, int, float, int, uint64_t, const int64_t*, const uint8_t*, long*,
              float*, hipStream_t);
int rt_grad_sumsq(const float*, long, float*, int, hipStream_t);
int rt_adamw(float*, const float*, float*, float*, void*, long, float, float, float, float, float, int, float,
             const float*, int, float*, int*, hipStream_t);
int rt_grad_sumsq_mixed(const void*, long, const float*, long, float*, int, hipStream_t);
int rt_adamw_mixed(float*, const void*, long, const float*, float*, float*, void*, long, float, float, float, float,
                   float, int, float, const float*, int, float*, int*, hipStream_t);
int rt_pool_norm(const void*, const int*, int, int, int, int, float*, hipStream_t);
int rt_scatter_scaled(const long*, int, long, hipStream_t);
int rt_lora_grad_accum(const long*, int, long, hipStream_t);
int rt_topk(const float*, long, long, int, int, const long*, long, float*, long*, hipStream_t);
int rt_segment_mean(const float*, int, const long*, const int*, int, int, float*, hipStream_t);
int rt_ivf_scan(const void*, int, int, const int*, int, const int*, const int*, const void*, const long*, const float*,
                int, int, float*, long*,
                hipStream_t);
int rt_gae(const float*, const float*, const float*, int, int, float, float, float*, float*, hipStream_t);
int rt_ppo_advantages(const float*, const float*, const float*, const float*, const int*, int, int, float, float, float,
                      int, float, float*, float*, float*, float*, hipStream_t);
int rt_ppo_loss(const float*, const float*, const float*, const float*, const float*, const float*, const float*,
                const float*, long, float, float, float, float, const float*, float, float*, float*, float*, float*,
                hipStream_t);
int rt_rowdot(const void*, long, const float*, const float*, int, long, float*, hipStream_t);
int rt_decode_update(const long*, long*, int, float*, const float*, float*, const float*, uint8_t*, int*, int*, long*,
                     int*, int64_t*, int64_t*, int, const long*, int, long, int*, const int*, hipStream_t);
}

namespace {

using at::Tensor;
using c10::optional;

// ---- rt::Tuning <-> dict (csrc/include/rt_tuning.h) ----
struct TuningField {
  const char* name;
  int rt::Tuning::*i;
  float rt::Tuning::*f;
};
static const TuningField kTuningFields[] = {
    {"decode_mw_bh", &rt::Tuning::decode_mw_bh, nullptr},
    {"attn_lpt", &rt::Tuning::attn_lpt, nullptr},
    {"decode_mw_kpp", &rt::Tuning::decode_mw_kpp, nullptr},
    {"decode_mw_smax", &rt::Tuning::decode_mw_smax, nullptr},
    {"attn_fwd_hp_maxs", &rt::Tuning::attn_fwd_hp_maxs, nullptr},
    {"attn_dq_hp_maxs", &rt::Tuning::attn_dq_hp_maxs, nullptr},
    {"norm_slab_threads", &rt::Tuning::norm_slab_threads, nullptr},
    {"gemm_variant", &rt::Tuning::gemm_variant, nullptr},
    {"gemv16", &rt::Tuning::gemv16, nullptr},
    {"gemv16_maxm", &rt::Tuning::gemv16_maxm, nullptr},
    {"gemv16_depth", &rt::Tuning::gemv16_depth, nullptr},
    {"gemv16_waves", &rt::Tuning::gemv16_waves, nullptr},
    {"decode_split", &rt::Tuning::decode_split, nullptr},
    {"decode_depth", &rt::Tuning::decode_depth, nullptr},
    {"m64_split", &rt::Tuning::m64_split, nullptr},
    {"wide_split", &rt::Tuning::wide_split, nullptr},
    {"m64_wide", &rt::Tuning::m64_wide, nullptr},
    {"gemm_bn128_cost", nullptr, &rt::Tuning::gemm_bn128_cost},
    {"gemm_group_m", &rt::Tuning::gemm_group_m, nullptr},
    {"sample_window", &rt::Tuning::sample_window, nullptr},
    {"sample_fast64", &rt::Tuning::sample_fast64, nullptr},
};

py::dict get_tuning() {
  py::dict d;
  const rt::Tuning& t = rt::tuning();
  for (const auto& f : kTuningFields) {
    if (f.i) d[f.name] = t.*(f.i);
    else d[f.name] = t.*(f.f);
  }
  return d;
}

void set_tuning(const py::dict& d) {
  rt::Tuning t = rt::tuning();
  for (auto kv : d) {
    const std::string k = py::str(kv.first);
    bool found = false;
    for (const auto& f : kTuningFields) {
      if (k == f.name) {
        if (f.i) t.*(f.i) = kv.second.cast<int>();
        else t.*(f.f) = kv.second.cast<float>();
        found = true;
        break;
      }
    }
    TORCH_CHECK(found, "set_tuning: unknown field '", k, "'");
  }
  rt_set_tuning(&t);
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " launch failed (code ", rc, ")");
}

#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_I64(t) TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")
#define CHECK_ROWS(t) TORCH_CHECK((t).dim() == 2 && (t).stride(1) == 1, #t " must be 2-D with unit column stride")
#define CHECK_ALIGN16(t)                                                                             \
  TORCH_CHECK(reinterpret_cast<uintptr_t>((t).data_ptr()) % 16 == 0, #t " must be 16-byte aligned")

const void* opt_ptr(const optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }

// Split-K workspace of the decode GEMM (fp32 slabs + self-resetting arrival tickets), one per
// (device, stream) so GEMMs on concurrent streams never share tickets. Allocated on first use
// (eager warm-up precedes graph capture); intentionally never freed.
struct DecodeWS {
  Tensor slabs, tickets;
};
static std::mutex g_ws_mu;
static std::unordered_map<uint64_t, DecodeWS*>* g_ws_map = new std::unordered_map<uint64_t, DecodeWS*>();
std::vector<Tensor> decode_ws_all() {
  std::lock_guard<std::mutex> g(g_ws_mu);
  std::vector<Tensor> v;
  for (auto& kv : *g_ws_map) v.push_back(kv.second->tickets);
  return v;
}
DecodeWS& decode_ws(const Tensor& like, hipStream_t st) {
  auto& mu = g_ws_mu;
  auto* map = g_ws_map;
  std::lock_guard<std::mutex> g(mu);
  const uint64_t key = (uint64_t)like.get_device() << 56 ^ (uint64_t)(uintptr_t)st;
  auto it = map->find(key);
  if (it != map->end()) return *it->second;
  auto* w = new DecodeWS();
  w->slabs = at::empty({RT_SPLITK_SLAB_FLOATS}, like.options().dtype(at::kFloat));
  w->tickets = at::zeros({RT_SPLITK_TICKETS}, like.options().dtype(at::kInt));
  (*map)[key] = w;
  return *w;
}

// diagnostics: per decode workspace, the number of arrival tickets not back at zero (every
// split-K launch leaves them at zero; a non-zero count means two launches raced on one workspace)
std::vector<int64_t> decode_ws_dirty_tickets() {
  std::vector<int64_t> out;
  for (auto& t : decode_ws_all()) out.push_back((t.ne(0)).sum().item<int64_t>());
  return out;
}

// ---------------------------------------------------------------------------------------------
Tensor gemm(const Tensor& a, const Tensor& w, const optional<Tensor>& u, const optional<Tensor>& ub,
            const optional<Tensor>& bias, int64_t act, bool out_f32, optional<Tensor> out,
            const optional<Tensor>& residual, double norm_eps, bool w_shuffled) {
  CHECK_CUDA(a); CHECK_CUDA(w); CHECK_BF16(a); CHECK_BF16(w); CHECK_ROWS(a); CHECK_ROWS(w);
  if (w_shuffled)
    TORCH_CHECK(a.size(0) <= 64 && w.size(0) % 16 == 0 && w.is_contiguous(),
                "gemm: a shuffled decode weight needs M <= 64, N % 16 == 0 and a contiguous image");
  CHECK_ALIGN16(a); CHECK_ALIGN16(w);
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm: K mismatch ", w.size(1), " vs ", K);
  TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64, got ", K);
  TORCH_CHECK(N % 8 == 0, "gemm: N must be a multiple of 8, got ", N);
  TORCH_CHECK(a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm: row strides must be multiples of 8");
  int Rp = 0;
  if (u.has_value() && u->defined()) {
    TORCH_CHECK(ub.has_value() && ub->defined(), "gemm: LoRA U given without UB");
    CHECK_BF16(*u); CHECK_BF16(*ub); CHECK_ROWS(*u); CHECK_ROWS(*ub); CHECK_ALIGN16(*u); CHECK_ALIGN16(*ub);
    TORCH_CHECK(u->size(0) == M && ub->size(0) == N && u->size(1) == ub->size(1), "gemm: LoRA shape mismatch");
    Rp = (int)u->size(1);
    TORCH_CHECK(Rp % 64 == 0, "gemm: LoRA rank must be padded to a multiple of 64");
    TORCH_CHECK(u->stride(0) % 8 == 0 && ub->stride(0) % 8 == 0, "gemm: LoRA row strides must be multiples of 8");
  }
  if (bias.has_value() && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N && bias->is_contiguous()); }
  // act 5 = SwiGLU pair mode: w = [gate; up] (2F rows), output [M, F] (skinny kernels, M <= 64)
  const bool pair = act == 5;
  if (pair) TORCH_CHECK(M <= 64 && N % 64 == 0 && Rp == 0, "gemm: SwiGLU pair mode needs M <= 64, N % 64 == 0, no LoRA");
  const int64_t Nout = pair ? N / 2 : N;
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.size(0) == M && c.size(1) == Nout && c.stride(1) == 1, "gemm: bad out shape");
    TORCH_CHECK(c.scalar_type() == (out_f32 ? at::kFloat : at::kBFloat16), "gemm: bad out dtype");
    TORCH_CHECK(c.stride(0) % 8 == 0, "gemm: out row stride must be a multiple of 8");
    CHECK_ALIGN16(c);
  } else {
    c = at::empty({M, Nout}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  if (M == 0) return c;
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res || norm_eps > 0) {
    TORCH_CHECK(M <= 64, "gemm: residual / in-GEMM norm are decode (M <= 64) features");
    if (has_res) {
      CHECK_BF16(*residual);
      TORCH_CHECK(residual->size(0) == M && residual->size(1) == Nout && residual->stride(1) == 1, "gemm: residual shape");
    }
  }
  hipStream_t st = cur_stream();
  float* slabs = nullptr;
  unsigned* tickets = nullptr;
  if (M <= 64) {
    DecodeWS& ws = decode_ws(a, st);
    slabs = ws.slabs.data_ptr<float>();
    tickets = (unsigned*)ws.tickets.data_ptr<int>();
    TORCH_CHECK((N + 63) / 64 <= ws.tickets.numel(), "gemm: N too large for the decode workspace");
  }
  check_rc(rt_gemm_nt(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), opt_ptr(u), Rp ? u->stride(0) : 0,
                      opt_ptr(ub), Rp ? ub->stride(0) : 0, Rp, opt_ptr(bias), c.data_ptr(), c.stride(0), (int)M,
                      (int)N, (int)K, (int)act, out_f32 ? 1 : 0, slabs, tickets,
                      has_res ? residual->data_ptr() : nullptr, has_res ? residual->stride(0) : 0, (float)norm_eps,
                      w_shuffled ? 1 : 0, st),
           "gemm");
  return c;
}

// W [N, K] -> the decode kernel's tile-ordered image (same shape, permuted content; gemm(...,
// w_shuffled=True) reads it). Written into `out` when given (in-place refresh of a captured buffer).
Tensor shuffle_decode_weight(const Tensor& w, optional<Tensor> out) {
  CHECK_CUDA(w); CHECK_BF16(w);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "shuffle_decode_weight: contiguous [N, K] weight expected");
  const int64_t N = w.size(0), K = w.size(1);
  TORCH_CHECK(N % 16 == 0 && K % 64 == 0, "shuffle_decode_weight: needs N % 16 == 0 and K % 64 == 0");
  Tensor o = (out.has_value() && out->defined()) ? *out : at::empty_like(w);
  TORCH_CHECK(o.sizes() == w.sizes() && o.is_contiguous() && o.scalar_type() == w.scalar_type(), "shuffle_decode_weight: bad out");
  TORCH_CHECK(o.data_ptr() != w.data_ptr(), "shuffle_decode_weight: out must not alias w");
  check_rc(rt_shuffle_decode_weight(w.data_ptr(), o.data_ptr(), N, K, cur_stream()), "shuffle_decode_weight");
  return o;
}

// q [N, K] e4m3fn bytes -> the fp8 tile-ordered image of gemv16_kernel<W8> (same shape, permuted).
Tensor shuffle_decode_weight_fp8(const Tensor& q, optional<Tensor> out) {
  CHECK_CUDA(q);
  TORCH_CHECK(q.scalar_type() == at::kByte && q.dim() == 2 && q.is_contiguous(),
              "shuffle_decode_weight_fp8: contiguous uint8 [N, K] expected");
  const int64_t N = q.size(0), K = q.size(1);
  TORCH_CHECK(N % 16 == 0 && K % 128 == 0, "shuffle_decode_weight_fp8: needs N % 16 == 0 and K % 128 == 0");
  Tensor o = (out.has_value() && out->defined()) ? *out : at::empty_like(q);
  TORCH_CHECK(o.sizes() == q.sizes() && o.is_contiguous() && o.scalar_type() == at::kByte,
              "shuffle_decode_weight_fp8: bad out");
  TORCH_CHECK(o.data_ptr() != q.data_ptr(), "shuffle_decode_weight_fp8: out must not alias q");
  check_rc(rt_shuffle_decode_weight_fp8(q.data_ptr(), o.data_ptr(), N, K, cur_stream()), "shuffle_decode_weight_fp8");
  return o;
}

// ---------------------------------------------------------------------------------------------
// Token-parallel GEMM family (csrc/kernels/gemm_big.hip). 2-D operands with unit column stride:
//   layout_a 0: a = [M, K]   1: a = [K, M]        layout_b 0: b = [N, K]   1: b = [K, N]
// a2 / b2: K-extension (LoRA) in the same layouts with their own reduction length K2.
// out_mode 0: bf16 (bias + act epilogue; act 5 = SwiGLU: b = [gate; up] (2F rows), C = [M, F],
// out2 = optional [M, 2F] pre-activation), 1: fp32, 2: fp32 atomic accumulate into `out`
// (split-K `nsplit`; `out` must be given and initialised).
const Tensor& zero_page(const Tensor& like) {
  static std::mutex mu;
  static auto* map = new std::unordered_map<int, Tensor>();
  std::lock_guard<std::mutex> g(mu);
  auto it = map->find(like.get_device());
  if (it != map->end()) return it->second;
  (*map)[like.get_device()] = at::zeros({2048}, like.options().dtype(at::kBFloat16));
  return (*map)[like.get_device()];
}

Tensor gemm_big(const Tensor& a, const Tensor& b, int64_t layout_a, int64_t layout_b, const optional<Tensor>& a2,
                const optional<Tensor>& b2, const optional<Tensor>& bias, int64_t act, int64_t out_mode,
                int64_t nsplit, optional<Tensor> out, const optional<Tensor>& out2, const optional<Tensor>& residual,
                int64_t bn) {
  CHECK_CUDA(a); CHECK_CUDA(b); CHECK_BF16(a); CHECK_BF16(b); CHECK_ROWS(a); CHECK_ROWS(b);
  CHECK_ALIGN16(a); CHECK_ALIGN16(b);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_big: row strides must be multiples of 8");
  const int64_t M = layout_a ? a.size(1) : a.size(0), K = layout_a ? a.size(0) : a.size(1);
  const int64_t N = layout_b ? b.size(1) : b.size(0), Kb = layout_b ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm_big: K mismatch ", K, " vs ", Kb);
  TORCH_CHECK((layout_a && layout_b) || K % 8 == 0, "gemm_big: K must be a multiple of 8 (a K-contiguous operand)");
  TORCH_CHECK(!layout_a || M % 8 == 0, "gemm_big: [K, M] operand needs M % 8 == 0");
  TORCH_CHECK(!layout_b || N % 8 == 0, "gemm_big: [K, N] operand needs N % 8 == 0");
  int64_t K2 = 0;
  const bool ext = a2.has_value() && a2->defined();
  if (ext) {
    TORCH_CHECK(b2.has_value() && b2->defined(), "gemm_big: a2 without b2");
    CHECK_BF16(*a2); CHECK_BF16(*b2); CHECK_ROWS(*a2); CHECK_ROWS(*b2); CHECK_ALIGN16(*a2); CHECK_ALIGN16(*b2);
    TORCH_CHECK(a2->stride(0) % 8 == 0 && b2->stride(0) % 8 == 0, "gemm_big: extension row strides % 8");
    K2 = layout_a ? a2->size(0) : a2->size(1);
    const int64_t M2 = layout_a ? a2->size(1) : a2->size(0);
    const int64_t N2 = layout_b ? b2->size(1) : b2->size(0), K2b = layout_b ? b2->size(0) : b2->size(1);
    TORCH_CHECK(M2 == M && N2 == N && K2b == K2, "gemm_big: extension shape mismatch");
    TORCH_CHECK((layout_a && layout_b) || K2 % 8 == 0, "gemm_big: K2 must be a multiple of 8");
  }
  const bool swiglu = act == 5;
  // act 6: SwiGLU backward in the epilogue of the down projection's dX (NN): out = d[gate | up]
  // [M, 2N] from residual = the forward's [gate | up] pre-activation [M, 2N]
  const bool dswiglu = act == 6;
  if (dswiglu) {
    TORCH_CHECK(layout_a == 0 && layout_b == 1 && out_mode == 0 && nsplit <= 1, "gemm_big: act 6 is NN, bf16, no split");
    TORCH_CHECK(out.has_value() && out->defined() && residual.has_value() && residual->defined(),
                "gemm_big: act 6 needs out and residual = [gate | up] pre-activation");
    const Tensor* both[2] = {&out.value(), &residual.value()};
    for (const Tensor* t : both) {
      CHECK_BF16(*t); CHECK_ALIGN16(*t);
      TORCH_CHECK(t->dim() == 2 && t->size(0) == M && t->size(1) == 2 * N && t->stride(1) == 1 && t->stride(0) % 8 == 0,
                  "gemm_big: act 6 out / residual must be bf16 [M, 2N]");
    }
    TORCH_CHECK(N % 8 == 0 && !(bias.has_value() && bias->defined()), "gemm_big: act 6 needs N % 8 == 0, no bias");
    if (M == 0 || N == 0) return *out;
    check_rc(rt_gemm_big(0, 1, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), ext ? a2->data_ptr() : nullptr,
                         ext ? a2->stride(0) : 0, ext ? b2->data_ptr() : nullptr, ext ? b2->stride(0) : 0, (int)K2,
                         nullptr, out->data_ptr(), out->stride(0), nullptr, 0, residual->data_ptr(),
                         residual->stride(0), (int)M, (int)N, (int)K, 6, 0, 1, zero_page(a).data_ptr(), (int)bn,
                         cur_stream()),
             "gemm_big(act 6)");
    return *out;
  }
  if (bias.has_value() && bias->defined()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous() && !swiglu, "gemm_big: bias");
  }
  const int64_t Nout = swiglu ? N / 2 : N;
  const auto odt = out_mode == 0 ? at::kBFloat16 : at::kFloat;
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == Nout && c.stride(1) == 1, "gemm_big: bad out shape");
    TORCH_CHECK(c.scalar_type() == odt, "gemm_big: bad out dtype");
    TORCH_CHECK(out_mode == 2 || c.stride(0) % 8 == 0, "gemm_big: out row stride must be a multiple of 8");
    // the epilogue stores whole 16-B (bf16) / 4-float chunks: a ragged last chunk of the last row
    // must still land inside the tensor's storage
    const int64_t chunk = out_mode == 0 ? 8 : 4;
    TORCH_CHECK(out_mode == 2 || Nout % chunk == 0 ||
                    (c.storage_offset() + (M - 1) * c.stride(0) + (Nout + chunk - 1) / chunk * chunk) * c.element_size() <=
                        (int64_t)c.storage().nbytes(),
                "gemm_big: out width ", Nout, " is not a multiple of ", chunk, " and its storage has no padding");
    CHECK_ALIGN16(c);
  } else {
    TORCH_CHECK(out_mode != 2, "gemm_big: atomic accumulation needs an initialised out");
    // an output width that is not a multiple of 8 (e.g. OpenChat's 32002-token vocabulary) gets a
    // row stride padded to 8 elements: the epilogue writes whole 16-B (bf16) / 4-float chunks
    const int64_t Np = (Nout + 7) / 8 * 8;
    c = at::empty({M, Np}, a.options().dtype(odt));
    if (Np != Nout) c = c.narrow(1, 0, Nout);
  }
  void* c2 = nullptr;
  int64_t ldc2 = 0;
  if (out2.has_value() && out2->defined()) {
    TORCH_CHECK(swiglu, "gemm_big: out2 is the SwiGLU pre-activation");
    CHECK_BF16(*out2);
    TORCH_CHECK(out2->size(0) == M && out2->size(1) == N && out2->stride(1) == 1 && out2->stride(0) % 8 == 0,
                "gemm_big: bad out2");
    CHECK_ALIGN16(*out2);
    c2 = out2->data_ptr();
    ldc2 = out2->stride(0);
  }
  const bool has_r = residual.has_value() && residual->defined();
  if (has_r) {
    CHECK_BF16(*residual);
    TORCH_CHECK(out_mode == 0 && !swiglu && residual->dim() == 2 && residual->size(0) == M && residual->size(1) == N &&
                    residual->stride(1) == 1 && residual->stride(0) % 8 == 0,
                "gemm_big: residual must be bf16 [M, N] (bf16 output, no SwiGLU)");
    // the epilogue reads the residual in 16-B chunks: the last chunk of the last row must not
    // run past the end of the tensor
    TORCH_CHECK(N % 8 == 0, "gemm_big: a residual needs N % 8 == 0, got N = ", N);
    CHECK_ALIGN16(*residual);
  }
  if (M == 0 || N == 0) return c;
  check_rc(rt_gemm_big((int)layout_a, (int)layout_b, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                       ext ? a2->data_ptr() : nullptr, ext ? a2->stride(0) : 0, ext ? b2->data_ptr() : nullptr,
                       ext ? b2->stride(0) : 0, (int)K2, opt_ptr(bias), c.data_ptr(), c.stride(0), c2, ldc2,
                       has_r ? residual->data_ptr() : nullptr, has_r ? residual->stride(0) : 0, (int)M,
                       (int)N, (int)K, (int)act, (int)out_mode, (int)nsplit, zero_page(a).data_ptr(), (int)bn,
                       cur_stream()),
           "gemm_big");
  return c;
}

// Fused qkv projection with the rotary embedding in the epilogue (gemm_big NT, E_ROPE):
// C = rope(a w^T (+ u ub^T) + bias); columns [0, rope_cols) are head_dim-wide heads rotated at
// position pos[row] (int32 [M]) with the cos / sin tables [positions, head_dim / 2] (fp32).
Tensor gemm_rope(const Tensor& a, const Tensor& w, const optional<Tensor>& u, const optional<Tensor>& ub,
                 const optional<Tensor>& bias, const Tensor& pos, const Tensor& cos, const Tensor& sin,
                 int64_t rope_cols, int64_t head_dim, optional<Tensor> out, int64_t bn) {
  CHECK_CUDA(a); CHECK_CUDA(w); CHECK_BF16(a); CHECK_BF16(w); CHECK_ROWS(a); CHECK_ROWS(w);
  CHECK_ALIGN16(a); CHECK_ALIGN16(w);
  CHECK_I32(pos); CHECK_F32(cos); CHECK_F32(sin);
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 8 == 0 && a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0,
              "gemm_rope: [M, K] x [N, K] with K and row strides % 8 == 0");
  TORCH_CHECK(N % 8 == 0, "gemm_rope: N must be a multiple of 8");
  TORCH_CHECK(pos.dim() == 1 && pos.size(0) == M && pos.is_contiguous(), "gemm_rope: pos must be int32 [M]");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous() && cos.dim() == 2 && cos.size(1) == head_dim / 2 &&
                  sin.sizes() == cos.sizes(),
              "gemm_rope: cos / sin must be contiguous fp32 [positions, head_dim / 2]");
  TORCH_CHECK(rope_cols >= 0 && rope_cols <= N && head_dim > 0 && rope_cols % head_dim == 0,
              "gemm_rope: rope_cols must be a multiple of head_dim within N");
  int64_t K2 = 0;
  const bool ext = u.has_value() && u->defined();
  if (ext) {
    TORCH_CHECK(ub.has_value() && ub->defined(), "gemm_rope: u without ub");
    CHECK_BF16(*u); CHECK_BF16(*ub); CHECK_ROWS(*u); CHECK_ROWS(*ub); CHECK_ALIGN16(*u); CHECK_ALIGN16(*ub);
    TORCH_CHECK(u->size(0) == M && ub->size(0) == N && u->size(1) == ub->size(1) && u->size(1) % 8 == 0 &&
                    u->stride(0) % 8 == 0 && ub->stride(0) % 8 == 0,
                "gemm_rope: LoRA extension shape");
    K2 = u->size(1);
  }
  if (bias.has_value() && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N && bias->is_contiguous()); }
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    CHECK_BF16(c); CHECK_ALIGN16(c);
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 && c.stride(0) % 8 == 0,
                "gemm_rope: bad out");
  } else {
    c = at::empty({M, N}, a.options());
  }
  if (M == 0) return c;
  check_rc(rt_gemm_big_rope(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), ext ? u->data_ptr() : nullptr,
                            ext ? u->stride(0) : 0, ext ? ub->data_ptr() : nullptr, ext ? ub->stride(0) : 0, (int)K2,
                            opt_ptr(bias), c.data_ptr(), c.stride(0), (int)M, (int)N, (int)K, pos.data_ptr<int>(),
                            cos.data_ptr<float>(), sin.data_ptr<float>(), (int)rope_cols, (int)head_dim,
                            zero_page(a).data_ptr(), (int)bn, cur_stream()),
           "gemm_rope");
  return c;
}

// 64x64-tile GEMM for narrow products (LoRA U / dU / dA / dB): same operand layouts as gemm_big;
// out_mode 0 bf16 / 1 fp32 / 2 fp32 atomic accumulate into `out` / 3 fp32 slabs [nsplit * M, N] (split-K over `nsplit`).
// bm: 64 (64x64 tiles) or 128 (128x64 tiles: the narrow B image staged once per 128 A rows).
Tensor gemm_small(const Tensor& a, const Tensor& b, int64_t layout_a, int64_t layout_b, int64_t out_mode,
                  int64_t nsplit, optional<Tensor> out, int64_t bm) {
  TORCH_CHECK(bm == 64 || bm == 128, "gemm_small: bm must be 64 or 128");
  CHECK_CUDA(a); CHECK_CUDA(b); CHECK_BF16(a); CHECK_BF16(b); CHECK_ROWS(a); CHECK_ROWS(b);
  CHECK_ALIGN16(a); CHECK_ALIGN16(b);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_small: row strides must be multiples of 8");
  const int64_t M = layout_a ? a.size(1) : a.size(0), K = layout_a ? a.size(0) : a.size(1);
  const int64_t N = layout_b ? b.size(1) : b.size(0), Kb = layout_b ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm_small: K mismatch");
  const auto odt = out_mode == 0 ? at::kBFloat16 : at::kFloat;
  // out_mode 3: split-K slabs [nsplit * M, N] (row stride N), one per split
  const int64_t rows = out_mode == 3 ? nsplit * M : M;
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.size(0) == rows && c.size(1) == N && c.stride(1) == 1 && c.scalar_type() == odt &&
                (out_mode != 3 || c.is_contiguous()), "gemm_small: out");
  } else {
    TORCH_CHECK(out_mode != 2, "gemm_small: atomic accumulation needs an initialised out");
    c = at::empty({rows, N}, a.options().dtype(odt));
  }
  if (M == 0 || N == 0) return c;
  check_rc(rt_gemm_small((int)layout_a, (int)layout_b, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                         c.data_ptr(), c.stride(0), (int)M, (int)N, (int)K, (int)out_mode, (int)nsplit,
                         zero_page(a).data_ptr(), (int)bm, cur_stream()),
           "gemm_small");
  return c;
}

// Small-M GEMM (decode at batch 65..256, any NT GEMM whose 256x256 tiles cannot fill the chip):
// K split over `nsplit` workgroup rows into fp32 slabs (workspace `slabs`, >= nsplit*M*N floats),
// then one reduce kernel with the epilogue (bias, act / SwiGLU pairing, residual).
Tensor gemm_splitk(const Tensor& a, const Tensor& w, int64_t nsplit, Tensor slabs, const optional<Tensor>& bias,
                   int64_t act, optional<Tensor> out, const optional<Tensor>& residual, int64_t bn) {
  CHECK_CUDA(a); CHECK_BF16(a); CHECK_BF16(w); CHECK_ROWS(a); CHECK_ROWS(w); CHECK_F32(slabs);
  CHECK_ALIGN16(a); CHECK_ALIGN16(w);
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 8 == 0 && N % 8 == 0, "gemm_splitk: shapes");
  TORCH_CHECK(a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_splitk: row strides % 8");
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * M * N, "gemm_splitk: workspace too small");
  const bool swiglu = act == 5;
  TORCH_CHECK(!swiglu || N % 16 == 0, "gemm_splitk: SwiGLU needs N % 16 == 0");
  const int64_t Nout = swiglu ? N / 2 : N;
  if (bias.has_value() && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(!swiglu && bias->numel() == N); }
  const bool has_r = residual.has_value() && residual->defined();
  if (has_r) {
    CHECK_BF16(*residual);
    TORCH_CHECK(!swiglu && residual->size(0) == M && residual->size(1) == N && residual->stride(1) == 1 &&
                    residual->stride(0) % 8 == 0, "gemm_splitk: residual");
  }
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    CHECK_BF16(c);
    TORCH_CHECK(c.size(0) == M && c.size(1) == Nout && c.stride(1) == 1 && c.stride(0) % 8 == 0, "gemm_splitk: out");
  } else {
    c = at::empty({M, Nout}, a.options());
  }
  if (M == 0) return c;
  check_rc(rt_gemm_big(0, 0, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), nullptr, 0, nullptr, 0, 0,
                       nullptr, slabs.data_ptr(), N, nullptr, 0, nullptr, 0, (int)M, (int)N, (int)K, 0, 3,
                       (int)nsplit, zero_page(a).data_ptr(), (int)bn, cur_stream()),
           "gemm_splitk");
  check_rc(rt_gemm_splitk_reduce(slabs.data_ptr<float>(), (int)nsplit, (int)M, (int)N, opt_ptr(bias), (int)act,
                                 has_r ? residual->data_ptr() : nullptr, has_r ? residual->stride(0) : 0, c.data_ptr(),
                                 c.stride(0), cur_stream()),
           "gemm_splitk_reduce");
  return c;
}

// ---------------------------------------------------------------------------------------------
// fp8 (OCP e4m3fn): per-row quantisation and the two fp8 GEMM forms
std::vector<Tensor> quant_fp8(const Tensor& x) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_ROWS(x);
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0, "quant_fp8: [R, C] with C % 8 == 0");
  auto q = at::empty({x.size(0), x.size(1)}, x.options().dtype(at::kByte));
  auto s = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  check_rc(rt_quant_fp8_rows(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0), s.data_ptr<float>(), x.size(0),
                             (int)x.size(1), cur_stream()),
           "quant_fp8");
  return {q, s};
}

// W8A8 forward of a LoRA-adapted frozen projection (config 5 training, M > 64): xq [M, K] e4m3fn
// with per-token scales sx, wq [N, K] with per-channel scales sw, plus the bf16 K-extension
// u8 [M, Rp] · ub8 [N, Rp]^T (pre-divided by sx / sw by the caller) on the same accumulators.
// act 5 = SwiGLU over [gate; up] (out [M, N / 2], optional pre-activation out2 [M, N]).
Tensor gemm_fp8_lora(const Tensor& xq, const Tensor& sx, const Tensor& wq, const Tensor& sw, const Tensor& u8,
                     const Tensor& ub8, int64_t act, const optional<Tensor>& out2) {
  CHECK_CUDA(xq); CHECK_F32(sx); CHECK_F32(sw); CHECK_BF16(u8); CHECK_BF16(ub8);
  TORCH_CHECK(xq.scalar_type() == at::kByte && wq.scalar_type() == at::kByte, "gemm_fp8_lora: e4m3fn operands");
  CHECK_ROWS(xq); CHECK_ROWS(wq); CHECK_ROWS(u8); CHECK_ROWS(ub8);
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0), Rp = u8.size(1);
  TORCH_CHECK(wq.size(1) == K && sx.numel() == M && sw.numel() == N && u8.size(0) == M && ub8.size(0) == N &&
                  ub8.size(1) == Rp && Rp % 8 == 0, "gemm_fp8_lora: shapes");
  TORCH_CHECK(act == 0 || act == 5, "gemm_fp8_lora: act 0 or SwiGLU");
  const int64_t Nout = act == 5 ? N / 2 : N;
  Tensor c = at::empty({M, Nout}, xq.options().dtype(at::kBFloat16));
  void* c2 = nullptr;
  long ldc2 = 0;
  if (out2.has_value() && out2->defined()) {
    TORCH_CHECK(act == 5 && out2->scalar_type() == at::kBFloat16 && out2->size(0) == M && out2->size(1) == N &&
                    out2->stride(1) == 1, "gemm_fp8_lora: out2 is the [M, N] SwiGLU pre-activation");
    c2 = out2->data_ptr();
    ldc2 = out2->stride(0);
  }
  if (M == 0) return c;
  check_rc(rt_gemm_big_fp8(xq.data_ptr(), xq.stride(0), sx.data_ptr<float>(), wq.data_ptr(), wq.stride(0),
                           sw.data_ptr<float>(), nullptr, c.data_ptr(), c.stride(0), (int)M, (int)N, (int)K, (int)act,
                           u8.data_ptr(), u8.stride(0), ub8.data_ptr(), ub8.stride(0), (int)Rp, c2, ldc2,
                           zero_page(u8).data_ptr(), cur_stream()),
           "gemm_fp8_lora");
  return c;
}

Tensor gemm_fp8(const Tensor& a, const optional<Tensor>& sa, const Tensor& wq, const Tensor& sw,
                const optional<Tensor>& bias, int64_t act, optional<Tensor> out, const optional<Tensor>& residual,
                double norm_eps, bool w_shuffled) {
  // a: bf16 [M, K] (W8A16, M <= 64) or uint8 e4m3fn [M, K] with sa [M] (W8A8). w_shuffled: wq is
  // the tile-ordered fp8 image of shuffle_decode_weight_fp8 (W8A16 at M <= 16 only)
  CHECK_CUDA(a); CHECK_CUDA(wq); CHECK_ROWS(a); CHECK_ROWS(wq); CHECK_F32(sw);
  TORCH_CHECK(wq.scalar_type() == at::kByte, "gemm_fp8: weight must be uint8 (e4m3fn bits)");
  const bool a_bf16 = a.scalar_type() == at::kBFloat16;
  const int64_t M = a.size(0), K = a.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K && sw.numel() == N, "gemm_fp8: shapes");
  if (a_bf16) {
    TORCH_CHECK(M <= 64 && K % 64 == 0, "gemm_fp8: bf16 activations only for M <= 64");
    if (w_shuffled)
      TORCH_CHECK(K % 128 == 0 && N % (act == 5 ? 64 : 16) == 0 && wq.is_contiguous(),
                  "gemm_fp8: the tile-ordered fp8 image needs K % 128 == 0, N % 16 == 0 (SwiGLU: N % 64 == 0)");
  } else {
    TORCH_CHECK(!w_shuffled, "gemm_fp8: tile-ordered weights are a W8A16 decode layout");
    TORCH_CHECK(a.scalar_type() == at::kByte && sa.has_value() && sa->numel() == M, "gemm_fp8: W8A8 needs sa [M]");
    TORCH_CHECK(K % 128 == 0 && N % 8 == 0, "gemm_fp8: K % 128 == 0, N % 8 == 0");
  }
  if (bias.has_value() && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N); }
  const bool pair = act == 5;  // SwiGLU pair mode (W8A16 skinny only)
  if (pair)
    TORCH_CHECK(a_bf16 ? N % 64 == 0 : N % 256 == 0,
                "gemm_fp8: SwiGLU pair mode needs N % 64 == 0 (W8A16) / N % 256 == 0 (W8A8)");
  const int64_t Nout = pair ? N / 2 : N;
  Tensor c = (out.has_value() && out->defined()) ? *out : at::empty({M, Nout}, a.options().dtype(at::kBFloat16));
  TORCH_CHECK(c.size(0) == M && c.size(1) == Nout && c.stride(1) == 1 && c.scalar_type() == at::kBFloat16, "gemm_fp8: out");
  if (M == 0) return c;
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res || norm_eps > 0) TORCH_CHECK(a_bf16, "gemm_fp8: residual / in-GEMM norm need the W8A16 (M <= 64) form");
  if (has_res) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == Nout && residual->stride(1) == 1, "gemm_fp8: residual shape");
  }
  hipStream_t st = cur_stream();
  float* slabs = nullptr;
  unsigned* tickets = nullptr;
  if (a_bf16) {
    DecodeWS& ws = decode_ws(wq, st);
    slabs = ws.slabs.data_ptr<float>();
    tickets = (unsigned*)ws.tickets.data_ptr<int>();
  }
  check_rc(rt_gemm_fp8(a.data_ptr(), a.stride(0), sa.has_value() && sa->defined() ? sa->data_ptr<float>() : nullptr,
                       wq.data_ptr(), wq.stride(0), sw.data_ptr<float>(), opt_ptr(bias), c.data_ptr(), c.stride(0),
                       (int)M, (int)N, (int)K, (int)act, a_bf16 ? 1 : 0, slabs, tickets,
                       has_res ? residual->data_ptr() : nullptr, has_res ? residual->stride(0) : 0, (float)norm_eps,
                       w_shuffled ? 1 : 0, st),
           "gemm_fp8");
  return c;
}

// ---------------------------------------------------------------------------------------------
std::vector<Tensor> norm_fwd(bool layernorm, const Tensor& x, const optional<Tensor>& res, const Tensor& w,
                             const optional<Tensor>& b, double eps) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.is_contiguous(), "norm: x must be contiguous");
  const int64_t H = x.size(-1), T = x.numel() / H;
  auto y = at::empty_like(x);
  Tensor h;
  if (res.has_value() && res->defined()) {
    CHECK_BF16(*res);
    TORCH_CHECK(res->is_contiguous() && res->numel() == x.numel(), "norm: residual shape");
    h = at::empty_like(x);
  }
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  Tensor mean = layernorm ? at::empty({T}, x.options().dtype(at::kFloat)) : Tensor();
  check_rc(rt_norm_fwd(layernorm, x.data_ptr(), opt_ptr(res), w.data_ptr(), opt_ptr(b), y.data_ptr(),
                       h.defined() ? h.data_ptr() : nullptr, rstd.data_ptr<float>(),
                       layernorm ? mean.data_ptr<float>() : nullptr, (int)T, (int)H, (float)eps, nullptr, 0,
                       cur_stream()),
           "norm_fwd");
  return {y, h, rstd, mean};
}

// reduce of split-K slabs [nsplit, M, N] -> bf16 [M, N] (fallback when a consumer cannot fuse it)
Tensor splitk_reduce(const Tensor& slabs, int64_t nsplit, int64_t M, int64_t N, Tensor out) {
  CHECK_CUDA(slabs); CHECK_F32(slabs); CHECK_BF16(out);
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * M * N && out.size(0) == M && out.size(1) == N &&
              out.stride(1) == 1 && out.stride(0) % 8 == 0, "splitk_reduce: shapes");
  check_rc(rt_gemm_splitk_reduce(slabs.data_ptr<float>(), (int)nsplit, (int)M, (int)N, nullptr, 0, nullptr, 0,
                                 out.data_ptr(), out.stride(0), cur_stream()),
           "splitk_reduce");
  return out;
}

// norm_fwd whose input is the sum of `nsplit` fp32 split-K slabs [nsplit, T, H] (the reduce of a
// split-K GEMM fused into the norm; residual required: returns y and the new residual stream)
std::vector<Tensor> norm_fwd_slabs(bool layernorm, const Tensor& slabs, int64_t nsplit, int64_t T, int64_t H,
                                   const Tensor& res, const Tensor& w, const optional<Tensor>& b, double eps) {
  CHECK_CUDA(slabs); CHECK_F32(slabs); CHECK_BF16(res); CHECK_BF16(w);
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * T * H && res.is_contiguous() && res.numel() == T * H,
              "norm_fwd_slabs: shapes");
  auto y = at::empty({T, H}, res.options());
  auto h = at::empty({T, H}, res.options());
  auto rstd = at::empty({T}, res.options().dtype(at::kFloat));
  Tensor mean = layernorm ? at::empty({T}, res.options().dtype(at::kFloat)) : Tensor();
  check_rc(rt_norm_fwd(layernorm, nullptr, res.data_ptr(), w.data_ptr(), opt_ptr(b), y.data_ptr(), h.data_ptr(),
                       rstd.data_ptr<float>(), layernorm ? mean.data_ptr<float>() : nullptr, (int)T, (int)H,
                       (float)eps, slabs.data_ptr<float>(), (int)nsplit, cur_stream()),
           "norm_fwd_slabs");
  return {y, h};
}

// W8A8 split-K into fp32 slabs (config-5 decode at batch > 64; the consumer sums them)
void gemm_fp8_splitk_raw(const Tensor& xq, const Tensor& sx, const Tensor& wq, const Tensor& sw, int64_t nsplit,
                         Tensor slabs, int64_t bn) {
  CHECK_CUDA(xq); CHECK_F32(sx); CHECK_F32(sw); CHECK_ROWS(xq); CHECK_ROWS(wq); CHECK_F32(slabs);
  TORCH_CHECK(xq.scalar_type() == at::kByte && wq.scalar_type() == at::kByte, "gemm_fp8_splitk_raw: e4m3fn operands");
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K && sx.numel() == M && sw.numel() == N && K % 128 == 0 && N % 8 == 0,
              "gemm_fp8_splitk_raw: shapes");
  TORCH_CHECK(xq.stride(0) % 16 == 0 && wq.stride(0) % 16 == 0, "gemm_fp8_splitk_raw: row strides % 16");
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * M * N, "gemm_fp8_splitk_raw: workspace too small");
  if (M == 0) return;
  check_rc(rt_gemm_big_fp8_slabs(xq.data_ptr(), xq.stride(0), sx.data_ptr<float>(), wq.data_ptr(), wq.stride(0),
                                 sw.data_ptr<float>(), slabs.data_ptr<float>(), (int)M, (int)N, (int)K, (int)nsplit,
                                 (int)bn, cur_stream()),
           "gemm_fp8_splitk_raw");
}

// split-K partial slabs only (the reduce is fused into the consumer): slabs [nsplit, M, N] fp32
void gemm_splitk_raw(const Tensor& a, const Tensor& w, int64_t nsplit, Tensor slabs, int64_t bn) {
  CHECK_CUDA(a); CHECK_BF16(a); CHECK_BF16(w); CHECK_ROWS(a); CHECK_ROWS(w); CHECK_F32(slabs);
  CHECK_ALIGN16(a); CHECK_ALIGN16(w);
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 8 == 0 && N % 8 == 0, "gemm_splitk_raw: shapes");
  TORCH_CHECK(a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_splitk_raw: row strides % 8");
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * M * N, "gemm_splitk_raw: workspace too small");
  if (M == 0) return;
  check_rc(rt_gemm_big(0, 0, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), nullptr, 0, nullptr, 0, 0,
                       nullptr, slabs.data_ptr(), N, nullptr, 0, nullptr, 0, (int)M, (int)N, (int)K, 0, 3,
                       (int)nsplit, zero_page(a).data_ptr(), (int)bn, cur_stream()),
           "gemm_splitk_raw");
}

std::vector<Tensor> norm_bwd(bool layernorm, const Tensor& dy, const Tensor& h, const Tensor& w, const Tensor& rstd,
                             const optional<Tensor>& mean, const optional<Tensor>& dh_res, bool need_dw, bool need_db) {
  CHECK_CUDA(dy); CHECK_BF16(dy); CHECK_BF16(h);
  TORCH_CHECK(dy.is_contiguous() && h.is_contiguous(), "norm_bwd: contiguous inputs required");
  const int64_t H = dy.size(-1), T = dy.numel() / H;
  auto dh = at::empty_like(dy);
  // dw / db: one fp32 partial row per workgroup (plain stores), summed in a fixed order below — no
  // arrival-order atomics (bitwise-reproducible full fine-tuning)
  const int64_t nb = rt_norm_bwd_blocks((int)T);
  Tensor dw = need_dw ? at::empty({nb, H}, dy.options().dtype(at::kFloat)) : Tensor();
  Tensor db = need_db ? at::empty({nb, H}, dy.options().dtype(at::kFloat)) : Tensor();
  if (dh_res.has_value() && dh_res->defined()) {
    CHECK_BF16(*dh_res);
    TORCH_CHECK(dh_res->is_contiguous(), "norm_bwd: dh_res contiguous");
  }
  check_rc(rt_norm_bwd(layernorm, dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(),
                       layernorm ? (const float*)mean->data_ptr() : nullptr, opt_ptr(dh_res), dh.data_ptr(),
                       need_dw ? dw.data_ptr<float>() : nullptr, need_db ? db.data_ptr<float>() : nullptr, (int)T,
                       (int)H, cur_stream()),
           "norm_bwd");
  return {dh, need_dw ? dw.sum(0) : dw, need_db ? db.sum(0) : db};
}

// ---------------------------------------------------------------------------------------------
void rope_qkv(Tensor qkv, const Tensor& pos, const optional<Tensor>& cos, const optional<Tensor>& sin, int64_t S,
              int64_t Hq, int64_t Hkv, int64_t D, double sign, const optional<Tensor>& kc, const optional<Tensor>& vc,
              const optional<Tensor>& slot_base, bool rope_q) {
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_ROWS(qkv); CHECK_I32(pos);
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D, "rope: qkv too narrow");
  int Smax = 0;
  if (kc.has_value() && kc->defined()) {
    CHECK_BF16(*kc); CHECK_BF16(*vc);
    TORCH_CHECK(kc->dim() == 4 && kc->size(1) == Hkv && kc->size(3) == D && kc->is_contiguous(), "rope: cache layout");
    Smax = (int)kc->size(2);
  }
  if (cos.has_value() && cos->defined()) { CHECK_F32(*cos); CHECK_F32(*sin); }
  if (slot_base.has_value() && slot_base->defined()) CHECK_I32(*slot_base);
  check_rc(rt_rope_qkv(qkv.data_ptr(), qkv.stride(0), pos.data_ptr<int>(),
                       (const float*)opt_ptr(cos), (const float*)opt_ptr(sin), (int)qkv.size(0), (int)S, (int)Hq,
                       (int)Hkv, (int)D, (float)sign, (void*)opt_ptr(kc), (void*)opt_ptr(vc),
                       (const int*)opt_ptr(slot_base), Smax, rope_q ? 1 : 0, cur_stream()),
           "rope_qkv");
}

Tensor swiglu_fwd(const Tensor& gu) {
  CHECK_CUDA(gu); CHECK_BF16(gu); TORCH_CHECK(gu.is_contiguous());
  const int64_t F2 = gu.size(-1), T = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F2 / 2;
  auto y = at::empty(sizes, gu.options());
  check_rc(rt_swiglu_fwd(gu.data_ptr(), y.data_ptr(), T, (int)(F2 / 2), cur_stream()), "swiglu_fwd");
  return y;
}

Tensor swiglu_bwd(const Tensor& gu, const Tensor& dy) {
  CHECK_CUDA(gu); CHECK_BF16(gu); CHECK_BF16(dy); TORCH_CHECK(gu.is_contiguous() && dy.is_contiguous());
  const int64_t F2 = gu.size(-1), T = gu.numel() / F2;
  auto dgu = at::empty_like(gu);
  check_rc(rt_swiglu_bwd(gu.data_ptr(), dy.data_ptr(), dgu.data_ptr(), T, (int)(F2 / 2), cur_stream()), "swiglu_bwd");
  return dgu;
}

Tensor embed(const Tensor& table, const Tensor& ids, const optional<Tensor>& ptable, const optional<Tensor>& pids) {
  CHECK_CUDA(table); CHECK_BF16(table); CHECK_I64(ids); TORCH_CHECK(table.is_contiguous() && ids.is_contiguous());
  const int64_t H = table.size(1), T = ids.numel();
  auto sizes = ids.sizes().vec();
  sizes.push_back(H);
  auto out = at::empty(sizes, table.options());
  check_rc(rt_embed(table.data_ptr(), ids.data_ptr<int64_t>() ? (const long*)ids.data_ptr() : nullptr, opt_ptr(ptable),
                    (const long*)opt_ptr(pids), out.data_ptr(), T, (int)H, cur_stream()),
           "embed");
  return out;
}

// src [N, H] (row stride % 8 == 0) -> out [R, H]: out[r] = src[inv[r]] or zeros where inv[r] < 0
Tensor rows_scatter(const Tensor& src, const Tensor& inv, int64_t R) {
  CHECK_CUDA(src); CHECK_BF16(src); CHECK_CUDA(inv);
  TORCH_CHECK(src.dim() == 2 && src.stride(1) == 1 && src.stride(0) % 8 == 0, "rows_scatter: [N, H] rows expected");
  TORCH_CHECK(inv.scalar_type() == at::kInt && inv.is_contiguous() && inv.numel() == R, "rows_scatter: inv int32 [R]");
  const int64_t H = src.size(1);
  TORCH_CHECK(H % 8 == 0, "rows_scatter: H % 8");
  auto out = at::empty({R, H}, src.options());
  check_rc(rt_rows_scatter(src.data_ptr(), src.stride(0), inv.data_ptr<int>(), out.data_ptr(), R, (int)H, src.size(0),
                           cur_stream()),
           "rows_scatter");
  return out;
}

// ---------------------------------------------------------------------------------------------
std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, int64_t B, int64_t Sq, int64_t Sk,
                             int64_t Hq, int64_t Hkv, int64_t D, bool causal, int64_t window, double scale,
                             const optional<Tensor>& kv_start, const optional<Tensor>& kv_len,
                             const optional<Tensor>& rel_bias, int64_t rb_L, bool need_lse) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_ROWS(q); CHECK_ROWS(k); CHECK_ROWS(v);
  TORCH_CHECK(q.size(0) == B * Sq && k.size(0) == B * Sk && v.size(0) == B * Sk, "attn_fwd: row counts");
  TORCH_CHECK(Hq % Hkv == 0, "attn_fwd: Hq % Hkv");
  TORCH_CHECK(q.stride(0) % 8 == 0 && k.stride(0) % 8 == 0 && v.stride(0) % 8 == 0, "attn_fwd: strides % 8");
  auto o = at::empty({B * Sq, Hq * D}, q.options());
  Tensor lse = need_lse ? at::empty({B, Hq, Sq}, q.options().dtype(at::kFloat)) : Tensor();
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  if (kv_len.has_value() && kv_len->defined()) CHECK_I32(*kv_len);
  if (rel_bias.has_value() && rel_bias->defined()) {
    CHECK_F32(*rel_bias);
    TORCH_CHECK(rel_bias->size(0) == Hq && rel_bias->size(1) == 2 * rb_L - 1 && rb_L >= std::max(Sq, Sk));
  }
  check_rc(rt_attn_fwd(q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0), o.data_ptr(),
                       o.stride(0), need_lse ? lse.data_ptr<float>() : nullptr, (const int*)opt_ptr(kv_start),
                       (const int*)opt_ptr(kv_len), (const float*)opt_ptr(rel_bias), (int)rb_L, (int)B, (int)Sq,
                       (int)Sk, (int)Hq, (int)Hkv, (int)D, causal ? 1 : 0, (int)window, (float)scale, cur_stream()),
           "attn_fwd");
  return {o, lse};
}

void attn_decode(const Tensor& q, const Tensor& kc, const Tensor& vc, const Tensor& kv_len,
                 const optional<Tensor>& kv_start, int64_t window, double scale, int64_t Hq, Tensor part, int64_t PS,
                 Tensor out) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_ROWS(q); CHECK_BF16(kc); CHECK_BF16(vc); CHECK_I32(kv_len); CHECK_F32(part);
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.is_contiguous(), "attn_decode: cache layout");
  const int64_t B = kc.size(0), Hkv = kc.size(1), Smax = kc.size(2), D = kc.size(3);
  const int64_t NP = (Smax + PS - 1) / PS, G = Hq / Hkv;
  TORCH_CHECK(part.numel() >= B * Hkv * NP * G * (D + 2), "attn_decode: partial workspace too small");
  TORCH_CHECK(q.size(0) == B && out.size(0) == B, "attn_decode: batch");
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  check_rc(rt_attn_decode(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(), (int)Smax, kv_len.data_ptr<int>(),
                          (const int*)opt_ptr(kv_start), (int)window, part.data_ptr<float>(), (int)NP, (int)PS,
                          out.data_ptr(), out.stride(0), (int)B, (int)Hq, (int)Hkv, (int)D, (float)scale,
                          cur_stream()),
           "attn_decode");
}

// fp8 K/V cache (config 5): kc / vc are e4m3fn byte caches [B, Hkv, Smax, D] (K rows k-permuted)
// with fp32 per-slot scales ksc / vsc [B, Hkv, SmaxP] (SmaxP >= Smax, a multiple of 16), passed to
// the decode call itself. Only the MFMA decode kernels read them.
struct KvScales {
  float* k = nullptr;
  float* v = nullptr;
  int smaxp = 0;
};
static KvScales check_cache(const Tensor& kc, const Tensor& vc, const optional<Tensor>& ksc,
                            const optional<Tensor>& vsc, const char* who) {
  KvScales r;
  const bool fp8 = ksc.has_value() && ksc->defined();
  TORCH_CHECK(fp8 == (vsc.has_value() && vsc->defined()), who, ": k and v scales go together");
  if (!fp8) {
    CHECK_BF16(kc); CHECK_BF16(vc);
    return r;
  }
  CHECK_CUDA(*ksc); CHECK_F32(*ksc); CHECK_F32(*vsc);
  TORCH_CHECK(ksc->dim() == 3 && ksc->is_contiguous() && vsc->is_contiguous() && vsc->sizes() == ksc->sizes(),
              who, ": scales must be contiguous [B, Hkv, SmaxP]");
  TORCH_CHECK(kc.scalar_type() == at::kByte && vc.scalar_type() == at::kByte, who, ": fp8 scales for a bf16 cache");
  TORCH_CHECK(ksc->size(2) >= kc.size(2) && kc.size(3) == 128, who, ": fp8 cache needs D = 128 and SmaxP >= Smax");
  TORCH_CHECK(ksc->size(0) == kc.size(0) && ksc->size(1) == kc.size(1), who, ": scale shape");
  r.k = ksc->data_ptr<float>();
  r.v = vsc->data_ptr<float>();
  r.smaxp = (int)ksc->size(2);
  return r;
}

// Prompt K / V of the rotated qkv rows [B * S] -> fp8 cache slots [0, S) with per-slot scales.
void kv_store_fp8(const Tensor& qkv, Tensor kc, Tensor vc, Tensor ksc, Tensor vsc, int64_t B, int64_t S, int64_t Hq) {
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_ROWS(qkv); CHECK_F32(ksc); CHECK_F32(vsc);
  TORCH_CHECK(kc.scalar_type() == at::kByte && vc.scalar_type() == at::kByte && kc.dim() == 4 && kc.is_contiguous() &&
                  vc.is_contiguous() && vc.sizes() == kc.sizes(), "kv_store_fp8: cache layout");
  const int64_t Hkv = kc.size(1), Smax = kc.size(2), D = kc.size(3);
  TORCH_CHECK(kc.size(0) == B && qkv.size(0) == B * S && qkv.size(1) >= (Hq + 2 * Hkv) * D, "kv_store_fp8: shapes");
  TORCH_CHECK(ksc.dim() == 3 && ksc.size(0) == B && ksc.size(1) == Hkv && ksc.is_contiguous() && vsc.is_contiguous() &&
                  vsc.sizes() == ksc.sizes(), "kv_store_fp8: scales");
  check_rc(rt_kv_store_fp8(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), ksc.data_ptr<float>(),
                           vsc.data_ptr<float>(), (int)B, (int)S, (int)Hq, (int)Hkv, (int)D, (int)Smax,
                           (int)ksc.size(2), cur_stream()),
           "kv_store_fp8");
}

void attn_decode_fused(const Tensor& qkv, Tensor kc, Tensor vc, const Tensor& slot, const Tensor& attn_len,
                       const optional<Tensor>& kv_start, const optional<Tensor>& pos, const optional<Tensor>& cos,
                       const optional<Tensor>& sin, double sign, int64_t window, double scale, int64_t Hq, Tensor part,
                       Tensor tickets, int64_t PS, Tensor out, const optional<Tensor>& ksc,
                       const optional<Tensor>& vsc, const optional<Tensor>& stamps) {
  const KvScales sc = check_cache(kc, vc, ksc, vsc, "attn_decode_fused");
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_ROWS(qkv); CHECK_I32(slot);
  CHECK_I32(attn_len); CHECK_F32(part); CHECK_I32(tickets); CHECK_BF16(out); CHECK_ROWS(out);
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.is_contiguous() && vc.sizes() == kc.sizes(),
              "attn_decode_fused: cache layout");
  const int64_t B = kc.size(0), Hkv = kc.size(1), Smax = kc.size(2), D = kc.size(3);
  const int64_t NP = (Smax + PS - 1) / PS, G = Hq / Hkv;
  TORCH_CHECK(G * Hkv == Hq, "attn_decode_fused: Hq must be a multiple of Hkv");
  TORCH_CHECK(qkv.size(0) == B && out.size(0) == B && slot.numel() == B && attn_len.numel() == B,
              "attn_decode_fused: batch");
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D && out.size(1) >= Hq * D, "attn_decode_fused: widths");
  TORCH_CHECK(part.numel() >= B * Hkv * NP * G * (D + 2), "attn_decode_fused: partial workspace too small");
  TORCH_CHECK(tickets.numel() >= B * Hkv, "attn_decode_fused: ticket workspace too small");
  const bool rot = cos.has_value() && cos->defined();
  if (rot) {
    CHECK_F32(*cos); CHECK_F32(*sin);
    TORCH_CHECK(pos.has_value() && pos->defined(), "attn_decode_fused: rotary needs pos");
    CHECK_I32(*pos);
    TORCH_CHECK(cos->size(-1) == D / 2 && cos->is_contiguous() && sin->is_contiguous(), "attn_decode_fused: tables");
  }
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  check_rc(rt_attn_decode_fused(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), (int)Smax,
                                slot.data_ptr<int>(), attn_len.data_ptr<int>(), (const int*)opt_ptr(kv_start),
                                rot ? pos->data_ptr<int>() : nullptr, rot ? cos->data_ptr<float>() : nullptr,
                                rot ? sin->data_ptr<float>() : nullptr, (float)sign, (int)window,
                                part.data_ptr<float>(), (unsigned*)tickets.data_ptr<int>(), (int)NP, (int)PS,
                                out.data_ptr(), out.stride(0), (int)B, (int)Hq, (int)Hkv, (int)D, (float)scale,
                                nullptr, 0, sc.k, sc.v, sc.smaxp,
                                stamps.has_value() && stamps->defined() ? (long long*)stamps->data_ptr() : nullptr,
                                cur_stream()),
           "attn_decode_fused");
}

// The same decode step with q | k | v given as the qkv GEMM's nsplit fp32 split-K slabs
// [nsplit, B, (Hq + 2 Hkv) D]: the MFMA kernel sums them in its prologue (no reduce launch).
// Returns false (nothing launched) when the MFMA kernel does not apply to the shape.
bool attn_decode_fused_slabs(const Tensor& slabs, int64_t nsplit, Tensor kc, Tensor vc, const Tensor& slot,
                             const Tensor& attn_len, const optional<Tensor>& kv_start, const optional<Tensor>& pos,
                             const optional<Tensor>& cos, const optional<Tensor>& sin, double sign, int64_t window,
                             double scale, int64_t Hq, Tensor part, Tensor tickets, int64_t PS, Tensor out,
                             const optional<Tensor>& ksc, const optional<Tensor>& vsc) {
  const KvScales sc = check_cache(kc, vc, ksc, vsc, "attn_decode_fused_slabs");
  CHECK_CUDA(slabs); CHECK_F32(slabs); CHECK_I32(slot); CHECK_I32(attn_len);
  CHECK_F32(part); CHECK_I32(tickets); CHECK_BF16(out); CHECK_ROWS(out);
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.is_contiguous() && vc.sizes() == kc.sizes(),
              "attn_decode_fused_slabs: cache layout");
  const int64_t B = kc.size(0), Hkv = kc.size(1), Smax = kc.size(2), D = kc.size(3);
  const int64_t NP = (Smax + PS - 1) / PS, G = Hq / Hkv;
  TORCH_CHECK(G * Hkv == Hq, "attn_decode_fused_slabs: Hq must be a multiple of Hkv");
  if (!rt_attn_decode_mfma_ok((int)B, (int)Hq, (int)Hkv, (int)D, (int)NP)) return false;  // caller reduces first
  const int64_t W = (Hq + 2 * Hkv) * D;
  TORCH_CHECK(slabs.is_contiguous() && slabs.numel() >= nsplit * B * W && nsplit >= 1, "attn_decode_fused_slabs: slabs");
  TORCH_CHECK(out.size(0) == B && slot.numel() == B && attn_len.numel() == B && out.size(1) >= Hq * D,
              "attn_decode_fused_slabs: batch");
  TORCH_CHECK(tickets.numel() >= B * Hkv && part.numel() >= B * Hkv * NP * G * (D + 2), "attn_decode_fused_slabs: ws");
  const bool rot = cos.has_value() && cos->defined();
  if (rot) {
    CHECK_F32(*cos); CHECK_F32(*sin);
    TORCH_CHECK(pos.has_value() && pos->defined(), "attn_decode_fused_slabs: rotary needs pos");
    CHECK_I32(*pos);
    TORCH_CHECK(cos->size(-1) == D / 2 && cos->is_contiguous() && sin->is_contiguous(), "attn_decode_fused_slabs: tables");
  }
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  check_rc(rt_attn_decode_fused(slabs.data_ptr(), W, kc.data_ptr(), vc.data_ptr(), (int)Smax, slot.data_ptr<int>(),
                                attn_len.data_ptr<int>(), (const int*)opt_ptr(kv_start),
                                rot ? pos->data_ptr<int>() : nullptr, rot ? cos->data_ptr<float>() : nullptr,
                                rot ? sin->data_ptr<float>() : nullptr, (float)sign, (int)window,
                                part.data_ptr<float>(), (unsigned*)tickets.data_ptr<int>(), (int)NP, (int)PS,
                                out.data_ptr(), out.stride(0), (int)B, (int)Hq, (int)Hkv, (int)D, (float)scale,
                                slabs.data_ptr<float>(), (int)nsplit, sc.k, sc.v, sc.smaxp, nullptr, cur_stream()),
           "attn_decode_fused_slabs");
  return true;
}

void attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& dout, const Tensor& lse,
              Tensor dq, Tensor dk, Tensor dv, int64_t B, int64_t S, int64_t Hq, int64_t Hkv, int64_t D, bool causal,
              int64_t window, double scale, const optional<Tensor>& kv_start, const optional<Tensor>& rope_pos,
              const optional<Tensor>& rope_cos, const optional<Tensor>& rope_sin) {
  CHECK_CUDA(q); CHECK_ROWS(q); CHECK_ROWS(k); CHECK_ROWS(v); CHECK_ROWS(o); CHECK_ROWS(dout);
  // RoPE backward fused into the dQ / dK stores: pos int32 [B * S], cos / sin fp32 [positions, D / 2]
  const bool rope = rope_cos.has_value() && rope_cos->defined();
  if (rope) {
    TORCH_CHECK(rope_pos.has_value() && rope_pos->defined() && rope_sin.has_value() && rope_sin->defined(),
                "attn_bwd: rope needs pos, cos and sin");
    CHECK_I32(*rope_pos); CHECK_F32(*rope_cos); CHECK_F32(*rope_sin);
    TORCH_CHECK(rope_pos->numel() == B * S && rope_pos->is_contiguous() && rope_cos->is_contiguous() &&
                    rope_sin->is_contiguous() && rope_cos->dim() == 2 && rope_cos->size(1) == D / 2 &&
                    rope_sin->sizes() == rope_cos->sizes(),
                "attn_bwd: rope tables [positions, D / 2] and pos [B * S]");
  }
  CHECK_ROWS(dq); CHECK_ROWS(dk); CHECK_ROWS(dv); CHECK_F32(lse);
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  check_rc(rt_attn_bwd(q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0), o.data_ptr(),
                       o.stride(0), dout.data_ptr(), dout.stride(0), lse.data_ptr<float>(), delta.data_ptr<float>(),
                       nullptr, dq.data_ptr(), dq.stride(0), dk.data_ptr(), dk.stride(0),
                       dv.data_ptr(), dv.stride(0), (const int*)opt_ptr(kv_start), (int)B, (int)S, (int)Hq, (int)Hkv,
                       (int)D, causal ? 1 : 0, (int)window, (float)scale,
                       rope ? rope_pos->data_ptr<int>() : nullptr, rope ? rope_cos->data_ptr<float>() : nullptr,
                       rope ? rope_sin->data_ptr<float>() : nullptr, cur_stream()),
           "attn_bwd");
}

// ---------------------------------------------------------------------------------------------
std::vector<Tensor> logprob_fwd(const Tensor& logits, const optional<Tensor>& targets, double inv_temp, bool need_ent) {
  CHECK_CUDA(logits); CHECK_ROWS(logits); CHECK_ALIGN16(logits);
  const bool f32 = logits.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || logits.scalar_type() == at::kBFloat16, "logprob: logits must be bf16 or f32");
  TORCH_CHECK((logits.stride(0) * logits.element_size()) % 16 == 0, "logprob: row stride must be 16-B aligned");
  const int64_t T = logits.size(0), V = logits.size(1);
  auto opts = logits.options().dtype(at::kFloat);
  auto logp = at::empty({T}, opts), lse = at::empty({T}, opts), ex = at::empty({T}, opts);
  Tensor ent = need_ent ? at::empty({T}, opts) : Tensor();
  if (targets.has_value() && targets->defined()) { CHECK_I64(*targets); TORCH_CHECK(targets->numel() == T); }
  check_rc(rt_logprob_fwd(logits.data_ptr(), f32, logits.stride(0), (const long*)opt_ptr(targets), (float)inv_temp, T,
                          (int)V, logp.data_ptr<float>(), need_ent ? ent.data_ptr<float>() : nullptr,
                          lse.data_ptr<float>(), ex.data_ptr<float>(), cur_stream()),
           "logprob_fwd");
  return {logp, ent, lse, ex};
}

Tensor logprob_bwd(const Tensor& logits, const optional<Tensor>& targets, double inv_temp, const Tensor& lse,
                   const Tensor& ex, const optional<Tensor>& g_logp, const optional<Tensor>& g_ent) {
  CHECK_CUDA(logits); CHECK_ROWS(logits);
  const bool f32 = logits.scalar_type() == at::kFloat;
  const int64_t T = logits.size(0), V = logits.size(1);
  auto d = at::empty({T, V}, logits.options().dtype(at::kBFloat16));
  check_rc(rt_logprob_bwd(logits.data_ptr(), f32, logits.stride(0), (const long*)opt_ptr(targets), (float)inv_temp, T,
                          (int)V, lse.data_ptr<float>(), ex.data_ptr<float>(), (const float*)opt_ptr(g_logp),
                          (const float*)opt_ptr(g_ent), d.data_ptr(), d.stride(0), cur_stream()),
           "logprob_bwd");
  return d;
}

void sample(const Tensor& logits, double inv_temp, int64_t top_k, double top_p, bool greedy, int64_t seed,
            const optional<Tensor>& offset, const optional<Tensor>& active, Tensor out_tok,
            const optional<Tensor>& out_logp) {
  CHECK_CUDA(logits); CHECK_ROWS(logits); CHECK_I64(out_tok);
  const bool f32 = logits.scalar_type() == at::kFloat;
  if (offset.has_value() && offset->defined()) CHECK_I64(*offset);
  check_rc(rt_sample(logits.data_ptr(), f32, logits.stride(0), logits.size(0), (int)logits.size(1), (float)inv_temp,
                     (int)top_k, (float)top_p, greedy ? 1 : 0, (uint64_t)seed, (const int64_t*)opt_ptr(offset),
                     (const uint8_t*)opt_ptr(active), (long*)out_tok.data_ptr(), (float*)opt_ptr(out_logp),
                     cur_stream()),
           "sample");
}

// ---------------------------------------------------------------------------------------------
void adamw(Tensor p, const Tensor& g, Tensor m, Tensor v, const optional<Tensor>& pbf, double lr, double b1, double b2,
           double eps, double wd, int64_t step, double max_norm, Tensor partials, Tensor norm_out, Tensor skipped) {
  CHECK_CUDA(p); CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(partials);
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous());
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw: sizes");
  if (pbf.has_value() && pbf->defined()) { CHECK_BF16(*pbf); TORCH_CHECK(pbf->numel() == n); }
  const int nparts = (int)partials.numel();
  check_rc(rt_grad_sumsq(g.data_ptr<float>(), n, partials.data_ptr<float>(), nparts, cur_stream()), "grad_sumsq");
  check_rc(rt_adamw(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                    (void*)opt_ptr(pbf), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                    (float)max_norm, partials.data_ptr<float>(), nparts, norm_out.data_ptr<float>(),
                    skipped.data_ptr<int>(), cur_stream()),
           "adamw");
}

// The update half of adamw() on partials another pass (and a cross-rank sum) already produced:
// ZeRO-1 (parallel.zero) reduces each rank's shard sum of squares over the ranks before any rank
// applies its clipped update.
void adamw_apply(Tensor p, const Tensor& g, Tensor m, Tensor v, const optional<Tensor>& pbf, double lr, double b1,
                 double b2, double eps, double wd, int64_t step, double max_norm, const Tensor& partials,
                 Tensor norm_out, Tensor skipped) {
  CHECK_CUDA(p); CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(partials);
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous() &&
              partials.is_contiguous(), "adamw_apply: buffers must be contiguous");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw_apply: sizes");
  CHECK_ALIGN16(p); CHECK_ALIGN16(g); CHECK_ALIGN16(m); CHECK_ALIGN16(v);
  if (pbf.has_value() && pbf->defined()) {
    CHECK_BF16(*pbf);
    TORCH_CHECK(pbf->numel() == n && pbf->is_contiguous(), "adamw_apply: bf16 copy");
  }
  TORCH_CHECK(partials.numel() >= 1 && partials.numel() <= 1024, "adamw_apply: partials");
  check_rc(rt_adamw(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                    (void*)opt_ptr(pbf), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                    (float)max_norm, partials.data_ptr<float>(), (int)partials.numel(), norm_out.data_ptr<float>(),
                    skipped.data_ptr<int>(), cur_stream()),
           "adamw_apply");
}

// per-workgroup partial sums of g^2 into partials (one launch of partials.numel() workgroups)
void grad_sumsq(const Tensor& g, Tensor partials) {
  CHECK_CUDA(g); CHECK_F32(g); CHECK_F32(partials);
  TORCH_CHECK(g.is_contiguous() && partials.is_contiguous(), "grad_sumsq: contiguous");
  check_rc(rt_grad_sumsq(g.data_ptr<float>(), g.numel(), partials.data_ptr<float>(), (int)partials.numel(),
                         cur_stream()),
           "grad_sumsq");
}

// LoRA backward epilogue: tab int64 [n, 9] on the device = {src, src_ld, dst, dst_ld, rows, cols,
// fp32 scale bits, slabs, slab stride}: dst += scale * (sum of the split-K slabs, fixed order)
void lora_grad_accum(const Tensor& tab, int64_t max_elems) {
  CHECK_CUDA(tab);
  TORCH_CHECK(tab.scalar_type() == at::kLong && tab.is_contiguous() && tab.dim() == 2 && tab.size(1) == 9,
              "lora_grad_accum: table must be contiguous int64 [n, 9]");
  check_rc(rt_lora_grad_accum((const long*)tab.data_ptr<int64_t>(), (int)tab.size(0), (long)max_elems, cur_stream()),
           "lora_grad_accum");
}

// Batched scaled fp32 -> bf16 scatter (LoRA compute images): tab int64 [n, 7] on the device =
// {src, src_ld, dst, dst_ld, rows, cols, fp32 scale bits}; max_elems = max rows * cols.
void scatter_scaled(const Tensor& tab, int64_t max_elems) {
  CHECK_CUDA(tab);
  TORCH_CHECK(tab.scalar_type() == at::kLong && tab.dim() == 2 && tab.size(1) == 7 && tab.is_contiguous(),
              "scatter_scaled: table must be contiguous int64 [n, 7]");
  check_rc(rt_scatter_scaled((const long*)tab.data_ptr<int64_t>(), (int)tab.size(0), (long)max_elems, cur_stream()),
           "scatter_scaled");
}

// Full-parameter training of a bf16 model (ops.MixedFlatParams): bf16 gradients g16 of the first
// n16 elements + fp32 gradients g32 of the fp32 tail; fp32 master p and moments over all n; the bf16
// compute copy p16 of the first n16 elements is rewritten in the same pass.
void adamw_mixed(Tensor p, const Tensor& g16, const Tensor& g32, Tensor m, Tensor v, Tensor p16, double lr,
                 double b1, double b2, double eps, double wd, int64_t step, double max_norm, Tensor partials,
                 Tensor norm_out, Tensor skipped) {
  CHECK_CUDA(p); CHECK_F32(p); CHECK_BF16(g16); CHECK_F32(g32); CHECK_F32(m); CHECK_F32(v); CHECK_BF16(p16);
  CHECK_F32(partials);
  TORCH_CHECK(p.is_contiguous() && g16.is_contiguous() && g32.is_contiguous() && m.is_contiguous() &&
              v.is_contiguous() && p16.is_contiguous(), "adamw_mixed: buffers must be contiguous");
  const int64_t n = p.numel(), n16 = g16.numel();
  TORCH_CHECK(p16.numel() == n16 && n16 + g32.numel() == n && m.numel() == n && v.numel() == n,
              "adamw_mixed: sizes");
  TORCH_CHECK(n16 % 16 == 0 && (n - n16) % 4 == 0, "adamw_mixed: segments must be 16 / 4-element aligned");
  CHECK_ALIGN16(p); CHECK_ALIGN16(g16); CHECK_ALIGN16(m); CHECK_ALIGN16(v); CHECK_ALIGN16(p16);
  const int nparts = (int)partials.numel();
  const float* g32p = g32.numel() ? g32.data_ptr<float>() : nullptr;
  check_rc(rt_grad_sumsq_mixed(g16.data_ptr(), n16, g32p, n - n16, partials.data_ptr<float>(), nparts, cur_stream()),
           "grad_sumsq_mixed");
  check_rc(rt_adamw_mixed(p.data_ptr<float>(), g16.data_ptr(), n16, g32p, m.data_ptr<float>(), v.data_ptr<float>(),
                          p16.data_ptr(), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                          (float)max_norm, partials.data_ptr<float>(), nparts, norm_out.data_ptr<float>(),
                          skipped.data_ptr<int>(), cur_stream()),
           "adamw_mixed");
}

Tensor grad_norm(const Tensor& g, Tensor partials) {
  CHECK_CUDA(g); CHECK_F32(g);
  check_rc(rt_grad_sumsq(g.data_ptr<float>(), g.numel(), partials.data_ptr<float>(), (int)partials.numel(),
                         cur_stream()),
           "grad_sumsq");
  return partials.sum().sqrt();
}

// ---------------------------------------------------------------------------------------------
Tensor pool_norm(const Tensor& x, const optional<Tensor>& lengths, bool normalize) {
  CHECK_CUDA(x); CHECK_BF16(x); TORCH_CHECK(x.dim() == 3 && x.is_contiguous());
  const int64_t B = x.size(0), S = x.size(1), H = x.size(2);
  auto out = at::empty({B, H}, x.options().dtype(at::kFloat));
  if (lengths.has_value() && lengths->defined()) CHECK_I32(*lengths);
  check_rc(rt_pool_norm(x.data_ptr(), (const int*)opt_ptr(lengths), (int)B, (int)S, (int)H, normalize ? 1 : 0,
                        out.data_ptr<float>(), cur_stream()),
           "pool_norm");
  return out;
}

std::vector<Tensor> topk(const Tensor& scores, int64_t k, const optional<Tensor>& idmap) {
  CHECK_CUDA(scores); CHECK_F32(scores); CHECK_ROWS(scores);
  const int64_t nq = scores.size(0), N = scores.size(1);
  auto vals = at::empty({nq, k}, scores.options());
  auto ids = at::empty({nq, k}, scores.options().dtype(at::kLong));
  if (idmap.has_value() && idmap->defined()) { CHECK_I64(*idmap); CHECK_ROWS(*idmap); }
  check_rc(rt_topk(scores.data_ptr<float>(), scores.stride(0), nq, (int)N, (int)k, (const long*)opt_ptr(idmap),
                   idmap.has_value() && idmap->defined() ? idmap->stride(0) : 0, vals.data_ptr<float>(),
                   (long*)ids.data_ptr(), cur_stream()),
           "topk");
  return {vals, ids};
}

std::vector<Tensor> ivf_scan(const Tensor& q, const Tensor& probes, const Tensor& lstart, const Tensor& lsize,
                             const Tensor& vecs, const Tensor& ids, const optional<Tensor>& sqnorm, bool l2,
                             int64_t maxlen) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_I32(probes); CHECK_I32(lstart); CHECK_I32(lsize); CHECK_BF16(vecs); CHECK_I64(ids);
  TORCH_CHECK(q.is_contiguous() && probes.is_contiguous() && vecs.is_contiguous() && lstart.is_contiguous() &&
              lsize.is_contiguous());
  if (l2) { TORCH_CHECK(sqnorm.has_value() && sqnorm->defined(), "ivf_scan: l2 needs sqnorm"); CHECK_F32(*sqnorm); }
  const int64_t nq = q.size(0), d = q.size(1), nprobe = probes.size(1);
  auto cand = at::empty({nq, nprobe * maxlen}, q.options().dtype(at::kFloat));
  auto cid = at::empty({nq, nprobe * maxlen}, q.options().dtype(at::kLong));
  check_rc(rt_ivf_scan(q.data_ptr(), (int)nq, (int)d, probes.data_ptr<int>(), (int)nprobe, lstart.data_ptr<int>(),
                       lsize.data_ptr<int>(), vecs.data_ptr(), (const long*)ids.data_ptr(),
                       l2 ? sqnorm->data_ptr<float>() : nullptr, l2 ? 1 : 0, (int)maxlen, cand.data_ptr<float>(),
                       (long*)cid.data_ptr(), cur_stream()),
           "ivf_scan");
  return {cand, cid};
}

// mode bit 0: L2-normalise each segment mean; bit 1: segment sums instead of means
Tensor segment_mean(const Tensor& x, const Tensor& order, const Tensor& seg, int64_t mode, Tensor out) {
  CHECK_CUDA(x); CHECK_F32(x); CHECK_I64(order); CHECK_I32(seg); CHECK_F32(out);
  TORCH_CHECK(x.is_contiguous() && order.is_contiguous() && seg.is_contiguous() && out.is_contiguous());
  const int64_t k = seg.numel() - 1, d = x.size(1);
  TORCH_CHECK(out.size(0) == k && out.size(1) == d, "segment_mean: out shape");
  check_rc(rt_segment_mean(x.data_ptr<float>(), (int)d, (const long*)order.data_ptr(), seg.data_ptr<int>(), (int)k,
                           (int)mode, out.data_ptr<float>(), cur_stream()),
           "segment_mean");
  return out;
}

// (adv, returns, token rewards, per-sequence KL) of a rollout: see ppo_advantages_kernel
std::vector<Tensor> ppo_advantages(const Tensor& old_lp, const Tensor& ref_lp, const Tensor& values, const Tensor& score,
                                   const Tensor& len, double kl_coef, double gamma, double lam, bool whiten, double eps) {
  CHECK_CUDA(old_lp); CHECK_F32(old_lp); CHECK_F32(ref_lp); CHECK_F32(values); CHECK_F32(score); CHECK_I32(len);
  TORCH_CHECK(old_lp.is_contiguous() && ref_lp.is_contiguous() && values.is_contiguous() && score.is_contiguous() &&
              len.is_contiguous());
  const int64_t B = old_lp.size(0), T = old_lp.size(1);
  TORCH_CHECK(ref_lp.sizes() == old_lp.sizes() && values.sizes() == old_lp.sizes() && score.numel() == B &&
              len.numel() == B, "ppo_advantages: shapes");
  auto adv = at::empty_like(old_lp), ret = at::empty_like(old_lp), rew = at::empty_like(old_lp);
  auto kl = at::empty({B}, old_lp.options());
  check_rc(rt_ppo_advantages(old_lp.data_ptr<float>(), ref_lp.data_ptr<float>(), values.data_ptr<float>(),
                             score.data_ptr<float>(), len.data_ptr<int>(), (int)B, (int)T, (float)kl_coef, (float)gamma,
                             (float)lam, whiten ? 1 : 0, (float)eps, adv.data_ptr<float>(), ret.data_ptr<float>(),
                             rew.data_ptr<float>(), kl.data_ptr<float>(), cur_stream()),
           "ppo_advantages");
  return {adv, ret, rew, kl};
}

std::vector<Tensor> gae(const Tensor& rewards, const Tensor& values, const Tensor& mask, double gamma, double lam) {
  CHECK_CUDA(rewards); CHECK_F32(rewards); CHECK_F32(values); CHECK_F32(mask);
  TORCH_CHECK(rewards.is_contiguous() && values.is_contiguous() && mask.is_contiguous() && rewards.dim() == 2);
  auto adv = at::empty_like(rewards), ret = at::empty_like(rewards);
  check_rc(rt_gae(rewards.data_ptr<float>(), values.data_ptr<float>(), mask.data_ptr<float>(), (int)rewards.size(0),
                  (int)rewards.size(1), (float)gamma, (float)lam, adv.data_ptr<float>(), ret.data_ptr<float>(),
                  cur_stream()),
           "gae");
  return {adv, ret};
}

// fused token-level PPO objective: returns {stats[9], dlp, dv, dent} (see rl.hip); ``ref`` (optional,
// with kl_coef): the frozen reference's log-probs for the in-loss k3 KL penalty
std::vector<Tensor> ppo_loss(const Tensor& lp, const Tensor& old, const Tensor& adv, const Tensor& v,
                             const Tensor& ret, const optional<Tensor>& vold, const Tensor& ent, const Tensor& mask,
                             double eps, double c_v, double c_e, double vclip, const optional<Tensor>& ref,
                             double kl_coef) {
  for (const Tensor* t : {&lp, &old, &adv, &v, &ret, &ent, &mask}) {
    CHECK_CUDA(*t); CHECK_F32(*t);
    TORCH_CHECK(t->is_contiguous() && t->numel() == lp.numel(), "ppo_loss: operands must be contiguous, same size");
  }
  if (vclip > 0) {
    TORCH_CHECK(vold.has_value() && vold->defined() && vold->numel() == lp.numel() && vold->is_contiguous());
    CHECK_F32(*vold);
  }
  const bool has_ref = ref.has_value() && ref->defined();
  if (has_ref) {
    CHECK_CUDA(*ref); CHECK_F32(*ref);
    TORCH_CHECK(ref->is_contiguous() && ref->numel() == lp.numel(), "ppo_loss: ref must be contiguous, same size");
  }
  auto stats = at::zeros({9}, lp.options());
  auto dlp = at::empty_like(lp), dv = at::empty_like(lp), dent = at::empty_like(lp);
  check_rc(rt_ppo_loss(lp.data_ptr<float>(), old.data_ptr<float>(), adv.data_ptr<float>(), v.data_ptr<float>(),
                       ret.data_ptr<float>(), vclip > 0 ? vold->data_ptr<float>() : nullptr, ent.data_ptr<float>(),
                       mask.data_ptr<float>(), lp.numel(), (float)eps, (float)c_v, (float)c_e, (float)vclip,
                       has_ref ? ref->data_ptr<float>() : nullptr, (float)kl_coef, stats.data_ptr<float>(),
                       dlp.data_ptr<float>(), dv.data_ptr<float>(), dent.data_ptr<float>(), cur_stream()),
           "ppo_loss");
  return {stats, dlp, dv, dent};
}

// value head V = h . w + b per row (bf16 h [T, H], fp32 w [H], b [1]): batch-invariant row dot (loss.hip)
Tensor rowdot(const Tensor& h, const Tensor& w, const optional<Tensor>& b) {
  CHECK_CUDA(h); CHECK_CUDA(w); CHECK_F32(w);
  TORCH_CHECK(h.scalar_type() == at::kBFloat16 && h.dim() == 2 && h.stride(1) == 1, "rowdot: h bf16 [T, H] rows");
  TORCH_CHECK(w.is_contiguous() && w.numel() == h.size(1) && h.size(1) % 8 == 0, "rowdot: w [H], H % 8 == 0");
  TORCH_CHECK(((uintptr_t)h.data_ptr() % 16) == 0 && ((uintptr_t)w.data_ptr() % 16) == 0, "rowdot: 16-B alignment");
  if (b.has_value() && b->defined()) { CHECK_CUDA(*b); CHECK_F32(*b); }
  auto out = at::empty({h.size(0)}, h.options().dtype(at::kFloat));
  check_rc(rt_rowdot(h.data_ptr(), h.stride(0), w.data_ptr<float>(), (const float*)opt_ptr(b), (int)h.size(1),
                     h.size(0), out.data_ptr<float>(), cur_stream()),
           "rowdot");
  return out;
}

void decode_update(const Tensor& tok, Tensor out_tokens, const optional<Tensor>& out_logp,
                   const optional<Tensor>& logp, const optional<Tensor>& out_values, const optional<Tensor>& values,
                   Tensor active, Tensor kv_len, Tensor pos, Tensor next_input, Tensor gen_len, Tensor step,
                   Tensor rng_offset, const Tensor& eos_ids, int64_t pad_id, const optional<Tensor>& attn_len,
                   const optional<Tensor>& kv_start) {
  CHECK_I64(tok); CHECK_I64(out_tokens); CHECK_I32(kv_len); CHECK_I32(pos); CHECK_I64(next_input); CHECK_I32(gen_len);
  const bool al = attn_len.has_value() && attn_len->defined();
  if (al) {
    CHECK_I32(*attn_len);
    TORCH_CHECK(attn_len->numel() >= tok.numel(), "decode_update: attn_len");
  }
  if (kv_start.has_value() && kv_start->defined()) CHECK_I32(*kv_start);
  CHECK_I64(step); CHECK_I64(rng_offset); CHECK_I64(eos_ids);
  TORCH_CHECK(active.scalar_type() == at::kByte || active.scalar_type() == at::kBool);
  check_rc(rt_decode_update((const long*)tok.data_ptr(), (long*)out_tokens.data_ptr(), (int)out_tokens.size(1),
                            (float*)opt_ptr(out_logp), (const float*)opt_ptr(logp), (float*)opt_ptr(out_values),
                            (const float*)opt_ptr(values), (uint8_t*)active.data_ptr(), kv_len.data_ptr<int>(),
                            pos.data_ptr<int>(), (long*)next_input.data_ptr(), gen_len.data_ptr<int>(),
                            (int64_t*)step.data_ptr(), (int64_t*)rng_offset.data_ptr(), (int)tok.numel(),
                            (const long*)eos_ids.data_ptr(), (int)eos_ids.numel(), (long)pad_id,
                            al ? attn_len->data_ptr<int>() : nullptr, (const int*)opt_ptr(kv_start), cur_stream()),
           "decode_update");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) HIP kernels + native host runtime";
  m.def("decode_ws_dirty_tickets", &decode_ws_dirty_tickets, "per decode workspace: tickets not at zero");
  m.def("gemm", &gemm, "bf16 MFMA GEMM C = act(rstd(A) A W^T + U UB^T + bias) + R", py::arg("a"), py::arg("w"),
        py::arg("u") = py::none(), py::arg("ub") = py::none(), py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("out_f32") = false, py::arg("out") = py::none(), py::arg("residual") = py::none(),
        py::arg("norm_eps") = 0.0, py::arg("w_shuffled") = false);
  m.def("rows_scatter", &rows_scatter, "varlen: out[r] = src[inv[r]] (zeros where inv[r] < 0)", py::arg("src"),
        py::arg("inv"), py::arg("R"));
  m.def("shuffle_decode_weight", &shuffle_decode_weight, "W [N, K] -> tile-ordered decode image (gemm w_shuffled=True)",
        py::arg("w"), py::arg("out") = py::none());
  m.def("shuffle_decode_weight_fp8", &shuffle_decode_weight_fp8,
        "fp8 W [N, K] -> tile-ordered W8A16 decode image (gemm_fp8 w_shuffled=True)", py::arg("q"),
        py::arg("out") = py::none());
  m.def("get_tuning", &get_tuning, "the launchers' kernel-selection knobs (rt::Tuning) as a dict");
  m.def("set_tuning", &set_tuning, "update rt::Tuning fields from a dict (unknown keys raise)");
  m.def("attn_decode_fused", &attn_decode_fused, "RoPE + KV append + split-K decode attention + combine",
        py::arg("qkv"), py::arg("kc"), py::arg("vc"), py::arg("slot"), py::arg("attn_len"), py::arg("kv_start"),
        py::arg("pos"), py::arg("cos"), py::arg("sin"), py::arg("sign"), py::arg("window"), py::arg("scale"),
        py::arg("Hq"), py::arg("part"), py::arg("tickets"), py::arg("PS"), py::arg("out"),
        py::arg("k_scale") = py::none(), py::arg("v_scale") = py::none(), py::arg("stamps") = py::none());
  m.def("attn_decode_fused_slabs", &attn_decode_fused_slabs, "decode attention with the qkv split-K reduce fused",
        py::arg("slabs"), py::arg("nsplit"), py::arg("kc"), py::arg("vc"), py::arg("slot"), py::arg("attn_len"),
        py::arg("kv_start"), py::arg("pos"), py::arg("cos"), py::arg("sin"), py::arg("sign"), py::arg("window"),
        py::arg("scale"), py::arg("Hq"), py::arg("part"), py::arg("tickets"), py::arg("PS"), py::arg("out"),
        py::arg("k_scale") = py::none(), py::arg("v_scale") = py::none());
  m.def("gemm_fp8_lora", &gemm_fp8_lora, "W8A8 GEMM + bf16 LoRA K-extension (config-5 training forward)");
  m.def("kv_store_fp8", &kv_store_fp8, "prompt K/V -> fp8 cache (per-slot scales)");
  m.def("attn_decode_fused_ps", &rt_attn_decode_fused_ps, "keys per partition of the fused decode kernel");
  m.def("quant_fp8", &quant_fp8, "per-row absmax e4m3fn quantisation -> (uint8 [R,C], scale fp32 [R])");
  m.def("gemm_big", &gemm_big, "token-parallel GEMM family (NT / NN / TN, LoRA K-extension, split-K, SwiGLU)",
        py::arg("a"), py::arg("b"), py::arg("layout_a"), py::arg("layout_b"), py::arg("a2") = py::none(),
        py::arg("b2") = py::none(), py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("out_mode") = 0,
        py::arg("nsplit") = 1, py::arg("out") = py::none(), py::arg("out2") = py::none(),
        py::arg("residual") = py::none(), py::arg("bn") = 0);
  m.def("gemm_rope", &gemm_rope, "NT GEMM with the rotary embedding of the q / k heads in the epilogue", py::arg("a"),
        py::arg("w"), py::arg("u") = py::none(), py::arg("ub") = py::none(), py::arg("bias") = py::none(),
        py::arg("pos"), py::arg("cos"), py::arg("sin"), py::arg("rope_cols"), py::arg("head_dim"),
        py::arg("out") = py::none(), py::arg("bn") = 0);
  m.def("gemm_splitk", &gemm_splitk, "small-M NT GEMM: split-K fp32 slabs + fused reduce epilogue", py::arg("a"),
        py::arg("w"), py::arg("nsplit"), py::arg("slabs"), py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("out") = py::none(), py::arg("residual") = py::none(), py::arg("bn") = 256);
  m.def("gemm_small", &gemm_small, "64x64-tile GEMM for narrow (LoRA) products", py::arg("a"), py::arg("b"),
        py::arg("layout_a"), py::arg("layout_b"), py::arg("out_mode") = 0, py::arg("nsplit") = 1,
        py::arg("out") = py::none(), py::arg("bm") = 64);
  m.def("gemm_fp8", &gemm_fp8, "fp8 GEMM: W8A8 (MX MFMA 256x256) or W8A16 (skinny, M <= 64)", py::arg("a"),
        py::arg("sa") = py::none(), py::arg("wq"), py::arg("sw"), py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("out") = py::none(), py::arg("residual") = py::none(), py::arg("norm_eps") = 0.0,
        py::arg("w_shuffled") = false);
  m.def("norm_fwd", &norm_fwd);
  m.def("splitk_reduce", &splitk_reduce, "sum of split-K slabs -> bf16");
  m.def("norm_fwd_slabs", &norm_fwd_slabs, "residual-add + norm whose input is a sum of split-K slabs");
  m.def("gemm_splitk_raw", &gemm_splitk_raw, "split-K NT GEMM into fp32 slabs (reduce fused into the consumer)");
  m.def("gemm_fp8_splitk_raw", &gemm_fp8_splitk_raw, "W8A8 split-K NT GEMM into fp32 slabs (scales applied per split)");
  m.def("norm_bwd", &norm_bwd);
  m.def("rope_qkv", &rope_qkv);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("embed", &embed);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_decode", &attn_decode);
  m.def("attn_bwd", &attn_bwd, "flash attention backward (RoPE backward optionally fused into dQ / dK)",
        py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"), py::arg("lse"), py::arg("dq"),
        py::arg("dk"), py::arg("dv"), py::arg("B"), py::arg("S"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"),
        py::arg("causal"), py::arg("window"), py::arg("scale"), py::arg("kv_start") = py::none(),
        py::arg("rope_pos") = py::none(), py::arg("rope_cos") = py::none(), py::arg("rope_sin") = py::none());
  m.def("logprob_fwd", &logprob_fwd);
  m.def("logprob_bwd", &logprob_bwd);
  m.def("sample", &sample);
  m.def("adamw", &adamw);
  m.def("scatter_scaled", &scatter_scaled, "batched scaled fp32 -> bf16 strided scatter (LoRA images)");
  m.def("lora_grad_accum", &lora_grad_accum, "LoRA backward: scaled sum of adapter-gradient slabs into grads");
  m.def("adamw_mixed", &adamw_mixed);
  m.def("grad_norm", &grad_norm);
  m.def("adamw_apply", &adamw_apply);
  m.def("grad_sumsq", &grad_sumsq);
  m.def("pool_norm", &pool_norm);
  m.def("topk", &topk);
  m.def("ivf_scan", &ivf_scan);
  m.def("segment_mean", &segment_mean, "k-means update: per-segment mean of sorted rows (+ L2 normalise)");
  m.def("gae", &gae);
  m.def("ppo_advantages", &ppo_advantages, "token KL rewards + GAE + advantage whitening in one launch");
  m.def("ppo_loss", &ppo_loss, "fused token-level PPO loss: {stats[9], dlp, dv, dent}");
  m.def("rowdot", &rowdot, "value head: batch-invariant per-row dot product");
  m.def("decode_update", &decode_update);
  ragtl::bind_tokenizer(m);
  ragtl::bind_ivf_host(m);
}
