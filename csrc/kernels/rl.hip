// RL kernels: token-level GAE reverse scan, and the decode-step bookkeeping kernel
// that keeps a hipGraph-captured generation loop free of host round trips.
//
// GAE follows reinforcement_learning_optimization_after_rag.py:176-191 (delta = r + g*V' - V,
// A = delta + g*lam*A') but over the tokens of each response instead of across batch samples, with
// lam a parameter (reference hard-codes 0.95) and padding tokens masked out.
#include "rt_common.h"

namespace rt {

__global__ void gae_kernel(const float* __restrict__ rewards, const float* __restrict__ values,
                           const float* __restrict__ mask, int B, int T, float gamma, float lam,
                           float* __restrict__ adv, float* __restrict__ ret) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float nextv = 0.f, last = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const long i = (long)b * T + t;
    if (mask[i] == 0.f) {
      adv[i] = 0.f;
      ret[i] = 0.f;
      continue;
    }
    const float v = values[i];
    const float delta = rewards[i] + gamma * nextv - v;
    last = delta + gamma * lam * last;
    adv[i] = last;
    ret[i] = last + v;
    nextv = v;
  }
}

// PPO advantages in one launch (one workgroup; a thread per sequence, then block reductions):
//   kl[b,t]   = old_logp - ref_logp                      (t < len[b])
//   r[b,t]    = -kl_coef kl + (t == len[b] - 1) score[b]  (reward at the last response token)
//   GAE over r with V = old values (the reverse scan of gae_kernel)
//   whiten: adv = (adv - mean) / sqrt(var + eps) over the valid tokens (masked_whiten)
//   kl_seq[b] = sum_t kl                                  (the KL-to-reference statistic)
// Replaces ~15 small ATen launches between the reference forward and the update
// (reinforcement_learning_optimization_after_rag.py:176-191 GAE, with the SURVEY B3 KL term).
__global__ __launch_bounds__(256) void ppo_advantages_kernel(const float* __restrict__ old_lp, const float* __restrict__ ref_lp,
                                                             const float* __restrict__ values, const float* __restrict__ score,
                                                             const int* __restrict__ len, int B, int T, float kl_coef,
                                                             float gamma, float lam, int whiten, float eps,
                                                             float* __restrict__ adv, float* __restrict__ ret,
                                                             float* __restrict__ rew, float* __restrict__ kl_seq) {
  __shared__ float sb[4];
  float s1 = 0.f, n = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int L = min(max(len[b], 0), T);
    float nextv = 0.f, last = 0.f, klsum = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const long i = (long)b * T + t;
      if (t >= L) {
        adv[i] = 0.f; ret[i] = 0.f; rew[i] = 0.f;
        continue;
      }
      const float kl = old_lp[i] - ref_lp[i];
      klsum += kl;
      const float r = -kl_coef * kl + (t == L - 1 ? score[b] : 0.f);
      rew[i] = r;
      const float v = values[i];
      const float delta = r + gamma * nextv - v;
      last = delta + gamma * lam * last;
      adv[i] = last;
      ret[i] = last + v;
      nextv = v;
      s1 += last;
    }
    n += (float)L;
    kl_seq[b] = klsum;
  }
  if (!whiten) return;
  const float tot = block_sum(s1, sb);
  const float cnt = block_sum(n, sb);
  const float mean = tot / fmaxf(cnt, 1.f);
  float s2 = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int L = min(max(len[b], 0), T);
    for (int t = 0; t < L; ++t) {
      const float d = adv[(long)b * T + t] - mean;
      s2 += d * d;
    }
  }
  const float var = block_sum(s2, sb) / fmaxf(cnt, 1.f);
  const float inv = rsqrtf(var + eps);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int L = min(max(len[b], 0), T);
    for (int t = 0; t < L; ++t) {
      const long i = (long)b * T + t;
      adv[i] = (adv[i] - mean) * inv;
    }
  }
}

// After sampling token `tok[b]` at decode step `step`: record it, update finished flags (eos or
// length budget), advance per-row cache length/position, bump the RNG offset and step counter.
// Rows that are finished keep emitting pad and stop advancing.
__global__ void decode_update_kernel(const long* __restrict__ tok, long* __restrict__ out_tokens, int max_new,
                                     float* __restrict__ out_logp, const float* __restrict__ logp,
                                     float* __restrict__ out_values, const float* __restrict__ values,
                                     uint8_t* __restrict__ active, int* __restrict__ kv_len, int* __restrict__ pos,
                                     long* __restrict__ next_input, int* __restrict__ gen_len,
                                     int64_t* __restrict__ step, int64_t* __restrict__ rng_offset, int B,
                                     const long* __restrict__ eos_ids, int n_eos, long pad_id,
                                     int* __restrict__ attn_len, const int* __restrict__ kv_start) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = *step;
  if (b < B) {
    const bool act = active[b] != 0;
    long t = tok[b];
    // the row's own output position: equal to the step counter for every active row of a static
    // batch (rows start together and never reactivate); rows admitted mid-flight by continuous
    // batching start at 0
    const int sr = gen_len[b];
    if (act && sr < max_new) {
      out_tokens[(long)b * max_new + sr] = t;
      if (out_logp) out_logp[(long)b * max_new + sr] = logp[b];
      if (out_values && values) out_values[(long)b * max_new + sr] = values[b];
      gen_len[b] = sr + 1;
      bool fin = (sr + 1 >= max_new);
      for (int e = 0; e < n_eos; ++e) fin = fin || (t == eos_ids[e]);
      if (fin) active[b] = 0;
      kv_len[b] += 1;
      pos[b] += 1;
      next_input[b] = t;
    } else {
      next_input[b] = pad_id;
    }
    // the next step's attention length and rotary position (kept here, not as two extra
    // elementwise launches at the head of every decode step)
    if (attn_len) {
      const int kl = kv_len[b];
      attn_len[b] = kl + 1;
      pos[b] = kl - (kv_start ? kv_start[b] : 0);
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *step = s + 1;
    *rng_offset = *rng_offset + 1;
  }
}

// Token-level PPO objective over [B, T] (masked mean over the n response tokens), forward AND its
// closed-form gradient in one single-workgroup launch (a minibatch holds a few thousand tokens):
//   pg   = mean(-min(r A, clip(r, 1 +- eps) A)),  r = exp(lp - old)
//   vl   = 0.5 mean((v - R)^2)   [value_clip > 0: 0.5 mean(max((v - R)^2, (vc - R)^2)),
//                                 vc = v_old + clamp(v - v_old, +-value_clip)]
//   ent  = mean(entropy);  loss = pg + c_v vl - c_e ent
//   stats[0..5] = loss, pg, vl, ent, approx_kl = mean(old - lp), clipfrac = mean(|r - 1| > eps)
//   ref != null (KL to the frozen reference in the loss, PPOConfig.kl_in_loss): with d = ref - lp,
//   loss += kl_coef mean(k3), k3 = e^d - d - 1 (the non-negative, unbiased-in-expectation
//   estimator of KL(pi || ref) on tokens drawn from pi); stats[6] = mean(k3), stats[7] =
//   mean(lp - ref) (k1); stats[8] = n (masked tokens); d k3 / d lp = 1 - e^d
//   dlp = d loss / d lp, dv = d loss / d v, dent = d loss / d entropy (per token, 0 off the mask)
// Formulas: reference PPOTrainer.ppo_update (reinforcement_learning_optimization_after_rag.py:212-225)
// at token level, with the SURVEY B5 true-entropy fix. Replaces ~25 tiny elementwise/reduction
// launches (and as many in the backward) per minibatch with one.
__global__ __launch_bounds__(1024) void ppo_loss_kernel(
    const float* __restrict__ lp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ v, const float* __restrict__ ret, const float* __restrict__ vold,
    const float* __restrict__ ent, const float* __restrict__ mask, long n_el, float eps, float c_v, float c_e,
    float vclip, const float* __restrict__ ref, float kl_coef, float* __restrict__ stats, float* __restrict__ dlp,
    float* __restrict__ dv, float* __restrict__ dent) {
  constexpr int NA = 8;
  __shared__ float red[16][NA];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float acc[NA] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // n, pg, vl, ent, kl, clipfrac, k3, k1 (sums)
  for (long i = tid; i < n_el; i += 1024) {
    const float m = mask[i];
    if (m == 0.f) continue;
    const float r = __expf(lp[i] - old[i]);
    const float A = adv[i];
    const float rc = fminf(fmaxf(r, 1.f - eps), 1.f + eps);
    acc[0] += m;
    acc[1] += m * fmaxf(-r * A, -rc * A);
    const float dvv = v[i] - ret[i];
    float vterm = dvv * dvv;
    if (vclip > 0.f) {
      const float vc = vold[i] + fminf(fmaxf(v[i] - vold[i], -vclip), vclip);
      vterm = fmaxf(vterm, (vc - ret[i]) * (vc - ret[i]));
    }
    acc[2] += m * vterm;
    acc[3] += m * ent[i];
    acc[4] += m * (old[i] - lp[i]);
    acc[5] += m * (fabsf(r - 1.f) > eps ? 1.f : 0.f);
    if (ref) {
      const float d = ref[i] - lp[i];
      acc[6] += m * (__expf(d) - d - 1.f);
      acc[7] -= m * d;
    }
  }
#pragma unroll
  for (int k = 0; k < NA; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NA; ++k) red[wid][k] = acc[k];
  __syncthreads();
  float tot[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][k];
    tot[k] = t;
  }
  const float inv_n = 1.f / fmaxf(tot[0], 1.f);
  if (tid == 0) {
    const float pg = tot[1] * inv_n, vl = 0.5f * tot[2] * inv_n, em = tot[3] * inv_n;
    const float k3 = tot[6] * inv_n;
    stats[0] = pg + c_v * vl - c_e * em + (ref && kl_coef != 0.f ? kl_coef * k3 : 0.f);
    stats[1] = pg;
    stats[2] = vl;
    stats[3] = em;
    stats[4] = tot[4] * inv_n;
    stats[5] = tot[5] * inv_n;
    stats[6] = k3;
    stats[7] = tot[7] * inv_n;
    stats[8] = tot[0];
  }
  for (long i = tid; i < n_el; i += 1024) {
    const float m = mask[i];
    float g_lp = 0.f, g_v = 0.f, g_e = 0.f;
    if (m != 0.f) {
      const float r = __expf(lp[i] - old[i]);
      const float A = adv[i];
      const float rc = fminf(fmaxf(r, 1.f - eps), 1.f + eps);
      // -min(rA, rc A): the unclipped branch is active (or tied) -> d/dlp = -A r; the clipped branch
      // only differs when r is outside the range, where clamp has no gradient
      g_lp = (r * A <= rc * A) ? -A * r : 0.f;
      if (ref && kl_coef != 0.f) g_lp += kl_coef * (1.f - __expf(ref[i] - lp[i]));
      const float dvv = v[i] - ret[i];
      float gv = dvv;
      if (vclip > 0.f) {
        const float d0 = v[i] - vold[i];
        const float vc = vold[i] + fminf(fmaxf(d0, -vclip), vclip);
        if ((vc - ret[i]) * (vc - ret[i]) > dvv * dvv) gv = (fabsf(d0) < vclip) ? (vc - ret[i]) : 0.f;
      }
      g_v = c_v * gv;  // d(0.5 x^2)/dx = x
      g_e = -c_e;
      g_lp *= m * inv_n;
      g_v *= m * inv_n;
      g_e *= m * inv_n;
    }
    dlp[i] = g_lp;
    dv[i] = g_v;
    dent[i] = g_e;
  }
}

}  // namespace rt

using namespace rt;

extern "C" int rt_ppo_loss(const float* lp, const float* old, const float* adv, const float* v, const float* ret,
                           const float* vold, const float* ent, const float* mask, long n_el, float eps, float c_v,
                           float c_e, float vclip, const float* ref, float kl_coef, float* stats, float* dlp,
                           float* dv, float* dent, hipStream_t stream) {
  hipLaunchKernelGGL(ppo_loss_kernel, dim3(1), dim3(1024), 0, stream, lp, old, adv, v, ret, vold, ent, mask, n_el,
                     eps, c_v, c_e, vclip, ref, kl_coef, stats, dlp, dv, dent);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_gae(const float* rewards, const float* values, const float* mask, int B, int T, float gamma, float lam,
                      float* adv, float* ret, hipStream_t stream) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(gae_kernel, dim3((B + 63) / 64), dim3(64), 0, stream, rewards, values, mask, B, T, gamma, lam, adv,
                     ret);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_ppo_advantages(const float* old_lp, const float* ref_lp, const float* values, const float* score,
                                 const int* len, int B, int T, float kl_coef, float gamma, float lam, int whiten,
                                 float eps, float* adv, float* ret, float* rew, float* kl_seq, hipStream_t stream) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(ppo_advantages_kernel, dim3(1), dim3(256), 0, stream, old_lp, ref_lp, values, score, len, B, T,
                     kl_coef, gamma, lam, whiten, eps, adv, ret, rew, kl_seq);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_decode_update(const long* tok, long* out_tokens, int max_new, float* out_logp, const float* logp,
                                float* out_values, const float* values, uint8_t* active, int* kv_len, int* pos,
                                long* next_input, int* gen_len, int64_t* step, int64_t* rng_offset, int B,
                                const long* eos_ids, int n_eos, long pad_id, int* attn_len, const int* kv_start,
                                hipStream_t stream) {
  if (B > 1024) return -1;
  hipLaunchKernelGGL(decode_update_kernel, dim3(1), dim3(((B + 63) / 64) * 64), 0, stream, tok, out_tokens, max_new,
                     out_logp, logp, out_values, values, active, kv_len, pos, next_input, gen_len, step, rng_offset, B,
                     eos_ids, n_eos, pad_id, attn_len, kv_start);
  RT_LAUNCH_CHECK();
  return 0;
}
