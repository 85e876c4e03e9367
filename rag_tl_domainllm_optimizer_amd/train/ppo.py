"""PPO after RAG (config 4): rollout -> reward -> frozen-reference KL -> token GAE -> clipped update.

Reference: PPOTrainer / RLTrainer (reinforcement_learning_optimization_after_rag.py:127-363). Kept:
hyper-parameter defaults (lr 5e-5, gamma 0.99, clip 0.2, value coef 0.5, entropy coef 0.01,
max grad norm 0.5, GAE lambda 0.95, AdamW wd 0.01), the reward, the 10 logged metric keys and the
checkpoint artifacts. Fixed: rollouts come from the current policy on the GPU (B2)
with the same RAG prompt that is trained on (B3); log-probs are per response token (B1); the
frozen reference enters as a per-token KL penalty (B4; the reference is the base weights with LoRA
disabled, no third model copy); "entropy" is the true token entropy (B5); values are read at the
last real position (B6) from the same forward as the log-probs (B7); GAE runs over tokens (B8).
Trainables: LoRA adapters + value head (default), or every policy weight (``full_finetune``, the
reference's mode: bf16 compute copies + fp32 master, ops.MixedFlatParams, frozen reference copy).

Device flow per step (one process per GPU, DP over RCCL):
  generate (hipGraph decode, behaviour log-probs + values emitted by the sampler step)
  -> reference log-probs (LoRA off, no grad) on the main stream
     || reward: rollout tokens reach the host right after the rollout, the host detokenises while
        the reference forward runs, the reward encoder runs on a side stream (``overlap_reward``)
  -> token rewards / GAE kernel
  -> ppo_epochs x minibatches of (forward, backward with bucketed all-reduce, fused AdamW).
"""
from __future__ import annotations

import copy
import math
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..generation import Generator, SamplingParams
from ..models import ValueHead
from ..parallel import GradSync, info as dist_info, reduce_metrics
from ..parallel.zero import ZeroAdamW, zero_enabled
from ..rag.prompt import build_prompt, encode_prompt, extract_answer
from ..runtime import PhaseTimer, StreamPair
from ..utils import MetricsSink, maybe_inject_fault
from .common import lr_at, score_sequences


@dataclass
class PPOConfig:
    lr: float = 5e-5                     # rl.py:132
    gamma: float = 0.99                  # rl.py:133
    lam: float = 0.95                    # rl.py:188 (hard-coded there)
    clip_range: float = 0.2              # rl.py:134
    value_coef: float = 0.5              # rl.py:135
    entropy_coef: float = 0.01           # rl.py:136
    max_grad_norm: float = 0.5           # rl.py:137
    weight_decay: float = 0.01           # torch AdamW default (rl.py:153)
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    value_clip: Optional[float] = None
    kl_coef: float = 0.05
    # where the frozen-reference KL penalty is applied: True = in the loss, as
    # kl_coef * mean_t k3(pi_theta || ref) on the update forward's own log-probs (training
    # numerics, the same batch-invariant scoring forward as the reference log-probs: exactly 0 at
    # LoRA B = 0, no extra forward); False = as a -kl_coef * (old - ref) per-token reward term,
    # where "old" are the old_logp below (with "rollout" these are the sampler's log-probs, whose
    # engine gap to the training forward then reads as KL: 1.83 nats / sequence at init,
    # profiles/r5/bench_old_logp_recompute.log)
    kl_in_loss: bool = True
    adaptive_kl: bool = False
    target_kl: float = 6.0
    kl_horizon: int = 10000
    ppo_epochs: int = 1                  # reference: one update per batch (rl.py:328)
    minibatch_size: int = 16
    ref_minibatch_size: int = 128       # reference log-prob scoring (no grad): 38k-token GEMMs (0.895 -> 0.879 s, profiles/r5/bench_ref_minibatch_ab.log)
    whiten_advantages: bool = True
    # generation (rl.py:38-44)
    max_new_tokens: int = 128
    temperature: float = 0.7
    top_k: int = 50
    top_p: float = 1.0
    max_prompt_tokens: int = 384
    # adapters
    lora_r: int = 16
    lora_alpha: float = 32.0
    lora_targets: Sequence[str] = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
    full_finetune: bool = False         # True: every weight (the reference's mode, rl.py:153)
    zero: bool = True                   # full_finetune at world > 1: ZeRO-1 sharded fp32 optimizer state
    gradient_checkpointing: bool = False
    overlap_reward: bool = True      # reward encoder on a side stream beside the reference forward
    rollout_chunks: int = 1          # >1: score chunk i while chunk i+1 decodes
    merged_lora_rollout: bool = True  # decode/prefill rollouts on W + sBA (refreshed per update)
    # where the PPO ratio's theta_old log-probs / values come from: "rollout" = the sampler of the
    # decode engine, i.e. the behaviour policy mu that drew the tokens (free; the importance ratio
    # pi_theta / mu then also corrects the two engines' bf16 numerics, ~0.09 nats / token on a
    # random-init Mistral-7B, profiles/r5/behaviour_gap_7b.log), or "recompute" = one no-grad
    # forward of the policy over the rollouts in the update forward's exact numerics (the
    # batch-invariant scoring forward: ratio bitwise 1 at theta = theta_old; costs a forward)
    old_logp: str = "rollout"
    lr_schedule: str = "constant"
    save_every: int = 0              # CLI: mid-epoch "latest" checkpoint every N steps (0 = epoch ends)
    save_full_policy: bool = True    # epoch / best checkpoints also write the merged HF policy
    bucket_mb: float = 64.0
    warmup_steps: int = 0
    total_steps: int = 0
    seed: int = 0


def _event():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


class _nullcontext:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class AdaptiveKL:
    """TRL-style proportional KL controller."""

    def __init__(self, init: float, target: float, horizon: int):
        self.value, self.target, self.horizon = init, target, horizon

    def update(self, current_kl: float, n_steps: int):
        err = float(np.clip(current_kl / self.target - 1, -0.2, 0.2))
        self.value *= 1 + err * n_steps / self.horizon


@dataclass
class Rollout:
    prompt_ids: torch.Tensor
    start: torch.Tensor
    resp: torch.Tensor
    resp_len: torch.Tensor
    old_logp: torch.Tensor
    old_values: torch.Tensor
    scores: torch.Tensor
    components: dict
    responses: List[str]
    queries: List[str]
    ref_logp: Optional[torch.Tensor] = None
    adv: Optional[torch.Tensor] = None
    returns: Optional[torch.Tensor] = None
    rewards_tok: Optional[torch.Tensor] = None
    n_tokens: int = 0
    kl_old_ref: Optional[torch.Tensor] = None  # per-sequence mean of sum_t (old - ref)
    # host copies of (start, resp_len) for the varlen (packed) scoring forwards
    host_lengths: Optional[tuple] = None


class PPOTrainer:
    def __init__(self, policy, tokenizer, reward_model, cfg: Optional[PPOConfig] = None, value_head=None,
                 sink: Optional[MetricsSink] = None, max_batch: int = 64):
        self.cfg = cfg or PPOConfig()
        c = self.cfg
        self.policy = policy
        self.tok = tokenizer
        self.reward_model = reward_model
        self.device = policy.embed.device
        self.sink = sink or MetricsSink(enabled=False)
        if c.full_finetune:
            # the reference's mode (rl.py:140-174): AdamW over EVERY policy weight and the value
            # head; the frozen reference is then a copy of the starting weights (the LoRA mode needs
            # no copy: reference = adapters off)
            from ..models.lora import merge_and_drop_lora

            merge_and_drop_lora(policy)
            self.ref_policy = copy.deepcopy(policy).requires_grad_(False)
            policy.requires_grad_(True)
            trainable = list(policy.parameters())
        else:
            self.ref_policy = None
            if getattr(policy, "lora_config", None) is None:
                policy.add_lora(c.lora_r, c.lora_alpha, list(c.lora_targets), seed=c.seed)
            policy.freeze_base()
            trainable = list(policy.lora_parameters())
        self.value_head = value_head or ValueHead(policy.cfg.hidden_size, device=self.device, seed=c.seed + 17)
        # trainables + value head re-homed into one flat buffer (fused AdamW, bucketed all-reduce):
        # fp32 LoRA adapters, or bf16 compute copies + fp32 master under full fine-tuning
        if zero_enabled(c.full_finetune, c.zero) and any(p.dtype == torch.bfloat16 for p in trainable):
            # ZeRO-1 (parallel.zero): each rank keeps the fp32 master / moments of 1/N of every
            # bucket; fp32 reduce-scatter of the gradients, bf16 all-gather of the updated weights
            w = dist_info().world
            self.flat = ops.flat_params(trainable + list(self.value_head.parameters()), align=16 * w,
                                        keep_master=False)
            self.opt = ZeroAdamW(self.flat, lr=c.lr, betas=c.betas, eps=c.eps, weight_decay=c.weight_decay,
                                 max_grad_norm=c.max_grad_norm, bucket_bytes=int(4 * c.bucket_mb * (1 << 20)))
            self.sync = self.opt.sync
        else:
            self.flat = ops.flat_params(trainable + list(self.value_head.parameters()))
            self.opt = ops.FusedAdamW(self.flat, lr=c.lr, betas=c.betas, eps=c.eps, weight_decay=c.weight_decay,
                                      max_grad_norm=c.max_grad_norm)
            self.sync = GradSync(self.flat, bucket_bytes=int(c.bucket_mb * (1 << 20)))
        policy.refresh_lora()
        self.kl = AdaptiveKL(c.kl_coef, c.target_kl, c.kl_horizon) if c.adaptive_kl else None
        self.max_batch = max_batch
        self.gen = Generator(policy, max_batch, c.max_prompt_tokens + c.max_new_tokens + 8, self.device,
                             value_head=self.value_head)
        self.gen.merge_lora = c.merged_lora_rollout
        self.sampling = SamplingParams(max_new_tokens=c.max_new_tokens, temperature=c.temperature, top_k=c.top_k,
                                       top_p=c.top_p, do_sample=True, seed=c.seed + 1000 * dist_info().rank)
        self.streams = StreamPair(self.device)
        self.timer = PhaseTimer(device=self.device)
        self.global_step = 0
        # set record_overlap_events = True to get HIP events of the reference forward / reward
        # encoder (tests and traces check that the two really overlap)
        self.record_overlap_events = False
        self.overlap_events: Dict[str, torch.cuda.Event] = {}

    @property
    def kl_coef(self):
        return self.kl.value if self.kl is not None else self.cfg.kl_coef

    # ------------------------------------------------------------------ prompts
    def encode_prompts(self, queries: Sequence[str], docs: Sequence[Sequence[str]]) -> List[List[int]]:
        # drop lowest-ranked docs until the prompt fits (SURVEY 5.7 d)
        return [encode_prompt(self.tok, q, ds, self.cfg.max_prompt_tokens) for q, ds in zip(queries, docs)]

    # ------------------------------------------------------------------ rollout + reward
    @torch.no_grad()
    def rollout(self, batch: Dict[str, list]) -> Rollout:
        """Generate responses. With ``rollout_chunks > 1`` the reward of chunk i is scored on the side
        stream while chunk i+1 decodes; with one chunk the reward is deferred to ``prepare`` where
        it overlaps the reference forward (one full-batch decode reads the weights half as often)."""
        c = self.cfg
        queries, docs = batch["query"], batch["retrieved_docs"]
        gts = batch.get("ground_truth") or [None] * len(queries)
        prompts = self.encode_prompts(queries, docs)
        B = len(prompts)
        n_chunks = max(1, min(c.rollout_chunks, B))
        bounds = [(i * B // n_chunks, (i + 1) * B // n_chunks) for i in range(n_chunks)]
        outs, pending = [], []

        def score_chunk(lo, hi, out):
            texts = self._texts(out)
            with self.streams.on_side():
                r, comp = self.reward_model.score(texts, queries[lo:hi], docs[lo:hi], gts[lo:hi])
            pending.append((lo, hi, texts, r, comp))

        if c.merged_lora_rollout:
            self.policy.set_lora_merged(True)
        try:
            with self.timer.phase("rollout"):
                prev = None
                for lo, hi in bounds:
                    # "async": the decode stops once every row has emitted EOS (checked behind
                    # events, two chunks ahead of the GPU; HF generate's stop rule, rl.py:38-44)
                    handle = self.gen.generate_async(prompts[lo:hi], self.sampling, pad_id=self.tok.pad_token_id,
                                                     eos_ids=[self.tok.eos_token_id], early_stop="async")
                    if prev is not None:
                        score_chunk(*prev)
                    out = handle.result()
                    outs.append(out)
                    prev = (lo, hi, out)
                if n_chunks > 1:
                    score_chunk(*prev)
                    self.streams.join()
        finally:
            self.policy.set_lora_merged(False)
        T = max(o.tokens.shape[1] for o in outs)
        S = max(o.prompt_ids.shape[1] for o in outs)
        pad = self.tok.pad_token_id

        def cat_pad(ts, width, left, value):
            res = []
            for t in ts:
                d = width - t.shape[1]
                if d:
                    p = torch.full((t.shape[0], d), value, dtype=t.dtype, device=t.device)
                    t = torch.cat([p, t], 1) if left else torch.cat([t, p], 1)
                res.append(t)
            return torch.cat(res, 0)

        ro = Rollout(cat_pad([o.prompt_ids for o in outs], S, True, pad),
                     torch.cat([o.prompt_start + (S - o.prompt_ids.shape[1]) for o in outs], 0),
                     cat_pad([o.tokens for o in outs], T, False, pad), torch.cat([o.lengths for o in outs], 0),
                     cat_pad([o.logprobs for o in outs], T, False, 0.0),
                     cat_pad([o.values for o in outs], T, False, 0.0), None, {}, [], list(queries))
        # generation has completed (result() waited): one small D2H copy of the response lengths
        rl_host = ro.resp_len.cpu().numpy()
        ro.host_lengths = (np.array([S - len(p) for p in prompts], dtype=np.int64), rl_host.astype(np.int64))
        ro.n_tokens = int(rl_host.sum())
        ro._outs, ro._pending, ro._batch = outs, pending, (queries, docs, gts)
        if not pending:
            # generation is complete here (result() waited): one D2H copy per output while the GPU
            # is idle; detokenisation happens later, beside the reference forward
            ro._host = [(o.tokens.cpu(), o.lengths.cpu()) for o in outs]
        return ro

    def _texts(self, out, host=None) -> List[str]:
        toks, lens = host if host is not None else (out.tokens.cpu(), out.lengths.cpu())
        lens = lens.tolist()
        return [extract_answer(self.tok.decode(toks[b, :lens[b]].tolist())) for b in range(toks.shape[0])]

    def _score_now(self, ro: Rollout, side: bool):
        """Detokenise the (host-resident) rollout and run the reward encoder — on the side stream
        when ``side`` (it then runs beside whatever the main stream has queued)."""
        queries, docs, gts = ro._batch
        host = getattr(ro, "_host", None) or [None] * len(ro._outs)
        texts = sum((self._texts(o, h) for o, h in zip(ro._outs, host)), [])
        with self.streams.on_side() if side else _nullcontext():
            if self.record_overlap_events and self.device.type == "cuda":
                self.overlap_events["reward_start"] = _event()
            r, comp = self.reward_model.score(texts, queries, docs, gts)
            if self.record_overlap_events and self.device.type == "cuda":
                self.overlap_events["reward_end"] = _event()
        ro._pending = [(0, len(texts), texts, r, comp)]

    def _collect_rewards(self, ro: Rollout):
        if not ro._pending:
            self._score_now(ro, side=True)
        self.streams.join()
        B = ro.resp.shape[0]
        scores = torch.zeros(B, device=self.device)
        comps_all, texts_all = {}, []
        for lo, hi, texts, r, comp in ro._pending:
            scores[lo:hi] = r
            texts_all += texts
            for k, v in comp.items():
                comps_all.setdefault(k, []).append(v)
        ro.scores = scores
        ro.responses = texts_all
        ro.components = {k: (torch.cat(v) if isinstance(v[0], torch.Tensor) else sum(v, [])) for k, v in comps_all.items()}

    # ------------------------------------------------------------------ reference KL, GAE
    @torch.no_grad()
    def prepare(self, ro: Rollout):
        """Frozen-reference log-probs (main stream) overlapped with reward scoring (side stream),
        then token rewards (score at the last token, -beta*KL per token) and GAE."""
        c = self.cfg
        with self.timer.phase("ref_logprobs+reward"):
            if not c.overlap_reward and not ro._pending:
                self._score_now(ro, side=False)  # serial schedule: reward first, on the main stream
            rec = self.record_overlap_events and self.device.type == "cuda"
            if rec:
                self.overlap_events["ref_start"] = _event()
            # the frozen reference: adapters off (LoRA) or the starting-weight copy (full FT)
            ref_model = self.ref_policy if self.ref_policy is not None else self.policy
            if c.old_logp == "recompute":
                # theta_old log-probs and values in the training forward's numerics (LoRA on, unmerged)
                self.policy.set_lora_enabled(True)
                old_lp, old_v = [], []
                mb = max(c.minibatch_size, c.ref_minibatch_size)
                hl = ro.host_lengths
                for s in range(0, ro.resp.shape[0], mb):
                    lp, _, v, _ = score_sequences(self.policy, ro.prompt_ids[s:s + mb], ro.start[s:s + mb],
                                                  ro.resp[s:s + mb], ro.resp_len[s:s + mb], 1.0 / c.temperature,
                                                  self.value_head,
                                                  lengths=(hl[0][s:s + mb], hl[1][s:s + mb]) if hl else None)
                    old_lp.append(lp)
                    old_v.append(v)
                ro.rollout_logp = ro.old_logp
                ro.old_logp = torch.cat(old_lp, 0).to(ro.old_logp.dtype)
                ro.old_values = torch.cat(old_v, 0).to(ro.old_values.dtype)
            ref_model.set_lora_enabled(False)
            try:
                ref_lp = []
                mb = max(c.minibatch_size, c.ref_minibatch_size)  # no-grad: larger GEMMs, no saved activations
                hl = ro.host_lengths
                for s in range(0, ro.resp.shape[0], mb):
                    lp, _, _, _ = score_sequences(ref_model, ro.prompt_ids[s:s + mb], ro.start[s:s + mb],
                                                  ro.resp[s:s + mb], ro.resp_len[s:s + mb],
                                                  1.0 / c.temperature,
                                                  lengths=(hl[0][s:s + mb], hl[1][s:s + mb]) if hl else None)
                    ref_lp.append(lp)
                ro.ref_logp = torch.cat(ref_lp, 0)
            finally:
                ref_model.set_lora_enabled(True)
            if rec:
                self.overlap_events["ref_end"] = _event()
            # the whole reference forward is queued and nothing above waited for the device: the
            # host detokenises now and the reward encoder runs on the side stream beside it
            self._collect_rewards(ro)
        # token rewards (-beta * KL per token unless the KL is in the loss, score at the last
        # token), GAE and whitening: one kernel on GPU (ops.ppo_advantages; the eager oracle on CPU)
        adv, ret, rewards, kl_seq = ops.ppo_advantages(ro.old_logp, ro.ref_logp, ro.old_values, ro.scores,
                                                       ro.resp_len, 0.0 if c.kl_in_loss else self.kl_coef,
                                                       c.gamma, c.lam, c.whiten_advantages)
        ro.adv, ro.returns, ro.rewards_tok = adv, ret, rewards
        # sum_t (old - ref) per sequence: the reference KL when "old" is a training-numerics forward;
        # with sampler log-probs it also holds the decode engine's numerics gap (reported apart)
        ro.kl_old_ref = kl_seq.mean()
        return ro

    # ------------------------------------------------------------------ update
    def update(self, ro: Rollout) -> dict:
        c = self.cfg
        B = ro.resp.shape[0]
        stats = []
        inv_t = 1.0 / c.temperature
        g = torch.Generator(device="cpu").manual_seed(c.seed + self.global_step)
        with self.timer.phase("update"):
            for _ in range(c.ppo_epochs):
                perm = torch.randperm(B, generator=g).tolist()
                hl = ro.host_lengths
                for s in range(0, B, c.minibatch_size):
                    rows = perm[s:s + c.minibatch_size]
                    idx = torch.tensor(rows, device=self.device)
                    lp, ent, vals, mask = score_sequences(self.policy, ro.prompt_ids[idx], ro.start[idx],
                                                          ro.resp[idx], ro.resp_len[idx], inv_t, self.value_head,
                                                          c.gradient_checkpointing,
                                                          lengths=(hl[0][rows], hl[1][rows]) if hl else None)
                    # fused token-level objective (clipped surrogate + value + entropy) and its
                    # gradient in one kernel on the GPU (ops.ppo_loss; eager oracle on CPU)
                    # the ratio's denominator: the behaviour log-probs old_logp (sampler mu, or the
                    # recomputed theta_old); the reference KL (kl_in_loss) on this forward's own lp
                    loss, st = ops.ppo_loss(lp, vals, ent, ro.old_logp[idx], ro.adv[idx], ro.returns[idx], mask,
                                            c.clip_range, c.value_coef, c.entropy_coef, c.value_clip,
                                            ro.old_values[idx] if c.value_clip is not None else None,
                                            ro.ref_logp[idx], self.kl_coef if c.kl_in_loss else 0.0)
                    if not stats:
                        # behaviour / target policy gap: the first minibatch scores the
                        # rollouts at theta = theta_old, so |logp - old_logp| is the rollout engine's
                        # (merged LoRA, decode kernels) deviation from the training forward
                        with torch.no_grad():
                            mf = mask.float()
                            first_gap = ((lp.detach().float() - ro.old_logp[idx].float()).abs() * mf).sum() / \
                                mf.sum().clamp(min=1.0)
                            # the rollout engine's own deviation (sampler log-probs vs the training
                            # forward at theta_old), whatever old_logp source the ratio uses
                            rl_lp = getattr(ro, "rollout_logp", None)
                            engine_gap = first_gap if rl_lp is None else \
                                ((lp.detach().float() - rl_lp[idx].float()).abs() * mf).sum() / mf.sum().clamp(min=1.0)
                    self.opt.zero_grad()
                    self.sync.start()
                    loss.backward()
                    self.sync.finish()
                    lr = lr_at(self.opt.step_count, c.lr, c.lr_schedule, c.warmup_steps, c.total_steps)
                    self.opt.step(lr)
                    self.policy.refresh_lora()
                    stats.append(st)
        # stats rows: [loss, policy_loss, value_loss, entropy, approx_kl, clipfrac, kl_ref_k3,
        # kl_ref_k1, n_tokens] (one D2H copy with the step's other device scalars)
        sts = torch.stack(stats)
        first_epoch = sts[: (B + c.minibatch_size - 1) // c.minibatch_size]
        # reference KL per sequence from the first epoch's forwards (every rollout token scored once;
        # the first minibatch at theta_old): sum_t (lp - ref) / B in training numerics
        kl_tok_sum = (first_epoch[:, 7] * first_epoch[:, 8]).sum()
        rows0 = min(B, c.minibatch_size)
        dev_scalars = torch.stack([kl_tok_sum / B, ro.kl_old_ref.to(sts.device).float(), first_gap.float(),
                                   engine_gap.float(), sts[0, 7] * sts[0, 8] / rows0]).tolist()
        sm = sts.mean(0).tolist()
        out = {"total_loss": sm[0], "policy_loss": sm[1], "value_loss": sm[2], "entropy": sm[3],
               "entropy_loss": -c.entropy_coef * sm[3], "approx_kl": sm[4], "clipfrac": sm[5],
               "kl_ref_k3": sm[6]}
        # kl_ref: nats per sequence. kl_in_loss: the update forwards' own lp vs the reference (what
        # the penalty acts on); otherwise sum_t (old - ref), the quantity in the reward
        out["kl_ref"] = dev_scalars[0] if c.kl_in_loss else dev_scalars[1]
        out["kl_old_ref"] = dev_scalars[1]
        # the first minibatch scores at theta = theta_old: KL(pi_theta_old || ref) per sequence in
        # training numerics (exactly 0 at LoRA B = 0 / before any full-FT update)
        out["kl_ref_theta_old"] = dev_scalars[4]
        out["behaviour_logp_gap"] = dev_scalars[2]
        out["rollout_engine_logp_gap"] = dev_scalars[3]
        out["clipfrac_first_mb"] = float(stats[0][5])
        out["grad_norm"] = float(self.opt.last_norm)
        out["skipped_steps"] = float(self.opt.skipped)
        out["time/allreduce_wait"] = self.sync.wait_s
        self.sync.wait_s = 0.0
        out["lr"] = lr
        return out

    # ------------------------------------------------------------------ one PPO iteration
    def step(self, batch: Dict[str, list]) -> dict:
        self.timer.reset()
        t0 = time.perf_counter()
        maybe_inject_fault(self.global_step)
        ro = self.rollout(batch)
        self.prepare(ro)
        upd = self.update(ro)
        dt = time.perf_counter() - t0
        comps = ro.components
        m = {
            "reward_mean": float(ro.scores.mean()), "reward_std": float(ro.scores.std(unbiased=False)),
            "factual_accuracy": float(comps["factual_accuracy"].mean()), "relevance": float(comps["relevance"].mean()),
            "conciseness": float(comps["conciseness"].mean()),
            **upd, "kl_coef": self.kl_coef, "rollout_tokens": float(ro.n_tokens),
            "response_len": float(ro.resp_len.float().mean()), "step_time_s": dt,
        }
        m.update(self.timer.as_dict())
        # means over ranks, except durations (max over ranks): throughput = all ranks' tokens /
        # the slowest rank's step, as the bench measures it
        m = reduce_metrics(m)
        m["rollout_tokens_per_s"] = m["rollout_tokens"] * dist_info().world / max(m["step_time_s"], 1e-9)
        if self.kl is not None:
            self.kl.update(m["kl_ref"], len(batch["query"]))
        self.global_step += 1
        if dist_info().is_main:
            self.sink.log(m, step=self.global_step)
        self.last_rollout = ro
        return m

    # ------------------------------------------------------------------ checkpoints
    def trainer_state(self, epoch: int = 0, best: float = -math.inf, batch_in_epoch: int = 0):
        from ..utils import rng_state

        return {"kind": "ppo", "global_step": self.global_step, "epoch": epoch, "batch_in_epoch": batch_in_epoch,
                "best_reward": best, "config": asdict(self.cfg),
                "kl_coef": self.kl_coef, "rng": rng_state(),
                # the on-device Philox counter of the rollout sampler: a resumed run continues the
                # random stream instead of replaying step 0's draws
                "gen_rng_offset": int(self.gen.rng_offset.item())}

    def save_checkpoint(self, prefix: str, epoch: int = 0, best: float = -math.inf, full_policy: bool = True,
                        batch_in_epoch: int = 0, extra_state: Optional[dict] = None):
        """Every rank calls this: rank 0 writes the artifacts, every other rank its RNG state, every
        rank its ZeRO-1 optimizer shard — all inside the trainer-state directory before it is
        renamed into place (checkpoint.save_checkpoint_dp)."""
        from .checkpoint import save_checkpoint_dp

        st = self.trainer_state(epoch, best, batch_in_epoch)  # collective-free; every rank
        st.update(extra_state or {})
        save_checkpoint_dp(prefix, self.policy, self.tok, self.value_head, self.opt, st, save_full_policy=full_policy)

    def load_checkpoint(self, prefix: str) -> dict:
        from ..utils import set_rng_state
        from .checkpoint import load_checkpoint

        st = load_checkpoint(prefix, self.policy, self.value_head, self.opt)
        self.global_step = int(st.get("global_step", 0))
        if self.kl is not None and "kl_coef" in st:
            self.kl.value = st["kl_coef"]
        if "rng" in st:
            set_rng_state(st["rng"])
        if "gen_rng_offset" in st:
            self.gen.rng_offset.fill_(int(st["gen_rng_offset"]))
        return st
