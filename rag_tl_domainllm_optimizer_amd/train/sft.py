"""Supervised fine-tuning with LoRA (config 3: "Mistral-7B LoRA r=16 RAFT-style SFT with
distractor docs, DP=8 over xGMI") — the README's Transfer Learning stage (README.md:15,29).

Loss = token cross-entropy on the answer tokens only (prompt tokens masked), computed by the fused
log-softmax kernel on the gathered answer rows (no full-vocabulary fp32 softmax over the prompt).
LoRA adapters are fused into the projection GEMMs; gradients of all ranks are averaged by bucketed
RCCL all-reduce overlapped with backward; the optimizer is the flat fused AdamW.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..models.decoder import pack_enabled, packed_index
from ..parallel import GradSync, info as dist_info, reduce_metrics
from ..utils import MetricsSink, maybe_inject_fault
from .common import lr_at


@dataclass
class SFTConfig:
    lr: float = 2e-4
    weight_decay: float = 0.0
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    max_grad_norm: float = 1.0
    batch_size: int = 8            # sequences per rank per micro-batch
    grad_accum: int = 1
    max_seq: int = 512
    lora_r: int = 16
    lora_alpha: float = 32.0
    lora_targets: Sequence[str] = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
    full_finetune: bool = False
    lr_schedule: str = "cosine"
    warmup_steps: int = 10
    total_steps: int = 0
    gradient_checkpointing: bool = False
    bucket_mb: float = 64.0          # DP all-reduce bucket size
    save_full_policy: bool = True    # also write the merged HF policy next to the PEFT adapter
    save_every: int = 0              # CLI: mid-epoch "latest" checkpoint every N steps (0 = epoch ends)
    seed: int = 0


class SFTTrainer:
    def __init__(self, model, tokenizer, cfg: Optional[SFTConfig] = None, sink: Optional[MetricsSink] = None):
        self.cfg = cfg or SFTConfig()
        c = self.cfg
        self.model, self.tok = model, tokenizer
        self.device = model.embed.device
        self.sink = sink or MetricsSink(enabled=False)
        if c.full_finetune:
            # every weight trains: bf16 compute copies + fp32 master on the GPU (ops.MixedFlatParams)
            model.requires_grad_(True)
            params = list(model.parameters())
        else:
            if getattr(model, "lora_config", None) is None:
                model.add_lora(c.lora_r, c.lora_alpha, list(c.lora_targets), seed=c.seed)
            model.freeze_base()
            params = model.lora_parameters()
        self.flat = ops.flat_params(params)
        if not c.full_finetune:
            model.refresh_lora()
        self.opt = ops.FusedAdamW(self.flat, lr=c.lr, betas=c.betas, eps=c.eps, weight_decay=c.weight_decay,
                                  max_grad_norm=c.max_grad_norm)
        self.sync = GradSync(self.flat, bucket_bytes=int(c.bucket_mb * (1 << 20)))
        self.global_step = 0
        self._pending = []  # (loss on device, grad norm on device, tokens, lr, t0) of uncollected steps

    # ------------------------------------------------------------------ batching
    def encode(self, prompts: Sequence[str], answers: Sequence[str]):
        """Left-padded [prompt | answer | eos] with a mask of answer positions."""
        c = self.cfg
        seqs, n_ans = [], []
        for p, a in zip(prompts, answers):
            pi = self.tok.encode(p)
            ai = self.tok.encode(a, add_special_tokens=False) + [self.tok.eos_token_id]
            pi = pi[-max(1, c.max_seq - len(ai)):]
            s = (pi + ai)[-c.max_seq:]
            seqs.append(s)
            n_ans.append(min(len(ai), len(s) - 1))
        S = max(len(s) for s in seqs)
        B = len(seqs)
        ids = torch.full((B, S), self.tok.pad_token_id, dtype=torch.long)
        start = torch.zeros(B, dtype=torch.int32)
        tgt = torch.full((B, S), -100, dtype=torch.long)
        for b, s in enumerate(seqs):
            ids[b, S - len(s):] = torch.tensor(s)
            start[b] = S - len(s)
            na = n_ans[b]
            tgt[b, S - na - 1:S - 1] = torch.tensor(s[len(s) - na:])  # position t predicts token t+1
        return ids.to(self.device), start.to(self.device), tgt.to(self.device)

    def loss(self, ids, start, tgt):
        flat_t = tgt.reshape(-1)
        rows = (flat_t >= 0).nonzero().squeeze(-1)
        B, S = ids.shape
        st = start.cpu().numpy().astype(np.int64) if pack_enabled() else None
        if st is not None and B * (S - 1) - int(st.sum()) < 0.97 * B * S:
            # varlen: row b's inputs are [start_b, S - 1) (the last token predicts nothing); the
            # GEMMs skip the left pads, the scored rows are looked up in the packed order
            idx, _ = packed_index(st, np.full(B, S - 1), S, ids.device)
            inv = torch.full((B * S,), -1, dtype=torch.long, device=ids.device)
            inv.index_copy_(0, idx, torch.arange(idx.numel(), device=ids.device))
            # hidden states of the answer rows only (last layer's o_proj / MLP skip the rest)
            hs = self.model(ids, kv_start=start, gradient_checkpointing=self.cfg.gradient_checkpointing,
                            packed_idx=idx, out_rows=inv.index_select(0, rows))
        else:
            hs = self.model(ids, kv_start=start, gradient_checkpointing=self.cfg.gradient_checkpointing,
                            out_rows=rows)
        logits = ops.linear(hs, self.model.head_weight)
        lp, _ = ops.token_logprobs(logits, flat_t[rows], 1.0)
        return -lp.mean(), int(rows.numel())

    # ------------------------------------------------------------------ step / fit
    def step(self, examples: List[Dict[str, str]], sync: bool = True) -> Optional[dict]:
        """One optimizer step over ``examples`` (``grad_accum`` micro-batches). The loss stays on
        the device: nothing in the step waits for the GPU, so the host enqueues the next step's
        encode / H2D while this one computes. ``sync`` (default) returns the rank-reduced metrics
        (one D2H copy at the end); ``sync=False`` queues them for :meth:`collect`."""
        c = self.cfg
        t0 = time.perf_counter()
        maybe_inject_fault(self.global_step)
        self.opt.zero_grad()
        self.sync.start()
        mbs = [examples[i::c.grad_accum] for i in range(c.grad_accum)]
        tot_loss, tot_tok = None, 0
        for i, mb in enumerate(mbs):
            ids, start, tgt = self.encode([e["prompt"] for e in mb], [e["answer"] for e in mb])
            loss, ntok = self.loss(ids, start, tgt)
            scaled = loss / c.grad_accum
            if i < len(mbs) - 1:
                with self.sync.no_sync():
                    scaled.backward()
            else:
                scaled.backward()
            tot_loss = loss.detach() if tot_loss is None else tot_loss + loss.detach()
            tot_tok += ntok
        self.sync.finish()
        lr = lr_at(self.opt.step_count, c.lr, c.lr_schedule, c.warmup_steps, c.total_steps)
        self.opt.step(lr)
        if not c.full_finetune:
            self.model.refresh_lora()
        self.global_step += 1
        # last_norm is rewritten in place by every optimizer step: queue a snapshot (a device copy,
        # no sync), or every queued step would report the norm of the last one
        norm = self.opt.last_norm
        norm = norm.detach().clone() if torch.is_tensor(norm) else float(norm)
        self._pending.append((tot_loss / len(mbs), norm, float(tot_tok), lr, t0))
        return self.collect()[-1] if sync else None

    def close(self):
        """Detach from the policy: remove the gradient-sync hooks on its parameters (a policy handed
        on to PPO must not fire this trainer's all-reduces on stale buffers) and drop the optimizer
        state. Idempotent."""
        self.sync.remove()
        self._pending = []

    def collect(self) -> List[dict]:
        """Metrics of every queued step: ONE device->host copy for all of them, then the rank
        reduction. ``step_time_s`` of a queued run is the wall time from the first queued step's
        start to now, spread evenly."""
        if not self._pending:
            return []
        pend, self._pending = self._pending, []
        vals = torch.stack([torch.stack([torch.as_tensor(l, dtype=torch.float32, device=self.device).reshape(()),
                                         torch.as_tensor(g, dtype=torch.float32, device=self.device).reshape(())])
                            for l, g, _, _, _ in pend]).cpu().tolist()
        dt = (time.perf_counter() - pend[0][4]) / len(pend)
        out = []
        for (loss, gn), (_, _, tok, lr, _) in zip(vals, pend):
            m = reduce_metrics({"loss": loss, "answer_tokens": tok, "step_time_s": dt, "grad_norm": gn, "lr": lr})
            m["tokens_per_s"] = m["answer_tokens"] * dist_info().world / max(m["step_time_s"], 1e-9)
            out.append(m)
        if dist_info().is_main:
            for k, m in enumerate(out):
                self.sink.log(m, step=self.global_step - len(out) + 1 + k)
        return out

    def epoch_order(self, n: int, epoch: int, shuffle: bool = True) -> List[int]:
        """This rank's example order for ``epoch`` — a function of (seed, epoch, rank, world) only,
        so a resumed run rebuilds it exactly. Wrap-around padding to a multiple of the world size:
        every rank gets a shard of the SAME length, hence the same number of steps (an extra step
        on one rank would wait forever in the gradient all-reduce of the others)."""
        import random

        di = dist_info()
        idx = list(range(n))
        if shuffle:
            random.Random(self.cfg.seed * 1000003 + epoch).shuffle(idx)
        if len(idx) % di.world:
            idx += idx[: di.world - len(idx) % di.world]
        return idx[di.rank::di.world]

    def fit(self, examples: List[Dict[str, str]], epochs: int = 1, shuffle: bool = True, log_every: int = 10,
            ckpt_dir: Optional[str] = None, save_every: int = 0, resume: bool = False):
        """Epochs of SFT with the reference's checkpoint pattern (rl.py:357-363): ``best_model``
        when the epoch's mean loss improves and ``epoch_{n}`` every epoch, under ``ckpt_dir``;
        ``save_every`` > 0 adds a mid-epoch ``latest`` checkpoint with the position in the epoch.
        ``resume`` continues from the most advanced of them (adapter or full weights, optimizer
        moments, every rank's RNG, the epoch and step)."""
        di = dist_info()
        bs = self.cfg.batch_size * self.cfg.grad_accum
        hist: List[dict] = []
        first_ep, first_k, best = 0, 0, math.inf
        ep_losses: List[float] = []
        if resume and ckpt_dir:
            from ..cli import latest_checkpoint

            prefix = latest_checkpoint(ckpt_dir, kind="sft")
            if prefix is not None:
                st = self.load_checkpoint(prefix)
                first_ep, first_k = int(st.get("epoch", 0)), int(st.get("step_in_epoch", 0))
                best = float(st.get("best_loss", best))
                ep_losses = list(st.get("epoch_losses", []))
                if di.is_main:
                    print(f"[sft] resumed from {prefix} (epoch {first_ep}, step {first_k})", flush=True)
        for ep in range(first_ep, epochs):
            idx = self.epoch_order(len(examples), ep, shuffle)
            n_steps = max(1, len(idx) // bs)
            k0 = first_k if ep == first_ep else 0
            if ep != first_ep:
                ep_losses = []
            for k in range(k0, n_steps):
                last = k == n_steps - 1
                logs = bool(log_every) and (self.global_step + 1) % log_every == 0
                mid = bool(save_every and ckpt_dir) and (self.global_step + 1) % save_every == 0 and not last
                self.step([examples[i] for i in idx[k * bs:(k + 1) * bs]], sync=False)
                if last or logs or mid:
                    got = self.collect()
                    hist += got
                    ep_losses += [m["loss"] for m in got]
                    if di.is_main and logs:
                        print(f"[sft] epoch {ep} step {self.global_step} loss {got[-1]['loss']:.4f}", flush=True)
                if mid:
                    self.save(os.path.join(ckpt_dir, "latest"), full_policy=False, epoch=ep, step_in_epoch=k + 1,
                              best_loss=best, extra_state={"epoch_losses": ep_losses})
            avg = sum(ep_losses) / max(len(ep_losses), 1)
            if di.is_main:
                print(f"Epoch {ep + 1}/{epochs}: Average Loss = {avg:.4f}", flush=True)
            if ckpt_dir:
                if avg < best:  # rl.py:358-360 (the reference's criterion is reward; SFT's is loss)
                    best = avg
                    self.save(os.path.join(ckpt_dir, "best_model"), full_policy=False, epoch=ep + 1, best_loss=best)
                self.save(os.path.join(ckpt_dir, f"epoch_{ep + 1}"), full_policy=False, epoch=ep + 1, best_loss=best)
        hist += self.collect()
        return hist

    # ------------------------------------------------------------------ checkpoints
    def trainer_state(self, epoch: int = 0, step_in_epoch: int = 0, best_loss: float = math.inf) -> dict:
        from ..utils import rng_state

        return {"kind": "sft", "global_step": self.global_step, "epoch": epoch, "step_in_epoch": step_in_epoch,
                "best_loss": best_loss, "config": asdict(self.cfg), "rng": rng_state()}

    def save(self, prefix: str, full_policy: bool = True, epoch: int = 0, step_in_epoch: int = 0,
             best_loss: float = math.inf, extra_state: Optional[dict] = None):
        """PEFT adapter (LoRA) + optimizer moments + trainer state (position, best loss, every
        rank's RNG), and the merged HF policy when ``full_policy`` (always under full fine-tuning);
        rank 0 writes the artifacts, every other rank its RNG state."""
        from .checkpoint import save_checkpoint_dp

        st = self.trainer_state(epoch, step_in_epoch, best_loss)
        st.update(extra_state or {})
        save_checkpoint_dp(prefix, self.model, self.tok, None, self.opt, st,
                           save_full_policy=full_policy or self.cfg.full_finetune)

    def load_checkpoint(self, prefix: str) -> dict:
        """Inverse of :meth:`save`: adapter (or, under full fine-tuning, the fp32 master restored
        from the optimizer file), optimizer moments, step counters, this rank's RNG."""
        from ..utils import set_rng_state
        from .checkpoint import load_checkpoint

        st = load_checkpoint(prefix, self.model, None, self.opt)
        self.global_step = int(st.get("global_step", 0))
        if "rng" in st:
            set_rng_state(st["rng"])
        return st
