"""Supervised fine-tuning with LoRA (config 3: "Mistral-7B LoRA r=16 RAFT-style SFT with
distractor docs, DP=8 over xGMI") — the README's Transfer Learning stage (README.md:15,29).

Loss = token cross-entropy on the answer tokens only (prompt tokens masked), computed by the fused
log-softmax kernel on the gathered answer rows (no full-vocabulary fp32 softmax over the prompt).
LoRA adapters are fused into the projection GEMMs; gradients of all ranks are averaged by bucketed
RCCL all-reduce overlapped with backward; the optimizer is the flat fused AdamW.
"""
from __future__ import annotations

import math
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
    def step(self, examples: List[Dict[str, str]]) -> dict:
        c = self.cfg
        t0 = time.perf_counter()
        maybe_inject_fault(self.global_step)
        self.opt.zero_grad()
        self.sync.start()
        mbs = [examples[i::c.grad_accum] for i in range(c.grad_accum)]
        tot_loss, tot_tok = 0.0, 0
        for i, mb in enumerate(mbs):
            ids, start, tgt = self.encode([e["prompt"] for e in mb], [e["answer"] for e in mb])
            loss, ntok = self.loss(ids, start, tgt)
            scaled = loss / c.grad_accum
            if i < len(mbs) - 1:
                with self.sync.no_sync():
                    scaled.backward()
            else:
                scaled.backward()
            tot_loss += float(loss.detach())
            tot_tok += ntok
        self.sync.finish()
        lr = lr_at(self.opt.step_count, c.lr, c.lr_schedule, c.warmup_steps, c.total_steps)
        self.opt.step(lr)
        if not c.full_finetune:
            self.model.refresh_lora()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m = reduce_metrics({"loss": tot_loss / len(mbs), "answer_tokens": float(tot_tok), "step_time_s": dt,
                            "grad_norm": float(self.opt.last_norm), "lr": lr})
        m["tokens_per_s"] = m["answer_tokens"] * dist_info().world / max(m["step_time_s"], 1e-9)
        self.global_step += 1
        if dist_info().is_main:
            self.sink.log(m, step=self.global_step)
        return m

    def fit(self, examples: List[Dict[str, str]], epochs: int = 1, shuffle: bool = True, log_every: int = 10):
        import random

        di = dist_info()
        rng = random.Random(self.cfg.seed)
        bs = self.cfg.batch_size * self.cfg.grad_accum
        hist = []
        for ep in range(epochs):
            idx = list(range(len(examples)))
            if shuffle:
                rng.shuffle(idx)
            # wrap-around padding to a multiple of the world size: every rank gets a shard of the
            # SAME length, hence the same number of steps (an extra step on one rank would wait
            # forever in the gradient all-reduce of the others)
            if len(idx) % di.world:
                idx += idx[: di.world - len(idx) % di.world]
            idx = idx[di.rank::di.world]
            n_steps = max(1, len(idx) // bs)
            for k in range(n_steps):
                m = self.step([examples[i] for i in idx[k * bs:(k + 1) * bs]])
                hist.append(m)
                if di.is_main and log_every and len(hist) % log_every == 0:
                    print(f"[sft] epoch {ep} step {self.global_step} loss {m['loss']:.4f}", flush=True)
        return hist

    def save(self, prefix: str, full_policy: bool = True):
        """PEFT adapter (LoRA) + trainer state, and the merged HF policy when ``full_policy``;
        rank 0 writes, the other ranks wait (every rank then reads the same files)."""
        from ..parallel import barrier
        from .checkpoint import save_checkpoint

        if dist_info().is_main:
            save_checkpoint(prefix, self.model, self.tok, None, self.opt,
                            {"global_step": self.global_step, "config": asdict(self.cfg)},
                            save_full_policy=full_policy or self.cfg.full_finetune)
        barrier()
