"""Batched generation: static KV cache, prefill, and a hipGraph-captured decode step.

Replaces HF ``generate`` as used by the reference (rollouts rl.py:38-44, evaluation rl.py:411-417):
prompts are left-padded into one batch, prefilled with the flash kernel (K/V appended to a static
cache by the fused RoPE kernel), then every decode step — embedding, 32 x (norm, LoRA-fused
projections, RoPE+append, split-K decode attention, SwiGLU), final norm, LM head, on-device
sampler (which also emits the behaviour log-prob), value head, and the bookkeeping kernel — is one
graph replay with zero host synchronisation. Finished rows are masked on device; the host polls
completion only every ``sync_every`` steps.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..models.decoder import pack_enabled, packed_index
from ..runtime import GraphRunner


@dataclass
class SamplingParams:
    max_new_tokens: int = 128
    temperature: float = 0.7            # reference rl.py:41
    top_k: int = 50                     # HF 4.x generate default the reference ran with
    top_p: float = 1.0
    do_sample: bool = True              # reference rl.py:42
    max_length: Optional[int] = None    # reference semantics: prompt + new tokens (rl.py:40)
    stop_token_ids: Sequence[int] = ()
    seed: int = 0

    @property
    def greedy(self) -> bool:
        return (not self.do_sample) or self.temperature <= 0

    @property
    def inv_temp(self) -> float:
        return 1.0 if self.greedy else 1.0 / self.temperature


@dataclass
class GenerationOutput:
    tokens: torch.Tensor        # [B, T] generated ids (pad after finish)
    lengths: torch.Tensor       # [B] number of generated tokens
    logprobs: torch.Tensor      # [B, T] behaviour log-probs of the drawn tokens (tempered dist.)
    values: Optional[torch.Tensor]  # [B, T] value-head outputs at each generating state
    prompt_ids: torch.Tensor    # [B, S] left-padded prompts
    prompt_start: torch.Tensor  # [B] first real prompt token
    timings: dict = field(default_factory=dict)


class _GraphSet:
    """Captured decode steps by key (sampling parameters, output width, row bucket): replaying a
    generator at another batch bucket switches graphs instead of recapturing. Least recently used
    graphs beyond ``max_graphs`` are dropped; ``reset()`` drops all (e.g. when the output buffers
    they captured are reallocated). Same interface as ``runtime.GraphRunner``."""

    def __init__(self, max_graphs: int = 8):
        from collections import OrderedDict

        self.graphs = OrderedDict()
        self.cur = None
        self.max_graphs = max_graphs

    def needs(self, key) -> bool:
        r = self.graphs.get(key)
        if r is None:
            return True
        self.graphs.move_to_end(key)
        self.cur = r
        return False

    def capture(self, fn, key=None, keep=(), restore=()):
        r = GraphRunner()
        r.capture(fn, key, keep, restore)
        self.graphs[key] = r
        self.cur = r
        while len(self.graphs) > self.max_graphs:
            self.graphs.popitem(last=False)

    def replay(self):
        self.cur.replay()

    def reset(self):
        self.graphs.clear()
        self.cur = None


class KVCache:
    """Static K/V cache [L, B, Hkv, Smax, D]. ``fp8``: e4m3fn bytes (K rows k-permuted) plus one
    fp32 scale per (layer, row, kv head, slot) in ``ks`` / ``vs`` [L, B, Hkv, SmaxP] (SmaxP = Smax
    rounded up to 16; zero-initialised so never-written slots scale to 0) — config 5's rollout
    cache, half the bytes the decode attention streams (``ops.kv_store_fp8``)."""

    def __init__(self, num_layers, B, Hkv, Smax, D, device, dtype=torch.bfloat16, fp8: bool = False):
        alloc = torch.empty if torch.device(device).type == "cuda" else torch.zeros
        self.fp8 = fp8
        cdt = torch.uint8 if fp8 else dtype
        self.k = alloc(num_layers, B, Hkv, Smax, D, device=device, dtype=cdt)
        self.v = alloc(num_layers, B, Hkv, Smax, D, device=device, dtype=cdt)
        self.ks = self.vs = None
        if fp8:
            if D != ops.FP8_KV_D:
                raise ValueError(f"fp8 KV cache needs head_dim {ops.FP8_KV_D}, got {D}")
            smaxp = (Smax + 15) // 16 * 16
            self.ks = torch.zeros(num_layers, B, Hkv, smaxp, device=device, dtype=torch.float32)
            self.vs = torch.zeros(num_layers, B, Hkv, smaxp, device=device, dtype=torch.float32)
        self.B, self.Smax = B, Smax

    def scales(self, layer: int):
        """(k_scale, v_scale) of one layer, or (None, None) for a bf16 cache"""
        return (self.ks[layer], self.vs[layer]) if self.fp8 else (None, None)

    @property
    def nbytes(self):
        n = 2 * self.k.numel() * self.k.element_size()
        if self.fp8:
            n += 2 * self.ks.numel() * 4
        return n


class Generator:
    """Owns the cache and captured graph for one (model, max_batch, max_seq) configuration."""

    def __init__(self, model, max_batch: int, max_seq: int, device=None, use_graph: bool = True,
                 value_head=None, sync_every: int = 16, kv_fp8: Optional[bool] = None):
        self.model = model
        cfg = model.cfg
        self.cfg = cfg
        self.device = torch.device(device or model.embed.device)
        self.max_batch, self.max_seq = max_batch, max_seq
        self.use_graph = use_graph and self.device.type == "cuda"
        self.value_head = value_head
        self.sync_every = sync_every
        # generation never differentiates: by default adapters run on merged bf16 weights (one
        # weight stream per projection). False: the unmerged LoRA K-extension, i.e. exactly the
        # weights the training forward scores with (PPO behaviour policy == target policy at
        # theta_old, PPOConfig.merged_lora_rollout = False)
        self.merge_lora = True
        # fp8 K/V cache (config 5): the model's setting unless given; GPU MFMA decode kernels only
        # (head_dim 128), the CPU path runs the quantise / dequantise reference
        kv_fp8 = getattr(model, "kv_fp8", False) if kv_fp8 is None else kv_fp8
        self.cache = KVCache(cfg.num_layers, max_batch, cfg.num_kv_heads, max_seq, cfg.head_dim, self.device,
                             model.dtype, fp8=bool(kv_fp8))
        dev = self.device
        B = max_batch
        self.workspace = ops.decode_workspace(B, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, max_seq, dev) \
            if dev.type == "cuda" else None
        # device-resident decode state (static addresses for graph replay)
        self.tok_in = torch.zeros(B, dtype=torch.long, device=dev)
        self.kv_len = torch.zeros(B, dtype=torch.int32, device=dev)
        self.kv_start = torch.zeros(B, dtype=torch.int32, device=dev)
        self.pos = torch.zeros(B, dtype=torch.int32, device=dev)
        self.attn_len = torch.zeros(B, dtype=torch.int32, device=dev)
        self.active = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.gen_len = torch.zeros(B, dtype=torch.int32, device=dev)
        self.step = torch.zeros(1, dtype=torch.long, device=dev)
        self.rng_offset = torch.zeros(1, dtype=torch.long, device=dev)
        self.sampled = torch.zeros(B, dtype=torch.long, device=dev)
        self.sampled_lp = torch.zeros(B, dtype=torch.float32, device=dev)
        self.values = torch.zeros(B, dtype=torch.float32, device=dev)
        self.out_tokens = None
        self.runner = _GraphSet()  # captured decode steps (runtime.GraphRunner each, shared graph pool)

    # ------------------------------------------------------------------ one decode step (device only)
    def _bucket(self, B: int) -> int:
        """Rows a decode step runs for a batch of B: the next power of two (capped at max_batch).
        A serving generator sized for 16 or 64 users then decodes one answer at the batch-1 cost;
        each bucket has its own captured graph (the rows past B stay inactive)."""
        nb = 1
        while nb < B:
            nb *= 2
        return min(nb, self.max_batch)

    def _step(self, params: SamplingParams, eos_ids: torch.Tensor, pad_id: int):
        # attn_len = kv_len + 1 and pos = kv_len - kv_start were set by the previous bookkeeping
        # (decode_update on the GPU, _update_cpu on the CPU) — no elementwise launches here
        nb = self._nb
        cache = self.cache if nb == self.max_batch else _SubCache(self.cache, nb)
        h = self.model.decode(self.tok_in[:nb], self.pos[:nb], self.kv_len[:nb], self.attn_len[:nb],
                              self.kv_start[:nb], cache, self.workspace)
        self._emit(h, params, eos_ids, pad_id)

    def _emit(self, h, params: SamplingParams, eos_ids, pad_id, r0: int = 0):
        """Sample from the hidden states of rows [r0, r0 + len(h)) and run the bookkeeping for them
        (the decode step's row bucket, or one row admitted by continuous batching)."""
        r1 = r0 + h.shape[0]
        logits = self.model.logits(h)
        ops.sample(logits, params.inv_temp, params.top_k, params.top_p, params.greedy, params.seed,
                   self.rng_offset, self.active[r0:r1], self.sampled[r0:r1], self.sampled_lp[r0:r1])
        if self.value_head is not None:
            self.values[r0:r1].copy_(self.value_head(h))
        if h.is_cuda:
            vh = self.value_head is not None
            ops.native().decode_update(self.sampled[r0:r1], self.out_tokens[r0:r1], self.out_logp[r0:r1],
                                       self.sampled_lp[r0:r1], self.out_values[r0:r1] if vh else None,
                                       self.values[r0:r1] if vh else None, self.active[r0:r1],
                                       self.kv_len[r0:r1], self.pos[r0:r1], self.tok_in[r0:r1],
                                       self.gen_len[r0:r1], self.step, self.rng_offset, eos_ids, pad_id,
                                       self.attn_len[r0:r1], self.kv_start[r0:r1])
        else:
            self._update_cpu(eos_ids, pad_id, r0, r1)

    def _update_cpu(self, eos_ids, pad_id, r0: int = 0, r1: Optional[int] = None):
        """CPU twin of decode_update_kernel over rows [r0, r1): each active row writes at its own
        output position gen_len[b] (the step counter for a static batch)."""
        r1 = self.max_batch if r1 is None else r1
        T = self.out_tokens.shape[1]
        act = self.active[r0:r1].bool()
        gl = self.gen_len[r0:r1]
        act = act & (gl < T)
        rows = torch.nonzero(act).flatten()
        if rows.numel():
            idx = gl[rows].long()
            samp = self.sampled[r0:r1]
            self.out_tokens[r0 + rows, idx] = samp[rows]
            self.out_logp[r0 + rows, idx] = self.sampled_lp[r0:r1][rows]
            if self.value_head is not None:
                self.out_values[r0 + rows, idx] = self.values[r0:r1][rows]
            fin = torch.isin(samp, eos_ids) | (gl + 1 >= T)
            gl[act] += 1
            self.kv_len[r0:r1][act] += 1
            self.tok_in[r0:r1].copy_(torch.where(act, samp, torch.full_like(samp, pad_id)))
            self.active[r0:r1][act & fin] = 0
        else:
            self.tok_in[r0:r1].fill_(pad_id)
        self.step += 1
        self.rng_offset += 1
        torch.add(self.kv_len, 1, out=self.attn_len)
        torch.sub(self.kv_len, self.kv_start, out=self.pos)

    # ------------------------------------------------------------------ public
    @torch.no_grad()
    def generate(self, prompts: List[List[int]], params: SamplingParams, pad_id: int = 0,
                 eos_ids: Sequence[int] = ()) -> GenerationOutput:
        """Synchronous generation with early exit once every row has finished."""
        return self.generate_async(prompts, params, pad_id, eos_ids, early_stop=True).result()

    @torch.no_grad()
    def generate_async(self, prompts: List[List[int]], params: SamplingParams, pad_id: int = 0,
                       eos_ids: Sequence[int] = (), early_stop=False) -> "_Pending":
        """Enqueue prefill + the decode steps on the current stream and return.

        ``early_stop``:
          * False   — every decode step is enqueued now (the host never waits);
          * True    — stop once every row has finished, polling with a blocking read every
            ``sync_every`` steps (batch-1 answers: the host is idle anyway);
          * "async" — the same early exit without stalling the GPU: steps are enqueued in chunks
            of ``sync_every``; after each chunk the "any row active" flag is copied to pinned host
            memory behind an event, and the host, keeping two chunks queued ahead of the GPU,
            reads a chunk's flag only when the GPU has already started the next one. The first
            two chunks are enqueued here, the rest by ``result()`` (so work the caller does
            between the two calls, e.g. reward scoring, overlaps the decode). Rows are masked
            after EOS, and the sampler's RNG counter is advanced by the skipped steps, so outputs
            and later draws are identical to a run without the exit."""
        import time

        cfg = self.cfg
        dev = self.device
        B = len(prompts)
        assert 0 < B <= self.max_batch, f"batch {B} > max_batch {self.max_batch}"
        S = max(len(p) for p in prompts)
        T = params.max_new_tokens
        if params.max_length is not None:
            T = max(1, min(T, params.max_length - S))
        assert S + T <= self.max_seq, f"prompt {S} + new {T} exceeds cache {self.max_seq}"
        t0 = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if dev.type == "cuda" else None
        if ev:
            ev[0].record()
        ids = torch.full((B, S), pad_id, dtype=torch.long)
        start = torch.zeros(B, dtype=torch.int32)
        for b, p in enumerate(prompts):
            ids[b, S - len(p):] = torch.tensor(p, dtype=torch.long)
            start[b] = S - len(p)
        ids = ids.to(dev, non_blocking=True)
        MB = self.max_batch
        # reset device state (rows >= B stay inactive)
        self.kv_start.zero_()
        self.kv_start[:B].copy_(start.to(dev))
        self.active.zero_()
        self.active[:B] = 1
        self.gen_len.zero_()
        self.step.zero_()
        self.tok_in.fill_(pad_id)
        if self.out_tokens is None or self.out_tokens.shape[1] != T:
            self.out_tokens = torch.full((MB, T), pad_id, dtype=torch.long, device=dev)
            self.out_logp = torch.zeros(MB, T, dtype=torch.float32, device=dev)
            self.out_values = torch.zeros(MB, T, dtype=torch.float32, device=dev)
            self.runner.reset()
        else:
            self.out_tokens.fill_(pad_id)
            self.out_logp.zero_()
            self.out_values.zero_()
        eos_list = list(eos_ids) or [cfg.eos_token_id]
        eos = torch.tensor(eos_list, dtype=torch.long, device=dev)
        # prefill on the first B rows of the cache
        sub = _SubCache(self.cache, B)
        # generation never differentiates: run adapters on merged weights (one weight stream per
        # projection; the merged images are refreshed in place after each adapter update)
        prev_merged = self.model.set_lora_merged(self.merge_lora) if hasattr(self.model, "set_lora_merged") else None
        try:
            return self._enqueue(params, B, S, T, ids, start, eos, eos_list, pad_id, sub, early_stop, t0, ev)
        finally:
            if prev_merged is not None:
                self.model.set_lora_merged(prev_merged)

    def _enqueue(self, params, B, S, T, ids, start, eos, eos_list, pad_id, sub, early_stop, t0, ev):
        cfg, dev, MB = self.cfg, self.device, self.max_batch
        packed = None
        n_real = B * S - int(start.sum())
        if pack_enabled() and n_real < 0.97 * B * S:
            # varlen prefill: the projection GEMMs run on the real prompt tokens only
            packed = packed_index(start.numpy(), np.full(B, S), S, dev)
        h_last = self.model.prefill(ids, self.kv_start[:B], sub, packed=packed) if packed is not None else \
            self.model.prefill(ids, self.kv_start[:B], sub)
        if hasattr(self.model, "refresh_decode_weights"):
            self.model.refresh_decode_weights(self._bucket(B))  # folded / tile-ordered / fp8 images of graph replays
        self._nb = self._bucket(B)
        h = torch.zeros(self._nb, cfg.hidden_size, dtype=h_last.dtype, device=dev)
        h[:B] = h_last
        # the first sampled token is not in the cache yet: the bookkeeping kernel advances kv_len
        # to S, so the first decode step writes it at slot S
        self.kv_len.fill_(S - 1)
        self._emit(h, params, eos, pad_id)
        if ev:
            ev[1].record()
        steps = T - 1
        if steps > 0:
            self._ensure_graph(params, eos, eos_list, pad_id, T)
        loop = _DecodeLoop(self, steps, params, eos, pad_id, early_stop)
        loop.run()
        pend = _Pending(self, B, ids, start, t0, ev, loop)
        if loop.finished and ev:
            ev[2].record()
            pend._recorded = True
        return pend

    def _ensure_graph(self, params, eos, eos_list, pad_id, T):
        """The captured decode step for (sampling parameters, output width, row bucket)."""
        key = (T, params.inv_temp, params.top_k, params.top_p, params.greedy, params.seed, tuple(eos_list), pad_id,
               self._nb)
        if self.use_graph and self.runner.needs(key):
            # the EOS tensor is created per call: the runner keeps the captured one alive
            self.runner.capture(lambda: self._step(params, eos, pad_id), key, keep=(eos,), restore=self._state())

    def _replay(self, params, eos, pad_id):
        if self.use_graph:
            self.runner.replay()
        else:
            self._step(params, eos, pad_id)

    def _state(self):
        return [self.tok_in, self.kv_len, self.pos, self.attn_len, self.active, self.gen_len, self.step,
                self.rng_offset, self.sampled, self.sampled_lp, self.values, self.out_tokens, self.out_logp,
                self.out_values]


class _DecodeLoop:
    """Enqueues the decode steps of one generation (see ``Generator.generate_async``)."""

    AHEAD = 2  # chunks kept queued ahead of the GPU in the "async" early-exit mode

    def __init__(self, gen: "Generator", steps: int, params, eos, pad_id, early_stop):
        self.gen, self.steps, self.params, self.eos, self.pad_id = gen, steps, params, eos, pad_id
        self.mode = early_stop
        self.done = 0
        self.pending = []  # (chunk index, event) of flags not read yet
        self.stopped = False
        if early_stop == "async" and steps > 0:
            dev = gen.device
            n = (steps + gen.sync_every - 1) // gen.sync_every
            self.flags_dev = torch.zeros(n, dtype=torch.int32, device=dev)
            self.flags = torch.zeros(n, dtype=torch.int32, pin_memory=dev.type == "cuda")

    @property
    def finished(self) -> bool:
        return self.stopped or self.done >= self.steps

    def _chunk(self, n):
        g = self.gen
        for _ in range(n):
            g._replay(self.params, self.eos, self.pad_id)
        self.done += n

    def run(self, to_end: bool = False):
        g = self.gen
        if self.mode is False:
            self._chunk(self.steps - self.done)
            return
        if self.mode is True:
            while not self.finished:
                self._chunk(min(g.sync_every, self.steps - self.done))
                if self.done < self.steps and int(g.active.sum().item()) == 0:
                    self._stop()
            return
        # "async": keep AHEAD chunks queued; read a chunk's flag once the GPU is past it
        while not self.finished:
            if len(self.pending) >= self.AHEAD:
                c, ev = self.pending.pop(0)
                if not to_end and not ev.query():
                    return  # result() continues from here
                ev.synchronize()
                if int(self.flags[c]) == 0:
                    self._stop()
                    break
            c = self.done // g.sync_every
            self._chunk(min(g.sync_every, self.steps - self.done))
            if self.done < self.steps:
                self.flags_dev[c:c + 1].copy_(g.active.amax().reshape(1))
                self.flags[c:c + 1].copy_(self.flags_dev[c:c + 1], non_blocking=True)
                ev = torch.cuda.Event() if g.device.type == "cuda" else None
                if ev is not None:
                    ev.record()
                    self.pending.append((c, ev))
                elif int(self.flags[c]) == 0:
                    self._stop()
            if not to_end and len(self.pending) >= self.AHEAD:
                return

    def _stop(self):
        """Every row has finished: skip the remaining steps, but advance the sampler's RNG counter
        as if they had run (later generations draw the same numbers either way)."""
        skipped = self.steps - self.done
        if skipped > 0:
            self.gen.rng_offset.add_(skipped)
        self.stopped = True
        self.skipped = skipped


class _Pending:
    """Handle of an enqueued generation; ``result()`` finishes enqueuing (async early exit), waits
    and copies the outputs out."""

    def __init__(self, gen: "Generator", B, ids, start, t0, ev, loop: Optional[_DecodeLoop] = None):
        self.gen, self.B, self.ids, self.start, self.t0, self.ev = gen, B, ids, start, t0, ev
        self.loop = loop
        self._recorded = False

    @torch.no_grad()
    def result(self) -> GenerationOutput:
        import time

        g, B = self.gen, self.B
        if self.loop is not None and not self.loop.finished:
            # the remaining steps run under the same conditions the loop started with: no autograd,
            # adapters merged (generate_async restored the caller's mode on return; the eager
            # non-graph path would otherwise decode with unmerged adapters)
            m = g.model
            prev = m.set_lora_merged(g.merge_lora) if hasattr(m, "set_lora_merged") else None
            try:
                self.loop.run(to_end=True)
            finally:
                if prev is not None:
                    m.set_lora_merged(prev)
        if self.ev and not self._recorded:
            self.ev[2].record()
            self._recorded = True
        if self.ev:
            self.ev[2].synchronize()
        t_total = time.perf_counter() - self.t0
        tim = {"total_s": t_total}
        if self.ev:
            tim["prefill_s"] = self.ev[0].elapsed_time(self.ev[1]) / 1e3
            tim["decode_s"] = self.ev[1].elapsed_time(self.ev[2]) / 1e3
        if self.loop is not None:
            tim["decode_steps"] = self.loop.done
        return GenerationOutput(g.out_tokens[:B].clone(), g.gen_len[:B].clone().long(), g.out_logp[:B].clone(),
                                g.out_values[:B].clone() if g.value_head is not None else None, self.ids,
                                self.start.to(g.device).long(), tim)


class _SubCache:
    """View of the first B batch rows of a KVCache (prefill of a partial batch)."""

    def __init__(self, cache: KVCache, B: int):
        self.k = [cache.k[l, :B] for l in range(cache.k.shape[0])]
        self.v = [cache.v[l, :B] for l in range(cache.v.shape[0])]
        self.fp8 = cache.fp8
        if cache.fp8:
            self.ks = [cache.ks[l, :B] for l in range(cache.ks.shape[0])]
            self.vs = [cache.vs[l, :B] for l in range(cache.vs.shape[0])]

    def scales(self, layer: int):
        return (self.ks[layer], self.vs[layer]) if self.fp8 else (None, None)


def generate_text(model, tokenizer, prompts: List[str], params: SamplingParams, generator: Optional[Generator] = None,
                  max_prompt_tokens: Optional[int] = None) -> List[str]:
    enc = tokenizer.encode_batch(prompts)
    if max_prompt_tokens:
        enc = [e[-max_prompt_tokens:] for e in enc]
    if generator is None:
        S = max(len(e) for e in enc)
        generator = Generator(model, len(enc), S + params.max_new_tokens + 1)
    out = generator.generate(enc, params, pad_id=tokenizer.pad_token_id, eos_ids=[tokenizer.eos_token_id])
    res = []
    for b in range(len(prompts)):
        n = int(out.lengths[b])
        res.append(tokenizer.decode(out.tokens[b, :n].tolist()))
    return res


class _RowCache:
    """View of batch rows [b, b + n) of a KVCache (prefill of admitted requests)."""

    def __init__(self, cache: KVCache, b: int, n: int = 1):
        self.k = [cache.k[l, b:b + n] for l in range(cache.k.shape[0])]
        self.v = [cache.v[l, b:b + n] for l in range(cache.v.shape[0])]
        self.fp8 = cache.fp8
        if cache.fp8:
            self.ks = [cache.ks[l, b:b + n] for l in range(cache.ks.shape[0])]
            self.vs = [cache.vs[l, b:b + n] for l in range(cache.vs.shape[0])]

    def scales(self, layer: int):
        return (self.ks[layer], self.vs[layer]) if self.fp8 else (None, None)


@dataclass
class FinishedRow:
    tag: object
    tokens: List[int]
    logprobs: List[float]
    prompt_len: int
    steps_waited: int


class ContinuousBatcher:
    """Iteration-level (continuous) batching over one Generator's static cache and captured decode
    step: a request is admitted into a free batch row between decode steps — its prompt is
    prefilled into that row alone (``_RowCache``), its first token sampled from the prefill — and
    the graph-replayed decode step then advances every active row at once; each row writes at its
    own output position (``decode_update_kernel`` indexes by the row's generated length) and
    leaves the batch when it emits EOS or reaches ``max_new_tokens``, freeing the row for the next
    request. Rows are independent: other rows' K/V, positions and attention lengths are untouched
    by an admission. One sampling configuration per batcher; the decode step runs the
    power-of-two bucket of rows that covers the active ones (inactive rows in it are masked).

    Usage: ``admit(prompt_ids, tag)`` while ``free_rows()``; ``step(n)``; ``collect()`` returns the
    rows that finished (a host read of the per-row flags once per call)."""

    def __init__(self, gen: Generator, params: SamplingParams, pad_id: int = 0, eos_ids: Sequence[int] = ()):
        self.gen, self.params, self.pad_id = gen, params, pad_id
        g = gen
        dev, MB, T = g.device, g.max_batch, params.max_new_tokens
        self.T = T
        self.eos_list = list(eos_ids) or [g.cfg.eos_token_id]
        self.eos = torch.tensor(self.eos_list, dtype=torch.long, device=dev)
        g.active.zero_()
        g.gen_len.zero_()
        g.step.zero_()
        g.kv_start.zero_()
        g.kv_len.zero_()
        g.tok_in.fill_(pad_id)
        if g.out_tokens is None or g.out_tokens.shape[1] != T:
            g.out_tokens = torch.full((MB, T), pad_id, dtype=torch.long, device=dev)
            g.out_logp = torch.zeros(MB, T, dtype=torch.float32, device=dev)
            g.out_values = torch.zeros(MB, T, dtype=torch.float32, device=dev)
            g.runner.reset()
        g._nb = 1
        self._prev_merged = g.model.set_lora_merged(g.merge_lora) if hasattr(g.model, "set_lora_merged") else None
        if hasattr(g.model, "refresh_decode_weights"):
            g.model.refresh_decode_weights(MB)
        if T > 1:
            g._ensure_graph(params, self.eos, self.eos_list, pad_id, T)  # captured while no row is active
        self.rows = {}  # row -> (tag, prompt_len, steps at admission)
        self.free = list(range(MB))
        self.steps = 0

    def close(self):
        if self._prev_merged is not None:
            self.gen.model.set_lora_merged(self._prev_merged)
            self._prev_merged = None

    def free_rows(self) -> int:
        return len(self.free)

    def active_rows(self) -> int:
        return len(self.rows)

    @torch.no_grad()
    def admit(self, prompt: List[int], tag=None) -> int:
        return self.admit_many([prompt], [tag])[0]

    @torch.no_grad()
    def admit_many(self, prompts: List[List[int]], tags=None) -> List[int]:
        """Admit len(prompts) <= free_rows() requests. The lowest free rows are taken and every run
        of consecutive rows is prefilled as ONE left-padded batch into its cache rows."""
        g = self.gen
        tags = list(tags) if tags is not None else [None] * len(prompts)
        if len(prompts) > len(self.free):
            raise ValueError(f"{len(prompts)} requests for {len(self.free)} free rows")
        for p in prompts:
            if len(p) < 1 or len(p) + self.T > g.max_seq:
                raise ValueError(f"prompt of {len(p)} tokens + {self.T} new exceeds the cache ({g.max_seq})")
        self.free.sort()
        rows, self.free = self.free[:len(prompts)], self.free[len(prompts):]
        try:
            self._admit_runs(rows, prompts, tags)
        except BaseException:
            # all-or-nothing: rows of this call that were already prefilled leave the batch again
            # (inactive, back on the free list), so the caller can fail every request it passed
            for b in rows:
                self.rows.pop(b, None)
            g.active[torch.tensor(rows, device=g.device)] = 0
            self.free = sorted(self.free + rows)
            raise
        return rows

    def _admit_runs(self, rows, prompts, tags):
        g = self.gen
        i = 0
        while i < len(rows):
            j = i + 1
            while j < len(rows) and rows[j] == rows[j - 1] + 1:
                j += 1
            b0, n = rows[i], j - i
            grp = prompts[i:j]
            S = max(len(p) for p in grp)
            ids = torch.full((n, S), self.pad_id, dtype=torch.long)
            start = torch.zeros(n, dtype=torch.int32)
            for r, p in enumerate(grp):
                ids[r, S - len(p):] = torch.tensor(p, dtype=torch.long)
                start[r] = S - len(p)
            g.kv_start[b0:b0 + n].copy_(start.to(g.device, non_blocking=True))
            h_last = g.model.prefill(ids.to(g.device, non_blocking=True), g.kv_start[b0:b0 + n],
                                     _RowCache(g.cache, b0, n))
            g.kv_len[b0:b0 + n].fill_(S - 1)  # the first bookkeeping advances them to S
            g.gen_len[b0:b0 + n].zero_()
            g.active[b0:b0 + n].fill_(1)
            g._emit(h_last, self.params, self.eos, self.pad_id, r0=b0)
            for r in range(n):
                self.rows[b0 + r] = (tags[i + r], len(grp[r]), self.steps)
            i = j

    def step(self, n: int = 1):
        """n decode steps over the power-of-two bucket of rows covering every active row (rows are
        handed out lowest-first, so the active set stays compact); one captured graph per bucket."""
        g = self.gen
        nb = g._bucket(max(self.rows) + 1 if self.rows else 1)
        if nb != g._nb:
            g._nb = nb
            if self.T > 1:
                g._ensure_graph(self.params, self.eos, self.eos_list, self.pad_id, self.T)
        for _ in range(n):
            g._replay(self.params, self.eos, self.pad_id)
        self.steps += n

    def collect(self) -> List[FinishedRow]:
        """Rows that have finished since the last call (their outputs copied to the host)."""
        if not self.rows:
            return []
        g = self.gen
        act = g.active.cpu()
        done = [b for b in self.rows if not bool(act[b])]
        out = []
        if done:
            idx = torch.tensor(done, device=g.device)
            lens = g.gen_len.index_select(0, idx).cpu().tolist()
            toks = g.out_tokens.index_select(0, idx).cpu()
            lps = g.out_logp.index_select(0, idx).cpu()
            for b, n, t, lp in zip(done, lens, toks, lps):
                tag, S, s0 = self.rows.pop(b)
                out.append(FinishedRow(tag, t[:n].tolist(), lp[:n].tolist(), S, self.steps - s0))
                self.free.append(b)
        return out
