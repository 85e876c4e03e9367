"""HF-call-shaped view of a :class:`~..models.CausalLM` for reference-style code.

The reference drives its policy through the HF ``AutoModelForCausalLM`` calling convention
(reinforcement_learning_optimization_after_rag.py:200, 207-208, 313, 318-319)::

    out = policy(**tokenizer(query, return_tensors="pt").to(device), labels=response_ids)
    logp = -out.loss
    h = policy(**inputs, output_hidden_states=True).hidden_states[-1][:, -1, :]

:class:`HFCausalLM` accepts exactly that and runs it on this framework's forward (flash
attention, fused GEMMs). Every other attribute (``cfg``, ``layers``, ``refresh_lora``,
``set_lora_enabled`` …) is forwarded to the wrapped model.

``labels`` semantics (SURVEY B1 fix). HF computes a shifted cross-entropy of ``labels`` against
the positions of ``input_ids``; the reference passes the RESPONSE ids there, which raises unless
query and response tokenize to the same length and otherwise scores response token t+1 at query
position t. Here:

* ``labels`` that mirror ``input_ids`` (equal, or -100 where ignored) → the standard shifted
  causal-LM loss, exactly as HF;
* any other ``labels`` → a continuation: the loss is the mean negative log-likelihood of the
  label tokens GIVEN the input tokens (sequence = [input | labels]). -100 entries, leading /
  trailing runs of the pad id and a leading BOS (the tokenizer's template) are not scored.
  ``out.seq_logprobs`` [B] holds each row's mean token log-prob (= ``-out.loss`` at batch 1).

``hidden_states`` is a tuple of length ``num_layers + 1`` as in HF, but only the last entry (the
final post-norm hidden state, the one the reference reads) is materialised; the others are None.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from ..train.common import score_sequences


class CausalLMOutput:
    """``loss`` / ``logits`` (computed on first access) / ``hidden_states`` / ``seq_logprobs``."""

    def __init__(self, model, hidden: Optional[torch.Tensor], loss=None, seq_logprobs=None, num_layers: int = 0,
                 want_hidden: bool = False):
        self._model, self._hidden, self._logits = model, hidden, None
        self.loss = loss
        self.seq_logprobs = seq_logprobs
        self.hidden_states = ((None,) * num_layers + (hidden,)) if (want_hidden and hidden is not None) else None

    @property
    def logits(self):
        if self._logits is None and self._hidden is not None:
            B, S, H = self._hidden.shape
            h = self._hidden.reshape(B * S, H)
            lg = ops.linear(h, self._model.head_weight) if h.requires_grad else \
                ops.gemm(h.contiguous(), self._model.head_weight)
            self._logits = lg.float().view(B, S, -1)
        return self._logits

    def __getitem__(self, k):
        return getattr(self, k)


def _left_pack(input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor]):
    """-> (left-padded ids, start [B], gather index [B, S] from the original layout into the
    left-padded one or None when the input is already left-padded)."""
    B, S = input_ids.shape
    if attention_mask is None:
        return input_ids, torch.zeros(B, dtype=torch.long, device=input_ids.device), None
    m = attention_mask.to(torch.long)
    n = m.sum(1)
    start = S - n
    left = (m == (torch.arange(S, device=m.device)[None, :] >= start[:, None]).long()).all()
    if bool(left):
        return input_ids, start, None
    # right (or arbitrary) padding: move each row's real tokens to the end, keeping their order
    order = torch.argsort(m, dim=1, stable=True)  # zeros first, then real tokens in order
    ids = torch.gather(input_ids, 1, order)
    return ids, start, order


class HFCausalLM(torch.nn.Module):
    def __init__(self, model, tokenizer=None):
        super().__init__()
        self.model = model
        self._pad_id = getattr(tokenizer, "pad_token_id", None)
        self._bos_id = getattr(tokenizer, "bos_token_id", None)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._modules["model"], name)

    @property
    def config(self):
        return self.model.cfg

    @property
    def device(self):
        return self.model.embed.device

    def save_pretrained(self, path: str):
        """HF layout with every LoRA adapter folded into the weights (any HF loader reads it)."""
        from ..train.checkpoint import save_policy

        save_policy(self.model, path)

    def _strip(self, row: torch.Tensor):
        toks = [int(t) for t in row.tolist() if int(t) != -100]
        if self._pad_id is not None:
            while toks and toks[0] == self._pad_id:
                toks.pop(0)
            while toks and toks[-1] == self._pad_id:
                toks.pop()
        if self._bos_id is not None and len(toks) > 1 and toks[0] == self._bos_id:
            toks.pop(0)
        return toks

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None, output_hidden_states: bool = False, return_dict: bool = True,
                **unused):
        model = self.model
        dev = model.embed.device
        input_ids = input_ids.to(dev)
        if input_ids.dim() == 1:
            input_ids = input_ids[None]
        attention_mask = attention_mask.to(dev) if attention_mask is not None else None
        B, S = input_ids.shape
        L = len(model.layers)
        ids, start, order = _left_pack(input_ids, attention_mask)
        standard = labels is not None and labels.shape == input_ids.shape and bool(
            ((labels.to(dev) == input_ids) | (labels.to(dev) == -100)).all())
        if labels is not None and not standard:
            # continuation: mean NLL of the label tokens given the input tokens (B1 fix)
            resp = [self._strip(r) for r in labels.to("cpu").reshape(B, -1)]
            resp = [r if r else [model.cfg.eos_token_id] for r in resp]
            T = max(len(r) for r in resp)
            rt = torch.full((B, T), self._pad_id if self._pad_id is not None else 0, dtype=torch.long)
            for b, r in enumerate(resp):
                rt[b, :len(r)] = torch.tensor(r, dtype=torch.long)
            rl = torch.tensor([len(r) for r in resp], dtype=torch.long, device=dev)
            lp, _, _, mask = score_sequences(model, ids, start, rt.to(dev), rl)
            mf = mask.to(lp.dtype)
            seq_lp = (lp * mf).sum(-1) / mf.sum(-1).clamp(min=1.0)
            loss = -(lp * mf).sum() / mf.sum().clamp(min=1.0)
            hidden = None
            if output_hidden_states:
                hidden = model(ids, kv_start=start).view(B, S, -1)
            return CausalLMOutput(model, self._unpack(hidden, order), loss, seq_lp, L, output_hidden_states)
        hidden = model(ids, kv_start=start).view(B, S, -1)
        loss = None
        if standard:
            lab = torch.gather(labels.to(dev), 1, order) if order is not None else labels.to(dev)
            tgt = lab[:, 1:]
            keep = tgt != -100
            if attention_mask is not None:
                keep &= torch.arange(1, S, device=dev)[None, :] >= start[:, None] + 1
            h = hidden[:, :-1].reshape(-1, hidden.shape[-1])
            logits = ops.linear(h, model.head_weight) if h.requires_grad else ops.gemm(h.contiguous(), model.head_weight)
            lp, _ = ops.token_logprobs(logits, torch.where(keep, tgt, torch.full_like(tgt, -100)).reshape(-1), 1.0)
            kf = keep.reshape(-1).to(lp.dtype)
            loss = -(lp * kf).sum() / kf.sum().clamp(min=1.0)
        return CausalLMOutput(model, self._unpack(hidden, order), loss, None, L, output_hidden_states)

    @staticmethod
    def _unpack(hidden, order):
        """Back to the caller's layout (only when the input was not left-padded)."""
        if hidden is None or order is None:
            return hidden
        out = torch.empty_like(hidden)
        idx = order[:, :, None].expand_as(hidden)
        return out.scatter(1, idx, hidden)
