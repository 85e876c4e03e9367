"""Reference-API façade: the public classes of reinforcement_learning_optimization_after_rag.py with
identical constructor / method signatures, implemented on this framework.

Users of the reference can switch imports::

    from rag_tl_domainllm_optimizer_amd.compat import RAGEnvironment, RewardModel, PPOTrainer, RLTrainer, ModelEvaluator

``model_path`` / ``tokenizer_path`` accept a local HF-format directory or a preset / hub id (then a
random-init model of that architecture is built — there is no network); ``embedding_model_path``
likewise (default ``sentence-transformers/all-mpnet-base-v2`` as in the reference, rl.py:22).
Behavioural fixes relative to the reference are listed in SURVEY Appendix B; the formulas, defaults,
metric keys, prints and checkpoint layout are kept.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..data import RecordLoader, load_records
from ..eval import Evaluator
from ..generation import Generator, SamplingParams
from ..models import ValueHead, build_model
from ..rag.prompt import build_prompt, extract_answer
from ..retrieval import Encoder
from ..rewards import RewardModel as _BatchedReward
from ..tokenizer import load_tokenizer
from ..train.common import masked_mean, score_sequences
from ..train.ppo import PPOConfig, PPOTrainer as _PPOEngine
from .hf import HFCausalLM, CausalLMOutput  # noqa: F401

DEFAULT_EMBEDDING = "sentence-transformers/all-mpnet-base-v2"


def _device():
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _load_lm(model_path, tokenizer_path, device):
    model = build_model(model_path, device=device)
    tok = load_tokenizer(tokenizer_path if tokenizer_path else model_path, model.cfg.vocab_size, model.cfg.arch)
    return model, tok


# ----------------------------------------------------------------------------- RAGEnvironment
class RAGEnvironment:
    """rl.py:21-49. Inside :class:`RLTrainer` it shares the trained policy (rollouts from the
    current policy) instead of loading a separate never-updated copy."""

    def __init__(self, model_path, tokenizer_path, embedding_model_path=DEFAULT_EMBEDDING, *, model=None,
                 tokenizer=None):
        self.device = _device()
        if model is not None:
            self.model, self.tokenizer = model, tokenizer
            self.device = model.embed.device
        else:
            self.model, self.tokenizer = _load_lm(model_path, tokenizer_path, self.device)
        self.embedding_model_path = embedding_model_path  # the reference loads but never uses it
        self._gen = None

    @classmethod
    def from_model(cls, model, tokenizer, embedding_model_path=DEFAULT_EMBEDDING):
        return cls(None, None, embedding_model_path, model=getattr(model, "model", model), tokenizer=tokenizer)

    def generate_response(self, query, retrieved_docs, max_length=512):
        if isinstance(retrieved_docs, str):  # a CSV cell: parse list-literals / JSON
            from ..data import parse_docs

            retrieved_docs = parse_docs(retrieved_docs)
        prompt = build_prompt(query, retrieved_docs)
        ids = self.tokenizer.encode(prompt)
        if len(ids) >= max_length:
            raise ValueError(f"Input length of input_ids is {len(ids)}, but `max_length` is set to {max_length}")
        if self._gen is None or self._gen.max_seq < max_length + 1:
            self._gen = Generator(self.model, 1, max_length + 1, self.device)
        params = SamplingParams(max_new_tokens=max_length - len(ids), temperature=0.7, do_sample=True, top_k=50)
        out = self._gen.generate([ids], params, pad_id=self.tokenizer.pad_token_id,
                                 eos_ids=[self.tokenizer.eos_token_id])
        text = self.tokenizer.decode(out.tokens[0, :int(out.lengths[0])].tolist())
        return extract_answer(text)


# ----------------------------------------------------------------------------- RewardModel
class RewardModel(_BatchedReward):
    """rl.py:53-123 (weights, conciseness breakpoints, ground-truth mix identical)."""

    def __init__(self, embedding_model_path=DEFAULT_EMBEDDING):
        super().__init__(Encoder.from_name(embedding_model_path, device=_device()))
        self.embedding_model = self.encoder


# ----------------------------------------------------------------------------- PPOTrainer
class PPOTrainer:
    """rl.py:127-240, sequence-level PPO on (query -> response) pairs.

    Attributes as in the reference (rl.py:140-174): ``policy`` (HF-call-shaped, see
    :mod:`.hf`: ``policy(**inputs, labels=...)`` / ``output_hidden_states=True``), ``tokenizer``
    (HF-style call returning ``.to(device)``-able encodings), ``value_head`` (Linear(H, 1)
    semantics), ``optimizer``, ``ref_model``, ``device``.

    Fixed: a sequence's log-prob is the mean per-token log-prob of the RESPONSE given the query
    (the reference's ``-CE(policy(query), labels=response)`` raises on a length mismatch and scores
    response token t+1 at query position t, B1) — the same quantity ``-policy(**q, labels=r).loss``
    returns, so old log-probs gathered the reference's way and ``ppo_update`` agree; the value is
    read at the last real query token (B6); "entropy" is the mean token entropy (B5).
    Parameters trained: LoRA adapters + value head (fused AdamW; the reference fine-tunes all
    weights — pass ``full_finetune=True`` for that: bf16 compute copies + fp32 master on the GPU)."""

    def __init__(self, model_path, tokenizer_path, lr=5e-5, gamma=0.99, clip_range=0.2, value_coef=0.5,
                 entropy_coef=0.01, max_grad_norm=0.5, lora_r: int = 16, full_finetune: bool = False):
        self.device = _device()
        model, self.tokenizer = _load_lm(model_path, tokenizer_path, self.device)
        if self.tokenizer.pad_token_id is None:  # rl.py:143-146
            model.cfg.pad_token_id = model.cfg.eos_token_id
        self._model = model
        self.policy = HFCausalLM(model, self.tokenizer)
        self.value_head = ValueHead(model.cfg.hidden_size, device=self.device)
        self._ref_copy = None
        if full_finetune:
            # the reference's mode (rl.py:153-156): every weight trains; the frozen reference is a
            # copy of the starting weights (rl.py:171-174)
            import copy

            self._ref_copy = copy.deepcopy(model).requires_grad_(False)
            params = list(model.parameters())
        else:
            model.add_lora(lora_r, 2.0 * lora_r, "all")
            model.freeze_base()
            params = model.lora_parameters()
        self.flat = ops.flat_params(list(params) + list(self.value_head.parameters()))
        model.refresh_lora()
        self.optimizer = ops.FusedAdamW(self.flat, lr=lr, weight_decay=0.01, max_grad_norm=max_grad_norm)
        self.gamma, self.clip_range = gamma, clip_range
        self.value_coef, self.entropy_coef, self.max_grad_norm = value_coef, entropy_coef, max_grad_norm
        self.full_finetune = full_finetune
        self.engine = None

    @classmethod
    def from_engine(cls, engine: _PPOEngine) -> "PPOTrainer":
        """The reference-shaped view of a token-level PPO engine: same policy, tokenizer, value head,
        optimizer and frozen reference (what :class:`RLTrainer` exposes as ``ppo_trainer``)."""
        self = cls.__new__(cls)
        c = engine.cfg
        self.engine = engine
        self.device = engine.device
        self._model = engine.policy
        self.tokenizer = engine.tok
        self.policy = HFCausalLM(engine.policy, engine.tok)
        self.value_head = engine.value_head
        self.flat = engine.flat
        self.optimizer = engine.opt
        self._ref_copy = engine.ref_policy
        self.gamma, self.clip_range = c.gamma, c.clip_range
        self.value_coef, self.entropy_coef, self.max_grad_norm = c.value_coef, c.entropy_coef, c.max_grad_norm
        self.full_finetune = c.full_finetune
        return self

    @property
    def ref_model(self):
        """The frozen reference: base weights with LoRA disabled (no third model copy), or the
        starting-weight copy under full fine-tuning. HF-call-shaped like ``policy``."""
        return _RefView(self._ref_copy if self._ref_copy is not None else self._model, self.tokenizer)

    def compute_advantages(self, rewards, values, dones, next_value=0):
        """Exactly rl.py:176-191 (GAE over the batch, lambda 0.95)."""
        advantages = []
        advantage = 0
        for i in reversed(range(len(rewards))):
            if i == len(rewards) - 1:
                next_value = 0 if dones[i] else next_value
            else:
                next_value = values[i + 1]
            delta = rewards[i] + self.gamma * next_value * (1 - dones[i]) - values[i]
            advantage = delta + self.gamma * 0.95 * (1 - dones[i]) * advantage
            advantages.insert(0, advantage)
        return advantages

    def _pack(self, query_batch, response_batch):
        q = [self.tokenizer.encode(x) for x in query_batch]
        r = [self.tokenizer.encode(x, add_special_tokens=False) or [self.tokenizer.eos_token_id]
             for x in response_batch]
        pq = self.tokenizer.pad(q, side="left", device=self.device)
        pr = self.tokenizer.pad(r, side="right", device=self.device)
        return pq["input_ids"], pq["start"], pr["input_ids"], pr["lengths"]

    def sequence_logprobs(self, query_batch, response_batch, with_value=True):
        """-> (mean token log-prob of each response given its query [B], mean entropy, value [B])."""
        qi, qs, ri, rl_ = self._pack(query_batch, response_batch)
        # one forward (B7): the value of the state after the query is read at the last query
        # position, which is also the row that predicts response token 0 (B6)
        lp, ent, vals, mask = score_sequences(self._model, qi, qs, ri, rl_, 1.0,
                                              self.value_head if with_value else None)
        mf = mask.to(lp.dtype)
        seq_lp = (lp * mf).sum(-1) / mf.sum(-1).clamp(min=1.0)
        return seq_lp, masked_mean(ent, mask), (vals[:, 0] if with_value else None)

    def ppo_update(self, query_batch, response_batch, old_log_probs, rewards, values, advantages):
        """rl.py:193-240: clipped surrogate + 0.5*MSE(value, reward) + entropy term; returns the
        reference's 5 metrics."""
        log_probs, entropy, value_preds = self.sequence_logprobs(query_batch, response_batch)
        old_log_probs = torch.as_tensor(old_log_probs).to(self.device).float()
        advantages = torch.as_tensor(advantages).to(self.device).float()
        rewards = torch.as_tensor(rewards).to(self.device).float()
        ratio = torch.exp(log_probs - old_log_probs)
        surr1 = ratio * advantages
        surr2 = torch.clamp(ratio, 1.0 - self.clip_range, 1.0 + self.clip_range) * advantages
        policy_loss = -torch.min(surr1, surr2).mean()
        value_loss = 0.5 * ((value_preds - rewards) ** 2).mean()
        entropy_loss = -self.entropy_coef * entropy
        loss = policy_loss + self.value_coef * value_loss + entropy_loss
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        if not self.full_finetune:
            self._model.refresh_lora()
        return {"policy_loss": policy_loss.item(), "value_loss": value_loss.item(),
                "entropy_loss": entropy_loss.item(), "total_loss": loss.item(),
                "approx_kl": (old_log_probs - log_probs.detach()).mean().item()}


class _RefView(HFCausalLM):
    """The frozen reference, HF-call-shaped; adapters are switched off for the call."""

    def __init__(self, model, tokenizer=None):
        super().__init__(model, tokenizer)

    def forward(self, *a, **k):
        self.model.set_lora_enabled(False)
        try:
            with torch.no_grad():
                return super().forward(*a, **k)
        finally:
            self.model.set_lora_enabled(True)

    def parameters(self, recurse: bool = True):
        return (p for n, p in self.model.named_parameters() if "lora" not in n)


# ----------------------------------------------------------------------------- RLTrainer
class RLTrainer:
    """rl.py:244-379: epochs x batches of PPO after RAG, best/epoch checkpoints, wandb-style logging
    (JSONL sink; wandb only if installed).

    ``env`` is a :class:`RAGEnvironment` and ``ppo_trainer`` a :class:`PPOTrainer`, both on ONE
    shared policy, so code written against the reference's attributes (``env.generate_response``,
    ``ppo_trainer.{tokenizer, policy, value_head, device, optimizer, ref_model,
    compute_advantages, ppo_update}``, rl.py:293,309-334,367-376) runs unchanged. ``train`` itself
    runs the batched token-level engine (``self.engine``): one batched rollout on the GPU, reward
    on a side stream, frozen-reference KL, token GAE, minibatched clipped updates."""

    def __init__(self, model_path, tokenizer_path, embedding_model_path=DEFAULT_EMBEDDING, lr=5e-5, batch_size=8,
                 epochs=5, wandb_project="rl-after-rag", checkpoint_dir="./rl_model_checkpoints", **ppo_overrides):
        from ..utils import MetricsSink

        self.device = _device()
        policy, tok = _load_lm(model_path, tokenizer_path, self.device)
        self.reward_model = RewardModel(embedding_model_path)
        cfg = PPOConfig(lr=lr, **ppo_overrides)
        self.sink = MetricsSink(os.path.join(checkpoint_dir, "logs"), project=wandb_project,
                                use_wandb=os.environ.get("RAGTL_WANDB") == "1", config={"lr": lr, "batch_size": batch_size})
        self.engine = _PPOEngine(policy, tok, self.reward_model, cfg, sink=self.sink, max_batch=batch_size)
        self.ppo_trainer = PPOTrainer.from_engine(self.engine)
        # rollouts come from the current policy: the environment shares it
        self.env = RAGEnvironment.from_model(policy, tok, embedding_model_path)
        self.batch_size, self.epochs, self.checkpoint_dir = batch_size, epochs, checkpoint_dir
        os.makedirs(checkpoint_dir, exist_ok=True)

    def prepare_data(self, data_path):
        return RecordLoader(load_records(data_path), self.batch_size, shuffle=True)

    def train(self, data_loader):
        best_reward = -float("inf")
        for epoch in range(self.epochs):
            if hasattr(data_loader, "set_epoch"):
                data_loader.set_epoch(epoch)
            epoch_rewards, epoch_losses = [], []
            for batch in data_loader:
                m = self.engine.step(batch)
                epoch_rewards.extend(self.engine.last_rollout.scores.tolist())
                epoch_losses.append(m["total_loss"])
            avg_reward = float(np.mean(epoch_rewards)) if epoch_rewards else float("nan")
            print(f"Epoch {epoch + 1}/{self.epochs}: Average Reward = {avg_reward:.4f}, "
                  f"Average Loss = {np.mean(epoch_losses):.4f}")
            if avg_reward > best_reward:
                best_reward = avg_reward
                self.save_checkpoint(f"{self.checkpoint_dir}/best_model", epoch, best_reward)
            self.save_checkpoint(f"{self.checkpoint_dir}/epoch_{epoch + 1}", epoch, best_reward)
        return best_reward

    def save_checkpoint(self, path, epoch=0, best=-math.inf):
        self.engine.save_checkpoint(path, epoch, best)

    def load_checkpoint(self, path):
        return self.engine.load_checkpoint(path)


# ----------------------------------------------------------------------------- ModelEvaluator
class ModelEvaluator:
    """rl.py:381-463."""

    def __init__(self, embedding_model_path=DEFAULT_EMBEDDING):
        self.reward_model = RewardModel(embedding_model_path)
        self.evaluator = Evaluator(self.reward_model)

    def evaluate_model(self, model, tokenizer, test_data):
        return self.evaluator.evaluate_model(model, tokenizer, test_data)

    def compare_models(self, base_model, rag_model, rl_model, transfer_model=None, test_data=None):
        models = {"Base Model": base_model, "RAG Model": rag_model, "RL-finetuned Model": rl_model}
        if transfer_model:
            models["Transfer-learned Model"] = transfer_model
        return self.evaluator.compare_models(models, test_data)


def main(model_path: str = "tiny-llama:random", embedding_model_path: str = "tiny-bert:random",
         checkpoint_dir: str = "./rl_model_checkpoints", epochs: int = 1):
    """rl.py:467-531 on synthetic data (no network): train, evaluate base / RAG / RL, write the CSV."""
    import tempfile

    from ..data import SyntheticCorpus
    from ..tokenizer import load_tokenizer as _lt

    dev = _device()
    base, tok = _load_lm(model_path, model_path, dev)
    corpus = SyntheticCorpus(tok.words(), n_docs=64, doc_words=24)
    path = os.path.join(tempfile.mkdtemp(), "train.csv")
    corpus.to_csv(path, 32, k_docs=2)
    trainer = RLTrainer(model_path, model_path, embedding_model_path, lr=5e-5, batch_size=8, epochs=epochs,
                        checkpoint_dir=checkpoint_dir, max_new_tokens=16, max_prompt_tokens=160, minibatch_size=4)
    trainer.train(trainer.prepare_data(path))
    evaluator = ModelEvaluator(embedding_model_path)
    items = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
             for it in corpus.sample_queries(4, seed=5)]
    rl_model = trainer.engine.policy
    report = evaluator.compare_models((base, tok), (base, tok), (rl_model, trainer.ppo_trainer.tokenizer), test_data=items)
    print("Model Comparison Report:")
    print(report)
    report.to_csv("model_comparison_results.csv")
    return report
