"""Typed run configuration: nested dataclasses, YAML files, ``--section.key=value`` overrides, and
named presets for the five BASELINE.json configurations.

Every magic constant of the reference (reward weights, conciseness thresholds, GAE lambda, PPO
coefficients, sampling temperature, max_length) is a named field whose default is the
reference value.
"""
from __future__ import annotations

import ast
import dataclasses
import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from .eval import EvalConfig
from .rewards import RewardConfig
from .train.ppo import PPOConfig
from .train.raft import RaftConfig
from .train.sft import SFTConfig


@dataclass
class ModelSection:
    policy: str = "mistral-7b:random"     # preset name, hub id alias, or local HF directory
    encoder: str = "minilm-l6:random"
    dtype: str = "bfloat16"
    seed: int = 0
    # fp8 (OCP e4m3fn) weight images for every no-grad policy forward: rollout prefill / decode,
    # reference scoring, RAG answers (config 5). Training forwards keep the bf16 weights.
    fp8: bool = False
    # fp8 (e4m3fn, per-slot scales) K/V cache for rollout / RAG-answer generation (config 5): half
    # the bytes the decode attention streams
    fp8_kv: bool = False
    # with fp8: the frozen base product of LoRA training forwards on the fp8 MFMA too (adapter
    # term and backward stay bf16; loss parity checked in tests/test_kernels_gpu.py)
    fp8_train: bool = False


@dataclass
class DataSection:
    train_path: Optional[str] = None       # reference-schema CSV/JSONL; None -> synthetic corpus
    docs_path: Optional[str] = None        # plain-text documents (one per line / file) for the index
    synthetic_docs: int = 100_000
    doc_words: int = 48
    n_queries: int = 2048
    batch_size: int = 64                   # per rank
    epochs: int = 1


@dataclass
class RetrievalSection:
    index: str = "ivf"                     # flat | ivf
    nlist: int = 512
    nprobe: int = 16
    top_k: int = 3
    metric: str = "ip"
    index_path: Optional[str] = None
    chunk_words: int = 120
    chunk_overlap: int = 20


@dataclass
class RunConfig:
    name: str = "run"
    out_dir: str = "runs"
    model: ModelSection = field(default_factory=ModelSection)
    data: DataSection = field(default_factory=DataSection)
    retrieval: RetrievalSection = field(default_factory=RetrievalSection)
    reward: RewardConfig = field(default_factory=RewardConfig)
    ppo: PPOConfig = field(default_factory=PPOConfig)
    sft: SFTConfig = field(default_factory=SFTConfig)
    raft: RaftConfig = field(default_factory=RaftConfig)
    eval: EvalConfig = field(default_factory=EvalConfig)
    use_wandb: bool = False


PRESETS: Dict[str, Dict[str, Any]] = {
    # 1: all-MiniLM-L6 encoder + flat top-k over 1k synthetic docs, OPT-125m greedy answer on CPU
    "config1_cpu_plumbing": {"model.policy": "opt-125m:random", "model.encoder": "minilm-l6:random",
                             "model.dtype": "float32", "data.synthetic_docs": 1000, "retrieval.index": "flat",
                             "eval.do_sample": False},
    # 2: Mistral-7B bf16 RAG answer on 1 MI355X, 100k-doc IVF index in HBM
    "config2_rag_mistral7b": {"model.policy": "mistral-7b:random", "data.synthetic_docs": 100000,
                              "retrieval.index": "ivf"},
    # 3: Mistral-7B LoRA r=16 RAFT-style SFT with distractor docs, DP=8
    "config3_raft_sft_mistral7b": {"model.policy": "mistral-7b:random", "sft.lora_r": 16, "raft.num_distractors": 3},
    # 4: Mistral-7B PPO (actor+ref+reward colocated), DP=8, hipGraph decode
    "config4_ppo_mistral7b": {"model.policy": "mistral-7b:random", "ppo.lora_r": 16, "data.batch_size": 256,
                              "ppo.minibatch_size": 32},
    # 5: Llama-2-13B full pipeline (RAG -> LoRA SFT -> PPO) on 8 GPUs
    # 256 rollouts per GPU (64 -> 128 -> 256: 3343 -> 3614 -> 4444 tokens/s on one MI355X)
    "config5_pipeline_llama13b": {"model.policy": "llama2-13b:random", "sft.lora_r": 16, "ppo.lora_r": 16,
                                  "model.fp8": True, "model.fp8_kv": True, "model.fp8_train": True,
                                  "data.batch_size": 256, "ppo.minibatch_size": 32},
}


def _coerce(val: str, typ):
    if isinstance(val, str):
        if typ is bool or isinstance(typ, type) and issubclass(typ, bool):
            return val.lower() in ("1", "true", "yes", "on")
        try:
            return ast.literal_eval(val)
        except Exception:
            return val
    return val


def set_path(cfg, dotted: str, value):
    parts = dotted.split(".")
    obj = cfg
    for p in parts[:-1]:
        obj = getattr(obj, p)
    f = {x.name: x for x in dataclasses.fields(obj)}
    if parts[-1] not in f:
        raise KeyError(f"unknown config key {dotted!r}")
    cur = getattr(obj, parts[-1])
    v = _coerce(value, type(cur) if cur is not None else str)
    if isinstance(cur, tuple) and isinstance(v, list):
        v = tuple(v)
    setattr(obj, parts[-1], v)


def from_dict(d: dict, cfg: Optional[RunConfig] = None) -> RunConfig:
    cfg = cfg or RunConfig()

    def walk(prefix, x):
        for k, v in x.items():
            key = f"{prefix}.{k}" if prefix else k
            if isinstance(v, dict):
                walk(key, v)
            else:
                set_path(cfg, key, v)
    walk("", d)
    return cfg


def load(path: Optional[str] = None, preset: Optional[str] = None, overrides: Optional[List[str]] = None) -> RunConfig:
    cfg = RunConfig()
    if preset:
        for k, v in PRESETS[preset].items():
            set_path(cfg, k, v)
    if path:
        import yaml

        with open(path) as f:
            from_dict(yaml.safe_load(f) or {}, cfg)
    for o in overrides or []:
        o = o[2:] if o.startswith("--") else o
        k, v = o.split("=", 1)
        set_path(cfg, k, v)
    return cfg


def to_dict(cfg: RunConfig) -> dict:
    return json.loads(json.dumps(dataclasses.asdict(cfg), default=str))
