"""Seeding and RNG-state capture (for exact resume)."""
from __future__ import annotations

import random

import numpy as np
import torch


def seed_everything(seed: int):
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def rng_state() -> dict:
    st = {"python": random.getstate(), "numpy": np.random.get_state(), "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: dict):
    random.setstate(st["python"])
    np.random.set_state(st["numpy"])
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def rng_state_pack(st: dict):
    """(tensors, meta) form of an ``rng_state()`` dict for safetensors + JSON (no pickle)."""
    tensors = {"torch": st["torch"].clone().contiguous()}
    if "cuda" in st:
        tensors["cuda"] = st["cuda"].clone().contiguous()
    name, keys, pos, has_gauss, cached = st["numpy"]
    tensors["numpy_keys"] = torch.from_numpy(np.asarray(keys, dtype=np.int64))
    ver, internal, gauss = st["python"]
    meta = {"python": {"version": ver, "state": list(internal), "gauss": gauss},
            "numpy": {"name": name, "pos": int(pos), "has_gauss": int(has_gauss), "cached_gaussian": float(cached)}}
    return tensors, meta


def rng_state_unpack(tensors: dict, meta: dict) -> dict:
    py, npm = meta["python"], meta["numpy"]
    st = {"python": (py["version"], tuple(py["state"]), py["gauss"]),
          "numpy": (npm["name"], tensors["numpy_keys"].numpy().astype(np.uint32), npm["pos"], npm["has_gauss"],
                    npm["cached_gaussian"]),
          "torch": tensors["torch"]}
    if "cuda" in tensors:
        st["cuda"] = tensors["cuda"]
    return st
