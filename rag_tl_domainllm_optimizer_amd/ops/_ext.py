"""Loader for the native extension ``_C``.

GPU tensors always go through the HIP kernels. If the extension is missing or fails to load,
every op called with a GPU tensor raises immediately (no silent eager fallback on the GPU); CPU
tensors use the eager reference implementations in :mod:`.reference`.
"""
from __future__ import annotations

import importlib
import importlib.util
import os

_C = None
_err: Exception | None = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return
    alt = os.environ.get("RAGTL_EXT_PATH")
    if alt:  # e.g. the host-sanitizer build (python -m rag_tl_domainllm_optimizer_amd._build --sanitize)
        spec = importlib.util.spec_from_file_location("rag_tl_domainllm_optimizer_amd._C", alt)
        _C = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(_C)
        return
    try:
        _C = importlib.import_module("rag_tl_domainllm_optimizer_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        if os.environ.get("RAGTL_AUTOBUILD", "1") == "1":
            try:
                from .._build import build

                build()
                _C = importlib.import_module("rag_tl_domainllm_optimizer_amd._C")
                return
            except Exception as e2:
                _err = e2
                return
        _err = e


def native():
    """Return the native module, raising a clear error if it cannot be loaded."""
    _load()
    if _C is None:
        raise RuntimeError(
            "native extension rag_tl_domainllm_optimizer_amd._C is not available "
            f"({_err!r}); build it with `python -m rag_tl_domainllm_optimizer_amd._build`"
        )
    return _C


def native_available() -> bool:
    _load()
    return _C is not None


def on_gpu(*ts) -> bool:
    for t in ts:
        if t is not None and hasattr(t, "is_cuda"):
            return bool(t.is_cuda)
    return False


def get_tuning() -> dict:
    """The native launchers' kernel-selection knobs (csrc/include/rt_tuning.h: A/B switches of the
    measured alternatives, forced split-K factors) as a dict."""
    return dict(native().get_tuning())


def set_tuning(**fields) -> dict:
    """Update knobs by name (unknown names raise); returns the previous values of those fields."""
    cur = get_tuning()
    unknown = [k for k in fields if k not in cur]
    if unknown:
        raise KeyError(f"unknown tuning field(s): {unknown}; known: {sorted(cur)}")
    native().set_tuning(dict(fields))
    return {k: cur[k] for k in fields}


class tuning:
    """Context manager: ``with ops.tuning(decode_split=2): ...`` sets knobs and restores them."""

    def __init__(self, **fields):
        self.fields = fields
        self.prev = None

    def __enter__(self):
        self.prev = set_tuning(**self.fields)
        return self

    def __exit__(self, *exc):
        native().set_tuning(self.prev)
