"""Host C++ under AddressSanitizer + UBSan: the tokenizer runtime and IVF host
helpers are exercised from a child python with the sanitizer runtimes preloaded. GPU code is never
sanitized (not available on the pool); this runs on the CPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import numpy as np, torch
from rag_tl_domainllm_optimizer_amd.ops import native
from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
C = native()
for arch in ("llama", "bert", "opt", "mistral"):
    tok = Tokenizer.synthetic(4096, arch)
    texts = ["hello world " * 30, "", "Ünïcödé ✓ bytes \x00 \t tabs", "a" * 5000, "what is the answer ?"]
    ids = tok.encode_batch(texts * 20)
    for t, i in zip(texts, ids[:5]):
        tok.decode(i)
    tok.pad(ids[:7])
emb = torch.randn(3000, 32)
assign = torch.randint(0, 17, (3000,))
lists = C.ivf_build_lists(assign, 17) if hasattr(C, "ivf_build_lists") else None
if hasattr(C, "kmeanspp_init"):
    C.kmeanspp_init(emb, 17, 0)
print("asan-ok")
"""


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(900)
def test_host_code_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    sys.path.insert(0, ROOT)
    from rag_tl_domainllm_optimizer_amd._build import build

    so = build(sanitize=True)
    env = dict(os.environ, RAGTL_EXT_PATH=so, LD_PRELOAD=f"{asan}:{ubsan}", PYTHONPATH=ROOT,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               RAGTL_AUTOBUILD="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-4000:]
