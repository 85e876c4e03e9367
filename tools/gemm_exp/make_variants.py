"""Experiment copies of csrc/kernels/gemm_big.hip for tools/gemm_exp (timing-only diagnostics).

Each variant removes ONE kind of stall from the 256x256 kernel's steady-state loop so its time
shows how much that stall costs. Variants that drop a wait compute WRONG results on purpose; they
are never built into the extension. Exact string edits with counted matches, so a source change
that invalidates an edit fails loudly here instead of silently producing the base kernel.

  python tools/gemm_exp/make_variants.py OUTDIR
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "csrc", "kernels", "gemm_big.hip")


def _fast_loop_span(s):
    """The two-buffer steady-state loop of gemm_big_kernel (the RING form has its own loop)."""
    a = 0
    while True:
        a = s.index("for (; t < t_fast; ++t) {", a)
        b = s.index("for (; t < t_end; ++t) {", a)
        if "stage_fast(" in s[a:b]:
            return a, b
        a = b


def _sub_in(s, span, old, new, count):
    a, b = span
    body = s[a:b]
    n = body.count(old)
    assert n == count, (old, n, count)
    return s[:a] + body.replace(old, new) + s[b:]


def _macro_line(s, needle, repl, count):
    # GB_MMA_X lines end in padding + backslash: replace the statement, keep the continuation
    pat = re.compile(r"^(\s*)" + re.escape(needle) + r"(\s*\\)$", re.M)
    out, n = pat.subn(lambda m: m.group(1) + repl + m.group(2), s)
    assert n == count, (needle, n, count)
    return out


def variants(s):
    v = {"base": s}
    # the steady-state loop without its counted LDS-DMA waits (granules may not have landed)
    v["nowait"] = _sub_in(s, _fast_loop_span(s), "wait_granules<BN>(4);", "", 3)
    # GB_MMA without the barrier that closes each MFMA cluster (the stagger then drifts)
    t = s.replace("    __builtin_amdgcn_s_setprio(0);                                                          \\\n"
                  "    GB_BARRIER();                                                                           \\\n",
                  "    __builtin_amdgcn_s_setprio(0);                                                          \\\n", 1)
    assert t != s
    v["nobar_end"] = t
    # no priority raise around the MFMA clusters
    v["noprio"] = _macro_line(s, "__builtin_amdgcn_s_setprio(1);", ";", 2)
    # MFMAs start without waiting for the fragment reads (LDS latency exposure)
    v["nolgkm"] = _macro_line(s, 'asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");', ";", 2)
    # both: no DMA waits and no closing barrier
    v["nowait_nobar_end"] = _sub_in(t, _fast_loop_span(t), "wait_granules<BN>(4);", "", 3)
    # no operand traffic in the steady state: no LDS-DMA issue (the waits then return at once)
    nodma = _sub_in(s, _fast_loop_span(s), "stage_fast(", "if (0) stage_fast(", 4)
    v["nodma"] = nodma
    # no fragment reads from LDS in the steady state (MFMAs on the registers' stale contents)
    noread = _sub_in(s, _fast_loop_span(s), "read_a(buf, ", "if (0) read_a(buf, ", 2)
    noread = _sub_in(noread, _fast_loop_span(noread), "read_b(buf, ", "if (0) read_b(buf, ", 2)
    v["noread"] = noread
    # barriers + MFMAs only (no DMA, no reads): the schedule's ceiling
    both = _sub_in(nodma, _fast_loop_span(nodma), "read_a(buf, ", "if (0) read_a(buf, ", 2)
    both = _sub_in(both, _fast_loop_span(both), "read_b(buf, ", "if (0) read_b(buf, ", 2)
    v["mfma_bar"] = both
    # 4-wave kernel (gemm_w4_kernel, bn = 4): its stage loop without the LDS-DMA waits
    a = s.index("auto stage_body = [&](int s, bool fast) {")
    b = s.index("---- epilogue ----", a)
    body = s[a:b]
    w = 'if (fast || more2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(G::DMA) : "memory");'
    assert body.count(w) == 1, body.count(w)
    v["w4nowait"] = s[:a] + body.replace(w, "if (0) {}") + s[b:]
    return v


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    s = open(SRC).read()
    for name, text in variants(s).items():
        with open(os.path.join(out, f"gemm_big_{name}.hip"), "w") as f:
            f.write(text)
        print(name)


if __name__ == "__main__":
    main()
