"""Experiment copies of csrc/kernels/gemm_big.hip for tools/gemm_exp (timing-only diagnostics).

Round 5: MFMA issue order inside one phase of the 256x256 kernel. The K-step's 16 MFMAs of a
phase run over (A fragment i, B fragment j, k-half kk). The product kernel iterates i, j, kk, so
BOTH operand registers change between consecutive MFMAs (kk switches the A and the B half). The
kernel is bound by the clock the chip holds under its switching power (zero-filled operands run
23-27 % faster, docs/DESIGN.md), so orders that keep one operand fixed across consecutive MFMAs
are timed here:
  kij : kk, i, j -> the A half stays for NB consecutive MFMAs
  kji : kk, j, i -> the B half stays for 4 consecutive MFMAs
  ikj : i, kk, j -> the A half stays for NB consecutive MFMAs, kk inner to i
Every accumulator still receives its kk = 0 then kk = 1 product, so outputs are bitwise equal (the
harness checksum shows it). Exact string edits with counted matches: a source change that
invalidates an edit fails loudly here.

  python tools/gemm_exp/make_variants.py OUTDIR
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "csrc", "kernels", "gemm_big.hip")

L_I = '    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                           \\\n'
L_J = '      _Pragma("unroll") for (int j = 0; j < NB; ++j)                                        \\\n'
L_K = '        _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                    \\\n'


def _order(s, seq):
    old = L_I + L_J + L_K
    assert s.count(old) == 1, s.count(old)
    hdr = {"i": '_Pragma("unroll") for (int i = 0; i < 4; ++i)',
           "j": '_Pragma("unroll") for (int j = 0; j < NB; ++j)',
           "k": '_Pragma("unroll") for (int kk = 0; kk < 2; ++kk)'}
    lines = ""
    for d, c in enumerate(seq):
        txt = " " * (4 + 2 * d) + hdr[c]
        lines += txt.ljust(92) + "\\\n"
    return s.replace(old, lines)


def variants(s):
    return {"base": s, "kij": _order(s, "kij"), "kji": _order(s, "kji"), "ikj": _order(s, "ikj")}


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
