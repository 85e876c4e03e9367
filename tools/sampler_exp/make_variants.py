"""Timing-only copies of csrc/kernels/sampling.hip that stop the top-k search kernel after a phase
(the row's output token is still written), so tools/sampler_exp/main.cpp can price each phase of
the batch-1 sampler. Exact string edits with counted matches.

  python tools/sampler_exp/make_variants.py OUTDIR
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "csrc", "kernels", "sampling.hip")

P1 = "  const float M = key16_to_f(KM) * inv_temp;\n  // pass 2:"
P2 = "  const int AM = amin;\n\n  int tok = AM;\n"
P3 = "    }\n    __syncthreads();\n    const bool overflow = cnt > TK_CAP;"
EXIT = "  if (use_window >= 100) { if (tid == 0) out_tok[row] = (long)KM; return; }\n"


def _sub(s, old, new):
    assert s.count(old) == 1, (old, s.count(old))
    return s.replace(old, new)


def variants(s):
    # edits apply inside sample_topk_search_kernel only (the other kernels share some lines)
    cut = s.index("void sample_topk_search_kernel(")
    head, body = s[:cut], s[cut:]
    body = _sub(body, "    if (use_window) {\n", "    if (use_window % 100) {\n")
    out = {"full": s}
    out["p1"] = head + _sub(body, P1, EXIT + P1)
    out["p2"] = head + _sub(body, P2, P2 + EXIT)
    out["p3"] = head + _sub(body, P3, "    }\n    __syncthreads();\n" + EXIT + "    const bool overflow = cnt > TK_CAP;")
    out["pA"] = head + _sub(body, "      const int n = cnt;\n", "      const int n = cnt;\n" + EXIT)
    out["pB"] = head + _sub(body, "          if (lane == 0) cnt = ns;\n        }\n",
                            "          if (lane == 0) cnt = ns;\n        }\n" + EXIT)
    return out


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    s = open(SRC).read()
    for name, text in variants(s).items():
        with open(os.path.join(out, f"sampling_{name}.hip"), "w") as f:
            f.write(text)
        print(name)


if __name__ == "__main__":
    main()
