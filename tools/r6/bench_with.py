#!/usr/bin/env python3
"""Run bench.py with module-level Python switches set first (same-box A/B of host-side plans):
    python tools/r6/bench_with.py rag_tl_domainllm_optimizer_amd.ops.linear.SLAB_SPLITS_R6=0 -- --steps 3 --warmup 1
"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    sep = args.index("--") if "--" in args else len(args)
    for spec in args[:sep]:
        path, val = spec.split("=")
        mod, attr = path.rsplit(".", 1)
        setattr(importlib.import_module(mod), attr, type(getattr(importlib.import_module(mod), attr))(int(val)))
    sys.argv = [os.path.join(ROOT, "bench.py")] + args[sep + 1:]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
