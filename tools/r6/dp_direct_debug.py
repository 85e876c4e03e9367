"""Debug: 2-rank gloo DP on one GPU (tests/test_zz_dist_gpu.py setup) with the LoRA gradient
epilogue off / on / on-without-readiness-hooks: do the ranks hold the same reduced gradient, and
which flat-buffer parameters differ."""
import os
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def worker(rank, world, port, out_dir, mode):
    import importlib

    import test_zz_dist_gpu as T

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), RAGTL_DIST_BACKEND="gloo")
    L = importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear")
    L.DIRECT_LORA_GRADS = mode != "off"
    from rag_tl_domainllm_optimizer_amd import parallel

    di = parallel.init(device="cuda")
    tok, tr = T._setup(di.device)
    if mode == "nohook":
        for p in tr.flat.params:
            if hasattr(p, "_rt_grad_ready"):
                del p._rt_grad_ready
    mine = T._examples(tok)[rank::world]
    tr.opt.zero_grad()
    tr.sync.start()
    ids, start, tgt = tr.encode([e["prompt"] for e in mine], [e["answer"] for e in mine])
    loss, _ = tr.loss(ids, start, tgt)
    loss.backward()
    ready = list(tr.sync._ready)
    launched = [h is not None for h in tr.sync._handles]
    tr.sync.finish()
    torch.cuda.synchronize()
    torch.save({"g": tr.flat.grad.cpu(), "offsets": list(tr.flat.offsets), "need": list(tr.sync.need),
                "ready": ready, "launched": launched, "buckets": list(tr.sync.buckets)},
               os.path.join(out_dir, f"{mode}{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


if __name__ == "__main__":
    import tempfile

    import test_zz_dist_gpu as T

    d = tempfile.mkdtemp()
    for mode in ("off", "on", "nohook"):
        mp.start_processes(worker, args=(2, T._free_port(), d, mode), nprocs=2, start_method="spawn", join=True)
        a, b = torch.load(os.path.join(d, f"{mode}0.pt")), torch.load(os.path.join(d, f"{mode}1.pt"))
        diff = (a["g"] - b["g"]).abs()
        bad = [i for i, (s, e) in enumerate(zip(a["offsets"], a["offsets"][1:] + [a["g"].numel()]))
               if float(diff[s:e].max()) > 0]
        print(f"{mode}: max |rank0 - rank1| = {float(diff.max()):.3e}, differing params {bad[:20]} of {len(a['offsets'])}; "
              f"ready {a['ready']} need {a['need']} launched-by-hooks {sum(a['launched'])}/{len(a['launched'])}",
              flush=True)
