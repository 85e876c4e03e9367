"""Data parallelism through the GPU kernels: 2 ranks (gloo, both on cuda:0 — RCCL needs one GPU per
rank, this box has one) run the LoRA SFT backward on their shards with the bucketed all-reduce;
the reduced flat gradient equals one process accumulating the same shards on the same GPU. Covers
the native adapter-gradient path (shared zero-filled accumulators, views handed to autograd) under
the post-accumulate all-reduce hooks, which the CPU tests (eager oracle path) cannot reach."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _examples(tok, n=8):
    words = tok.words()
    return [{"prompt": " ".join(words[i:i + 40]), "answer": " ".join(words[90 + i:90 + i + 12])} for i in range(n)]


def _setup(device):
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.sft import SFTConfig, SFTTrainer

    torch.manual_seed(0)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    m = models.CausalLM(cfg, device=device, dtype=torch.bfloat16, seed=1)
    tr = SFTTrainer(m, tok, SFTConfig(lr=1e-2, lora_r=8, lr_schedule="constant", warmup_steps=0, batch_size=4,
                                      bucket_mb=1 / 64))
    g = torch.Generator(device="cpu").manual_seed(5)
    with torch.no_grad():
        for p in m.lora_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.05)
    m.refresh_lora()
    return tok, tr


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), RAGTL_DIST_BACKEND="gloo")
    from rag_tl_domainllm_optimizer_amd import parallel

    di = parallel.init(device="cuda")
    tok, tr = _setup(di.device)
    mine = _examples(tok)[rank::world]
    tr.opt.zero_grad()
    tr.sync.start()
    ids, start, tgt = tr.encode([e["prompt"] for e in mine], [e["answer"] for e in mine])
    loss, _ = tr.loss(ids, start, tgt)
    loss.backward()
    tr.sync.finish()
    torch.cuda.synchronize()
    torch.save(tr.flat.grad.cpu(), os.path.join(out_dir, f"dp{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


def test_dp_lora_grads_gpu_equal_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    dp0, dp1 = torch.load(tmp_path / "dp0.pt"), torch.load(tmp_path / "dp1.pt")
    assert torch.equal(dp0, dp1)  # every rank holds the same reduced gradient
    tok, tr = _setup(torch.device("cuda"))
    ex = _examples(tok)
    tr.opt.zero_grad()
    for r in range(world):
        shard = ex[r::world]
        ids, start, tgt = tr.encode([e["prompt"] for e in shard], [e["answer"] for e in shard])
        loss, _ = tr.loss(ids, start, tgt)
        (loss / world).backward()
    tr.flat.relink_grads()
    ref = tr.flat.grad.cpu()
    assert ref.abs().sum() > 0
    torch.testing.assert_close(dp0, ref, rtol=2e-3, atol=1e-5)
