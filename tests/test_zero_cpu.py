"""ZeRO-1 (parallel.zero.ZeroAdamW) on CPU with gloo at world 2 / 4 / 8: the sharded optimizer step
equals one process running AdamW (+ global-norm clipping) on the fp32 mean of the ranks' bf16
gradients, for bf16 members and the replicated fp32 tail; per-rank state at world 8 for Mistral-7B
is <= 40 GB; a sharded checkpoint round trip resumes bitwise."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

SIZES16 = [4096 + 40, 96, 3000, 128 * 33 + 7]
SIZE32 = 13
LR, BETAS, EPS, WD, CLIP = 1e-2, (0.9, 0.999), 1e-8, 0.01, 0.5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_values():
    g = torch.Generator().manual_seed(7)
    p16 = [(torch.randn(n, generator=g) * 0.1).to(torch.bfloat16) for n in SIZES16]
    p32 = torch.randn(SIZE32, generator=g) * 0.1
    return p16, p32


def _local_grad_coef(rank, step):
    g = torch.Generator().manual_seed(1000 + 31 * rank + step)
    c16 = [torch.randn(n, generator=g).to(torch.bfloat16) for n in SIZES16]
    c32 = torch.randn(SIZE32, generator=g)
    return c16, c32


def _build(world, bucket_bytes):
    from rag_tl_domainllm_optimizer_amd import ops
    from rag_tl_domainllm_optimizer_amd.parallel.zero import ZeroAdamW

    p16, p32 = _init_values()
    ps = [torch.nn.Parameter(t.clone()) for t in p16] + [torch.nn.Parameter(p32.clone())]
    flat = ops.flat_params(ps, align=16 * world, keep_master=False)
    opt = ZeroAdamW(flat, lr=LR, betas=BETAS, eps=EPS, weight_decay=WD, max_grad_norm=CLIP,
                    bucket_bytes=bucket_bytes)
    return ps, flat, opt


def _train_step(ps, opt, rank, step):
    c16, c32 = _local_grad_coef(rank, step)
    opt.zero_grad()
    opt.sync.start()
    loss = sum((p * c).sum() for p, c in zip(ps[:-1], c16)) + (ps[-1] * c32).sum()
    loss.backward()
    opt.sync.finish()
    opt.step()


def _worker(rank, world, port, out_dir, bucket_bytes, ckpt):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from rag_tl_domainllm_optimizer_amd import parallel

    parallel.init(device="cpu")
    ps, flat, opt = _build(world, bucket_bytes)
    assert len(opt.buckets) >= (2 if bucket_bytes < 1 << 16 else 1)
    for step in range(2):
        _train_step(ps, opt, rank, step)
    out = {"w16": [p.detach().clone() for p in ps[:-1]], "w32": ps[-1].detach().clone(),
           "norm": float(opt.last_norm), "bytes": opt.state_bytes(), "scratch": opt._scratch_pshard()}
    if ckpt:
        # sharded checkpoint round trip: a fresh optimizer resumes the third step bitwise
        d = os.path.join(out_dir, "ck")
        os.makedirs(d, exist_ok=True)
        opt.save_shard(d)
        meta = opt.state_dict()
        _train_step(ps, opt, rank, 2)
        out["w16_3"] = [p.detach().clone() for p in ps[:-1]]
        ps2, flat2, opt2 = _build(world, bucket_bytes)
        opt2.load_state_dict({**meta, "skipped": int(meta["skipped"])})
        opt2.load_shard(d)
        _train_step(ps2, opt2, rank, 2)
        out["w16_3_resumed"] = [p.detach().clone() for p in ps2[:-1]]
    torch.save(out, os.path.join(out_dir, f"z{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


def _reference(world, steps=2):
    """One process: fp32 master, AdamW on the fp32 mean of the ranks' bf16 local gradients."""
    p16, p32 = _init_values()
    master = [t.float() for t in p16] + [p32.clone()]
    m = [torch.zeros_like(t) for t in master]
    v = [torch.zeros_like(t) for t in master]
    norm = 0.0
    for step in range(steps):
        gs = None
        for r in range(world):
            c16, c32 = _local_grad_coef(r, step)
            loc = [c.float() for c in c16] + [c32]  # d(loss)/dp in bf16 == the bf16 coefficients
            gs = loc if gs is None else [a + b for a, b in zip(gs, loc)]
        gs = [g / world for g in gs]
        norm = float(torch.sqrt(sum(g.double().pow(2).sum() for g in gs)))
        clip = min(1.0, CLIP / (norm + 1e-6))
        t = step + 1
        for p, g, mm, vv in zip(master, gs, m, v):
            gr = g * clip
            mm.mul_(BETAS[0]).add_(gr, alpha=1 - BETAS[0])
            vv.mul_(BETAS[1]).addcmul_(gr, gr, value=1 - BETAS[1])
            p.mul_(1 - LR * WD)
            p.addcdiv_(mm, (vv / (1 - BETAS[1] ** t)).sqrt().add_(EPS), value=-LR / (1 - BETAS[0] ** t))
        # the compute copies the next forward sees are bf16(master); gradients here do not depend on them
    return master, norm


@pytest.mark.parametrize("world,bucket_bytes", [(2, 1 << 12), (4, 1 << 12), (8, 1 << 30)])
def test_zero_step_equals_unsharded(tmp_path, world, bucket_bytes):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), bucket_bytes, world == 4), nprocs=world,
                       start_method="spawn", join=True)
    outs = [torch.load(tmp_path / f"z{r}.pt") for r in range(world)]
    master, norm = _reference(world)
    for o in outs:
        for got, want in zip(o["w16"], master[:-1]):
            # bf16(master): equal up to one bf16 rounding of an fp32 master that differs in the last
            # bits (fp32 sums of the ranks' gradients in another order)
            torch.testing.assert_close(got.float(), want.to(torch.bfloat16).float(), rtol=2 ** -7, atol=1e-6)
            assert (got.float() != want.to(torch.bfloat16).float()).float().mean() < 0.01
        torch.testing.assert_close(o["w32"], master[-1], rtol=1e-5, atol=1e-6)
        assert abs(o["norm"] - norm) <= 1e-5 * norm
        # every rank holds the same compute copy
        for a, b in zip(o["w16"], outs[0]["w16"]):
            assert torch.equal(a, b)
    # the update shard lives in gradient scratch from world 3 on
    assert outs[0]["scratch"] == (world >= 3)
    if world == 4:
        for o in outs:
            for a, b in zip(o["w16_3"], o["w16_3_resumed"]):
                assert torch.equal(a, b)


def test_zero_state_bytes_mistral7b_world8():
    """Per-rank training state of Mistral-7B full fine-tuning at world 8: bf16 weights + bf16
    gradients + 1/8 of (fp32 master + two fp32 moments) — the gradient and update shards live
    inside the gradient buffer."""
    from rag_tl_domainllm_optimizer_amd.parallel.zero import per_rank_state_bytes

    n = 7_241_732_096  # Mistral-7B parameter count
    b8 = per_rank_state_bytes(n, 4097, 8)
    assert b8 <= 40e9, b8
    assert per_rank_state_bytes(n, 4097, 1) == pytest.approx(16 * n, rel=1e-3)  # replicated AdamW state
