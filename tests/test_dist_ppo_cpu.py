"""Data-parallel PPO and SFT on CPU with gloo (SURVEY §4.2 distributed layer).

PPO (world 2 and 8): the bucketed all-reduce of a real ``PPOTrainer.step`` averages the ranks'
local gradients; after the step every rank holds bitwise-identical LoRA and value-head parameters;
``reduce_metrics`` gives every rank the same dict (durations max-reduced); a rank-0 checkpoint
(+ per-rank RNG files) resumed on all ranks reproduces the uninterrupted next step.
SFT: an example count that is not a multiple of the world size runs the same number of steps on
every rank (regression test for the shard-imbalance deadlock).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _ppo_setup(seed=0):
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.data import SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    torch.manual_seed(seed)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    policy = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    enc_cfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(enc_cfg, dtype=torch.float32, seed=2).eval(),
                  Tokenizer.synthetic(enc_cfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
    items = corpus.sample_queries(64, seed=4)
    recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
            for it in items]
    pc = PPOConfig(max_new_tokens=6, max_prompt_tokens=64, minibatch_size=4, lora_r=4, lora_alpha=8.0, lr=1e-3,
                   bucket_mb=1e-3)  # tiny buckets: several all-reduces per backward
    return PPOTrainer(policy, tok, RewardModel(enc), pc, max_batch=8), recs


def _ppo_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rag_tl_domainllm_optimizer_amd import parallel
    from rag_tl_domainllm_optimizer_amd.data import RecordLoader

    parallel.init(device="cpu")
    tr, recs = _ppo_setup()
    assert len(tr.sync.buckets) >= 2
    batches = list(RecordLoader(recs, 4, seed=0, rank=rank, world=world))
    # step 1 with the gradient hand-off instrumented: hooks off -> local gradients only, then
    # finish() all-reduces every bucket; keep both
    tr.sync.sync_enabled = False
    real_finish = tr.sync.finish
    captured = []

    def finish():
        captured.append(tr.flat.grad.clone())
        real_finish()
        captured.append(tr.flat.grad.clone())
    tr.sync.finish = finish
    m1 = tr.step(batches[0])
    tr.sync.finish = real_finish
    tr.sync.sync_enabled = True
    ck = os.path.join(out_dir, "ck", "s1")
    tr.save_checkpoint(ck, 0, m1["reward_mean"], full_policy=False, batch_in_epoch=1)
    m2 = tr.step(batches[1])  # normal overlapped hooks
    params = torch.cat([p.detach().reshape(-1) for p in tr.flat.params])
    # resume on every rank from the rank-0 checkpoint + this rank's RNG, replay step 2
    tr2, _ = _ppo_setup()
    st = tr2.load_checkpoint(ck)
    m2b = tr2.step(batches[1])
    params_b = torch.cat([p.detach().reshape(-1) for p in tr2.flat.params])
    torch.save({"local": captured[0], "reduced": captured[1], "m1": m1, "m2": m2, "m2b": m2b, "params": params,
                "params_b": params_b, "batch_in_epoch": st.get("batch_in_epoch")},
               os.path.join(out_dir, f"ppo{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


@pytest.mark.parametrize("world", [2, 8])
def test_dp_ppo_step(tmp_path, world):
    mp.start_processes(_ppo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    r = [torch.load(tmp_path / f"ppo{i}.pt", weights_only=False) for i in range(world)]
    # the all-reduce averages the ranks' local gradients, and every rank ends with the same average
    mean_local = torch.stack([x["local"] for x in r]).mean(0)
    assert mean_local.abs().sum() > 0
    for x in r:
        torch.testing.assert_close(x["reduced"], mean_local, rtol=1e-5, atol=1e-7)
    # identical parameters on every rank after two optimizer steps
    for x in r[1:]:
        assert torch.equal(x["params"], r[0]["params"])
    # reduced metrics are the same dict on every rank; throughput uses the slowest rank's time
    for k in ("reward_mean", "total_loss", "kl_ref", "step_time_s", "rollout_tokens_per_s"):
        assert all(x["m2"][k] == r[0]["m2"][k] for x in r), k
    assert r[0]["m2"]["rollout_tokens_per_s"] == pytest.approx(
        r[0]["m2"]["rollout_tokens"] * world / r[0]["m2"]["step_time_s"])
    # rank-0 checkpoint resumed on all ranks reproduces the uninterrupted step 2 exactly
    for x in r:
        assert x["batch_in_epoch"] == 1
        torch.testing.assert_close(x["params_b"], x["params"], rtol=1e-6, atol=1e-7)
        assert abs(x["m2b"]["total_loss"] - x["m2"]["total_loss"]) < 1e-5


def _sft_worker(rank, world, port, out_dir, n_examples):
    _env(rank, world, port)
    from rag_tl_domainllm_optimizer_amd import models, parallel
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.sft import SFTConfig, SFTTrainer

    parallel.init(device="cpu", timeout_s=120)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    m = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    tr = SFTTrainer(m, tok, SFTConfig(lr=1e-2, lora_r=4, lr_schedule="constant", warmup_steps=0, batch_size=4))
    words = tok.words()
    ex = [{"prompt": " ".join(words[i:i + 6]), "answer": " ".join(words[50 + i:54 + i])} for i in range(n_examples)]
    hist = tr.fit(ex, epochs=2, log_every=0)
    params = torch.cat([p.detach().reshape(-1) for p in tr.flat.params])
    torch.save({"steps": len(hist), "params": params}, os.path.join(out_dir, f"sft{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


@pytest.mark.parametrize("world,n", [(2, 15), (8, 13)])
def test_dp_sft_uneven_shards(tmp_path, world, n):
    mp.start_processes(_sft_worker, args=(world, _free_port(), str(tmp_path), n), nprocs=world, start_method="spawn",
                       join=True)
    r = [torch.load(tmp_path / f"sft{i}.pt", weights_only=False) for i in range(world)]
    assert len({x["steps"] for x in r}) == 1 and r[0]["steps"] >= 2
    for x in r[1:]:
        assert torch.equal(x["params"], r[0]["params"])


def _sft_resume_worker(rank, world, port, out_dir, mode):
    _env(rank, world, port)
    from rag_tl_domainllm_optimizer_amd import models, parallel
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.sft import SFTConfig, SFTTrainer
    from rag_tl_domainllm_optimizer_amd.utils.faults import InjectedFault

    parallel.init(device="cpu", timeout_s=120)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    words = tok.words()
    ex = [{"prompt": " ".join(words[i:i + 6]), "answer": " ".join(words[50 + i:54 + i])} for i in range(24)]

    def trainer():
        m = models.CausalLM(cfg, dtype=torch.float32, seed=1)
        return SFTTrainer(m, tok, SFTConfig(lr=1e-2, lora_r=4, lr_schedule="cosine", warmup_steps=1, total_steps=6,
                                            batch_size=4))
    ck = os.path.join(out_dir, f"ck_{mode}")
    tr = trainer()
    if mode == "crash":
        os.environ["RAGTL_FAULT_AT_STEP"] = "5"
        try:
            tr.fit(ex, epochs=2, log_every=0, ckpt_dir=ck, save_every=2)
            raise AssertionError("fault not injected")
        except InjectedFault:
            pass
        del os.environ["RAGTL_FAULT_AT_STEP"]
        parallel.barrier()
        tr = trainer()  # a fresh process' state: new model, new optimizer
        tr.fit(ex, epochs=2, log_every=0, ckpt_dir=ck, save_every=2, resume=True)
    else:
        tr.fit(ex, epochs=2, log_every=0, ckpt_dir=ck, save_every=2)
    params = torch.cat([p.detach().reshape(-1) for p in tr.flat.params])
    torch.save({"params": params, "step": tr.global_step, "m": tr.opt.state_dict()["exp_avg"].clone()},
               os.path.join(out_dir, f"sftr_{mode}{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


def test_dp_sft_resume_mid_epoch_matches_uninterrupted(tmp_path):
    """gloo world 2: an SFT run killed at step 5 (mid epoch 2) and resumed from its mid-epoch
    "latest" checkpoint (adapter, optimizer moments, LR-schedule position, each rank's RNG and
    place in the epoch) ends with exactly the parameters of the uninterrupted run."""
    world = 2
    for mode in ("full", "crash"):
        mp.start_processes(_sft_resume_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world,
                           start_method="spawn", join=True)
    for r in range(world):
        a = torch.load(tmp_path / f"sftr_full{r}.pt", weights_only=False)
        b = torch.load(tmp_path / f"sftr_crash{r}.pt", weights_only=False)
        assert a["step"] == b["step"] == 6
        assert torch.equal(a["params"], b["params"])
        assert torch.equal(a["m"], b["m"])
    assert (tmp_path / "ck_crash" / "latest_trainer_state").is_dir()


def _cli_pipeline_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rag_tl_domainllm_optimizer_amd import cli, parallel

    args = ["pipeline", "--model.policy=tiny-llama:random", "--model.encoder=tiny-bert:random",
            "--data.synthetic_docs=64", "--data.doc_words=16", "--retrieval.index=flat", f"--out_dir={out_dir}",
            "--data.n_queries=16", "--data.batch_size=4", "--ppo.max_new_tokens=6", "--ppo.max_prompt_tokens=96",
            "--ppo.minibatch_size=2", "--sft.batch_size=2", "--sft.lora_r=4", "--ppo.lora_r=4"]
    tr = cli.main(args)
    # post-accumulate-grad hooks per trainable parameter: PPO's GradSync only (the SFT trainer's
    # were removed when the policy was handed over)
    nhooks = [len(getattr(p, "_post_accumulate_grad_hooks", None) or {}) for p in tr.flat.params]
    torch.save({"params": torch.cat([p.detach().reshape(-1) for p in tr.flat.params]), "step": tr.global_step,
                "hooks": nhooks}, os.path.join(out_dir, f"pipe{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


def test_dp_cli_pipeline_world2(tmp_path):
    """Config 5 (`cli pipeline`: index -> RAFT LoRA SFT -> adapter on disk -> PPO) at world 2: the
    SFT adapter rank 0 writes is what both ranks reload, both ranks run the same number of PPO steps
    and end with identical trainable parameters, and the run directory holds every stage's output."""
    world = 2
    mp.start_processes(_cli_pipeline_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    r = [torch.load(tmp_path / f"pipe{i}.pt", weights_only=True) for i in range(world)]
    assert r[0]["step"] == r[1]["step"] > 0
    assert torch.equal(r[0]["params"], r[1]["params"])
    assert all(set(x["hooks"]) == {1} for x in r), [x["hooks"] for x in r]
    run = tmp_path / "run"
    assert os.path.isdir(run / "sft_adapter") and os.path.isdir(run / "best_model_adapter")
    assert os.path.exists(run / "metrics.jsonl")


def _zero_ppo_worker(rank, world, port, out_dir, zero):
    _env(rank, world, port)
    from rag_tl_domainllm_optimizer_amd import models, parallel
    from rag_tl_domainllm_optimizer_amd.data import RecordLoader, SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    parallel.init(device="cpu")

    def setup(zero=zero):
        torch.manual_seed(0)
        cfg = PRESETS["tiny-llama"]
        tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
        policy = models.CausalLM(cfg, dtype=torch.bfloat16, seed=1)
        ecfg = PRESETS["tiny-bert"]
        enc = Encoder(models.SentenceEncoder(ecfg, dtype=torch.float32, seed=2).eval(),
                      Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
        corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
        recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
                for it in corpus.sample_queries(32, seed=4)]
        pc = PPOConfig(full_finetune=True, zero=zero, max_new_tokens=6, max_prompt_tokens=64, minibatch_size=4,
                       lr=1e-3, bucket_mb=2e-3)
        return PPOTrainer(policy, tok, RewardModel(enc), pc, max_batch=8), recs

    tr, recs = setup()
    assert bool(getattr(tr.opt, "sharded", False)) == zero
    batches = list(RecordLoader(recs, 4, seed=0, rank=rank, world=world))
    m1 = tr.step(batches[0])
    ck = os.path.join(out_dir, f"ck{int(zero)}", "s1")
    tr.save_checkpoint(ck, 0, m1["reward_mean"], full_policy=True, batch_in_epoch=1)
    d = ck + "_trainer_state"
    files = os.listdir(d)
    assert not os.path.exists(d + ".tmp")
    assert all(f"rng_rank{r}.safetensors" in files for r in range(world)), files
    if zero:
        # every rank's shard is inside the committed directory (written before the rename)
        assert all(f"optimizer_zero{world}_rank{r}.safetensors" in files for r in range(world)), files
    m2 = tr.step(batches[1])
    params = torch.cat([p.detach().float().reshape(-1) for p in tr.policy.parameters()])
    tr2, _ = setup()
    tr2.load_checkpoint(ck)
    m2b = tr2.step(batches[1])
    params_b = torch.cat([p.detach().float().reshape(-1) for p in tr2.policy.parameters()])
    if zero:
        # an unsharded optimizer refuses the sharded state instead of silently resuming without it
        tr_rep, _ = setup(zero=False)
        with pytest.raises(RuntimeError, match="ZeRO-1 sharded"):
            tr_rep.load_checkpoint(ck)
    torch.save({"m1": m1, "m2": m2, "m2b": m2b, "params": params, "params_b": params_b},
               os.path.join(out_dir, f"zppo{int(zero)}_{rank}.pt"))
    parallel.barrier()
    parallel.shutdown()


def test_dp_ppo_full_finetune_zero_world2(tmp_path):
    """Full-parameter PPO at world 2 with ZeRO-1 (fp32 reduce-scatter, sharded fp32 master and
    moments, bf16 all-gather): every rank ends with the same bf16 weights; the step tracks the
    replicated optimizer (which rounds the reduced gradient to bf16 once) to bf16 tolerance; a
    checkpoint (rank-0 policy + per-rank optimizer shards) resumes the next step exactly."""
    world = 2
    for zero in (True, False):
        mp.start_processes(_zero_ppo_worker, args=(world, _free_port(), str(tmp_path), zero), nprocs=world,
                           start_method="spawn", join=True)
    z = [torch.load(tmp_path / f"zppo1_{i}.pt", weights_only=False) for i in range(world)]
    rep = [torch.load(tmp_path / f"zppo0_{i}.pt", weights_only=False) for i in range(world)]
    assert torch.equal(z[0]["params"], z[1]["params"])
    d = (z[0]["params"] - rep[0]["params"]).abs()
    # the two optimizers see the same mean gradient up to one bf16 rounding: a few bf16 ulps apart
    assert float(d.max()) < 0.05 and float((d > 0).float().mean()) < 0.2
    assert z[0]["m1"]["grad_norm"] == pytest.approx(rep[0]["m1"]["grad_norm"], rel=1e-2)
    for x in z:
        assert torch.equal(x["params_b"], x["params"])
        assert abs(x["m2b"]["total_loss"] - x["m2"]["total_loss"]) < 1e-6
