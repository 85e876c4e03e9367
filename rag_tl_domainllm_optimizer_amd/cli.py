"""Command line: ``python -m rag_tl_domainllm_optimizer_amd <command> [--config f.yaml] [--preset p]
[--section.key=value ...]``.

Commands: index | rag | sft | ppo | eval | pipeline | serve | bench | launch.
Multi-GPU: ``python -m rag_tl_domainllm_optimizer_amd launch --nproc 8 ppo ...`` starts one process
per GPU through torch.distributed.run (RCCL over xGMI) as a child process.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from typing import List, Optional

import torch

from . import config as C


def _device():
    from . import parallel

    di = parallel.init()
    return di


def build_stack(cfg: C.RunConfig, device, need_policy=True, need_index=True):
    """Tokenizer, policy, encoder, documents, index according to the config."""
    from .data import SyntheticCorpus
    from .models import build_model
    from .retrieval import Encoder, FlatIndex, IVFIndex, chunk_documents, load_index
    from .retrieval.chunking import read_text_file
    from .tokenizer import load_tokenizer

    dtype = getattr(torch, cfg.model.dtype) if device.type == "cuda" else torch.float32
    out = {}
    policy = build_model(cfg.model.policy, device=device, dtype=dtype, seed=cfg.model.seed,
                         fast_init=device.type == "cuda") if need_policy else None
    pcfg = policy.cfg if policy is not None else None
    from .models import resolve_preset

    if pcfg is None:
        pcfg = resolve_preset(cfg.model.policy)
    tok = load_tokenizer(cfg.model.policy, pcfg.vocab_size if pcfg else None, pcfg.arch if pcfg else "llama")
    enc_model = build_model(cfg.model.encoder, device=device, dtype=dtype, seed=cfg.model.seed + 1,
                            fast_init=device.type == "cuda").eval()
    enc_tok = load_tokenizer(cfg.model.encoder, enc_model.cfg.vocab_size, enc_model.cfg.arch)
    encoder = Encoder(enc_model, enc_tok)
    corpus = None
    if cfg.data.docs_path:
        p = cfg.data.docs_path
        raw = [read_text_file(os.path.join(p, f)) for f in sorted(os.listdir(p))] if os.path.isdir(p) else \
            [l.strip() for l in open(p) if l.strip()]
        docs, _ = chunk_documents(raw, cfg.retrieval.chunk_words, cfg.retrieval.chunk_overlap)
    else:
        corpus = SyntheticCorpus(tok.words(), n_docs=cfg.data.synthetic_docs, doc_words=cfg.data.doc_words,
                                 seed=cfg.model.seed + 7)
        docs = corpus.docs
    index = None
    if need_index:
        if cfg.retrieval.index_path and os.path.exists(os.path.join(cfg.retrieval.index_path, "index.json")):
            index = load_index(cfg.retrieval.index_path, device)
        else:
            emb = encoder.encode(docs)
            if cfg.retrieval.index == "flat":
                index = FlatIndex(encoder.dim, cfg.retrieval.metric, device)
            else:
                index = IVFIndex(encoder.dim, min(cfg.retrieval.nlist, max(1, len(docs) // 8)), cfg.retrieval.metric,
                                 device, cfg.retrieval.nprobe)
                index.train(emb)
            index.add(emb)
            if cfg.retrieval.index_path:
                index.save(cfg.retrieval.index_path)
    out.update(policy=policy, tokenizer=tok, encoder=encoder, docs=docs, corpus=corpus, index=index)
    return out


def _records(cfg: C.RunConfig, stack, n: int):
    from .data import load_records

    if cfg.data.train_path:
        return load_records(cfg.data.train_path)
    corpus, index, enc = stack["corpus"], stack["index"], stack["encoder"]
    items = corpus.sample_queries(n, seed=cfg.model.seed + 11)
    qs = [it.query for it in items]
    recs = []
    for s in range(0, len(qs), 256):
        _, ids = index.search(enc.encode(qs[s:s + 256]), cfg.retrieval.top_k)
        for it, row in zip(items[s:s + 256], ids.tolist()):
            recs.append({"query": it.query, "retrieved_docs": [stack["docs"][i] for i in row if i >= 0],
                         "ground_truth": it.ground_truth, "gold_doc": it.gold_doc})
    return recs


def cmd_index(cfg, args):
    di = _device()
    st = build_stack(cfg, di.device, need_policy=False)
    path = cfg.retrieval.index_path or os.path.join(cfg.out_dir, cfg.name, "index")
    st["index"].save(path)
    print(json.dumps({"index": path, "ntotal": st["index"].ntotal, "kind": st["index"].kind}))


def latest_checkpoint(run_dir: str, kind: str = "ppo"):
    """Prefix of the ``kind`` ("ppo" / "sft") checkpoint with the highest global step in
    ``run_dir`` (or None). States written before the kind field existed count as PPO."""
    if not os.path.isdir(run_dir):
        return None
    cands = []
    for d in os.listdir(run_dir):
        sf = os.path.join(run_dir, d, "state.json")
        if d.endswith("_trainer_state") and os.path.exists(sf):
            with open(sf) as f:
                st = json.load(f)
            if st.get("kind", "ppo") != kind:
                continue
            cands.append((int(st.get("global_step", 0)), os.path.join(run_dir, d[:-len("_trainer_state")])))
    return max(cands)[1] if cands else None


def _apply_fp8(cfg, policy):
    """config 5: fp8 e4m3fn weight images for the no-grad forwards (``model.fp8``)."""
    if policy is not None and getattr(cfg.model, "fp8", False) and hasattr(policy, "set_fp8"):
        if next(policy.parameters()).is_cuda:
            policy.set_fp8(True, train=getattr(cfg.model, "fp8_train", False))
    if policy is not None and getattr(cfg.model, "fp8_kv", False) and hasattr(policy, "kv_fp8"):
        if next(policy.parameters()).is_cuda:
            policy.kv_fp8 = True  # generators built on the policy keep an e4m3fn K/V cache
    return policy


def cmd_rag(cfg, args):
    from .generation import SamplingParams
    from .rag import RagPipeline

    di = _device()
    st = build_stack(cfg, di.device)
    _apply_fp8(cfg, st["policy"])
    sp = SamplingParams(max_new_tokens=cfg.ppo.max_new_tokens, temperature=cfg.eval.temperature,
                        do_sample=cfg.eval.do_sample, top_k=cfg.eval.top_k)
    rag = RagPipeline(st["encoder"], st["index"], st["docs"], st["policy"], st["tokenizer"], cfg.retrieval.top_k, sp,
                      cfg.ppo.max_prompt_tokens)
    queries = args.query or [it.query for it in st["corpus"].sample_queries(4)] if st["corpus"] else args.query
    for a in rag.answer(queries):
        print(json.dumps({"query": a.query, "answer": a.answer, "doc_ids": a.doc_ids, "timings": a.timings}))


def cmd_sft(cfg, args, stack=None):
    from .train import SFTTrainer, build_raft_examples
    from .utils import MetricsSink

    di = _device()
    st = stack or build_stack(cfg, di.device)
    recs = _records(cfg, st, cfg.data.n_queries)
    items = [r for r in recs if "gold_doc" in r] or recs
    examples = build_raft_examples(items, st["docs"], cfg.raft) if "gold_doc" in items[0] else \
        [{"prompt": __import__("rag_tl_domainllm_optimizer_amd.rag", fromlist=["build_prompt"]).build_prompt(
            r["query"], r["retrieved_docs"]), "answer": r["ground_truth"] or ""} for r in recs]
    run_dir = os.path.join(cfg.out_dir, cfg.name)
    sink = MetricsSink(run_dir if di.is_main else None, config=C.to_dict(cfg), use_wandb=cfg.use_wandb)
    tr = SFTTrainer(st["policy"], st["tokenizer"], cfg.sft, sink)
    if getattr(cfg.model, "fp8_train", False):
        _apply_fp8(cfg, st["policy"])  # config 5: frozen-base SFT forwards on W8A8 too
    # best / per-epoch / mid-epoch checkpoints (rl.py:357-363) in their own directory; --resume
    # continues from the most advanced of them
    hist = tr.fit(examples, epochs=cfg.data.epochs, ckpt_dir=os.path.join(run_dir, "sft_ckpt"),
                  save_every=cfg.sft.save_every, resume=bool(getattr(args, "resume", False)))
    tr.save(os.path.join(run_dir, "sft"), full_policy=getattr(cfg.sft, "save_full_policy", True),
            epoch=cfg.data.epochs)
    if di.is_main:
        print(json.dumps({"final_loss": hist[-1]["loss"] if hist else None, "steps": tr.global_step}))
    return tr, st


def cmd_ppo(cfg, args, policy=None, stack=None):
    from .data import RecordLoader
    from .rewards import RewardModel
    from .train import PPOTrainer
    from .utils import MetricsSink

    di = _device()
    st = stack or build_stack(cfg, di.device, need_policy=policy is None)
    if policy is not None:
        st["policy"] = policy
    _apply_fp8(cfg, st["policy"])
    recs = _records(cfg, st, cfg.data.n_queries)
    run_dir = os.path.join(cfg.out_dir, cfg.name)
    sink = MetricsSink(run_dir if di.is_main else None, config=C.to_dict(cfg), use_wandb=cfg.use_wandb)
    tr = PPOTrainer(st["policy"], st["tokenizer"], RewardModel(st["encoder"], cfg.reward), cfg.ppo, sink=sink,
                    max_batch=cfg.data.batch_size)
    loader = RecordLoader(recs, cfg.data.batch_size, seed=cfg.model.seed, rank=di.rank, world=di.world)
    best = -float("inf")
    first, start_batch, rewards = 0, 0, []
    if getattr(args, "resume", False):
        # resume from the run's most advanced checkpoint (epoch end or mid-epoch "latest"): model,
        # optimizer, every rank's RNG, the sampler's device RNG counter and the loader position
        prefix = latest_checkpoint(run_dir)
        if prefix is not None:
            st_ = tr.load_checkpoint(prefix)
            first, start_batch = int(st_.get("epoch", 0)), int(st_.get("batch_in_epoch", 0))
            best = float(st_.get("best_reward", best))
            rewards = list(st_.get("epoch_rewards", []))
            if di.is_main:
                print(f"Resumed from {prefix} (epoch {first}, batch {start_batch})")
    for ep in range(first, cfg.data.epochs):
        loader.set_epoch(ep, start_batch if ep == first else 0)
        if ep != first:
            rewards = []
        b = start_batch if ep == first else 0
        for batch in loader:
            m = tr.step(batch)
            rewards.append(m["reward_mean"])
            b += 1
            if di.is_main:
                print(json.dumps({k: m[k] for k in ("reward_mean", "total_loss", "kl_ref", "rollout_tokens_per_s")}),
                      flush=True)
            if cfg.ppo.save_every and tr.global_step % cfg.ppo.save_every == 0 and b < len(loader):
                tr.save_checkpoint(os.path.join(run_dir, "latest"), ep, best, full_policy=False, batch_in_epoch=b,
                                   extra_state={"epoch_rewards": rewards})
        avg = sum(rewards) / max(len(rewards), 1)
        if di.is_main:
            print(f"Epoch {ep + 1}/{cfg.data.epochs}: Average Reward = {avg:.4f}")
        full = cfg.ppo.save_full_policy
        if avg > best:  # rl.py:358-360
            best = avg
            tr.save_checkpoint(os.path.join(run_dir, "best_model"), ep + 1, best, full_policy=full)
        tr.save_checkpoint(os.path.join(run_dir, f"epoch_{ep + 1}"), ep + 1, best, full_policy=full)
    return tr


def cmd_eval(cfg, args):
    from .eval import Evaluator
    from .models import build_model
    from .rewards import RewardModel

    di = _device()
    st = build_stack(cfg, di.device)
    recs = _records(cfg, st, min(cfg.data.n_queries, 64))
    ev = Evaluator(RewardModel(st["encoder"], cfg.reward), cfg.eval)
    models = {"Base Model": (st["policy"], st["tokenizer"])}
    for p in args.checkpoint or []:
        models[os.path.basename(p.rstrip("/"))] = (build_model(p, device=di.device), st["tokenizer"])
    report = ev.compare_models(models, recs)
    out = os.path.join(cfg.out_dir, cfg.name, "model_comparison_results.csv")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    report.to_csv(out)
    print("Model Comparison Report:")
    print(report)


def cmd_pipeline(cfg, args):
    """Config 5: RAG index -> RAFT LoRA SFT -> PPO on ONE stack (tokenizer, encoder, embeddings and
    index are built once), with the policy handed from SFT to PPO THROUGH the SFT checkpoint on disk
    (as the reference hands stages over by path, rl.py:365-379,494-498): the PEFT adapter is
    re-read into the policy (LoRA), or the saved HF policy weights (``sft.full_finetune``). The SFT
    trainer (optimizer moments, flat buffers) is dropped before PPO builds its own."""
    from .models import io as mio
    from .models import load_adapter

    tr, st = cmd_sft(cfg, args)
    run_dir = os.path.join(cfg.out_dir, cfg.name)
    policy = tr.model
    del tr
    if cfg.sft.full_finetune:
        mio.load_hf_state_dict(policy, mio.read_state_dict(os.path.join(run_dir, "sft_policy")))
        policy.requires_grad_(False)
    else:
        load_adapter(policy, os.path.join(run_dir, "sft_adapter"))
    if policy.embed.is_cuda:
        torch.cuda.empty_cache()
    return cmd_ppo(cfg, args, policy=policy, stack=st)


def cmd_serve(cfg, args):
    from .serve import serve

    serve(cfg, host=args.host, port=args.port)


def cmd_bench(cfg, args, rest):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *rest])
    sys.exit(r.returncode)


def cmd_launch(args, rest):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={args.port}", "-m", "rag_tl_domainllm_optimizer_amd", *rest]
    # the caller's environment (NCCL_* / RCCL_* / HSA_* tuning) passes through to every rank;
    # --env KEY=VALUE adds or overrides entries (e.g. --env NCCL_MIN_NCHANNELS=32)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for kv in args.env or []:
        k, sep, v = kv.partition("=")
        if not sep or not k:
            raise SystemExit(f"launch: --env expects KEY=VALUE, got {kv!r}")
        env[k] = v
    sys.exit(subprocess.run(cmd, env=env).returncode)


def main(argv: Optional[List[str]] = None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="rag_tl_domainllm_optimizer_amd")
    ap.add_argument("command", choices=["index", "rag", "sft", "ppo", "eval", "pipeline", "serve", "bench", "launch"])
    ap.add_argument("--config", default=None)
    ap.add_argument("--preset", default=None, choices=sorted(C.PRESETS))
    ap.add_argument("--query", action="append")
    ap.add_argument("--checkpoint", action="append")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--env", action="append", default=[], help="launch: KEY=VALUE set for every rank (repeatable)")
    ap.add_argument("--resume", action="store_true",
                    help="sft / ppo / pipeline: continue from the run's latest checkpoint")
    if argv and argv[0] == "launch":
        a, rest = ap.parse_known_args(argv)
        return cmd_launch(a, [x for x in rest])
    if argv and argv[0] == "bench":
        return cmd_bench(None, None, argv[1:])
    args, rest = ap.parse_known_args(argv)
    overrides = [r for r in rest if r.startswith("--") and "=" in r]
    cfg = C.load(args.config, args.preset, overrides)
    fn = {"index": cmd_index, "rag": cmd_rag, "sft": cmd_sft, "ppo": cmd_ppo, "eval": cmd_eval,
          "pipeline": cmd_pipeline, "serve": cmd_serve}[args.command]
    return fn(cfg, args)


if __name__ == "__main__":
    main()
