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


# the reference's comparison columns (rl.py:446-453), in its order
REF_MODEL_NAMES = ("Base Model", "RAG Model", "RL-finetuned Model", "Transfer-learned Model")


def is_adapter_dir(path: str) -> bool:
    return os.path.isfile(os.path.join(path, "adapter_config.json"))


def _adapter_view(policy, path: Optional[str]):
    """``prepare`` hook: the shared base policy with the PEFT adapter at ``path`` loaded and enabled,
    or with its adapters disabled (the base model) when ``path`` is None."""
    from .models import load_adapter

    def prepare():
        if path is None:
            if hasattr(policy, "set_lora_enabled"):
                policy.set_lora_enabled(False)
            return
        load_adapter(policy, path)
        policy.set_lora_enabled(True)
    return prepare


def _held_out_records(cfg, st, n: int):
    """Evaluation queries with their retrieved documents, none of which occurs in the training
    sample of ``_records`` (the synthetic fact set is finite: a second seed alone can repeat
    training queries). With a configured training file the items come from that file and are NOT
    held out; that is printed."""
    if n <= 0:
        return []
    if cfg.data.train_path:
        print(f"[eval] data.train_path is set: evaluating on items of {cfg.data.train_path} (not held out)")
        return _records(cfg, st, n)[:n]
    corpus, index, enc = st["corpus"], st["index"], st["encoder"]
    train = {it.query for it in corpus.sample_queries(cfg.data.n_queries, seed=cfg.model.seed + 11)}
    items, seen = [], set()
    for it in corpus.sample_queries(max(8 * n, 64), seed=cfg.model.seed + 1013):
        if it.query not in train and it.query not in seen:
            seen.add(it.query)
            items.append(it)
            if len(items) == n:
                break
    if not items:
        raise RuntimeError("no evaluation query outside the training sample: enlarge the corpus")
    _, ids = index.search(enc.encode([it.query for it in items]), cfg.retrieval.top_k)
    return [{"query": it.query, "retrieved_docs": [st["docs"][i] for i in row if i >= 0],
             "ground_truth": it.ground_truth} for it, row in zip(items, ids.tolist())]


def write_comparison(report, run_dir: str, is_main: bool = True) -> str:
    out = os.path.join(run_dir, "model_comparison_results.csv")
    if is_main:
        os.makedirs(run_dir, exist_ok=True)
        report.to_csv(out)  # rl.py:525
        print("Model Comparison Report:")  # rl.py:521
        print(report)
    return out


def cmd_eval(cfg, args):
    """The reference's ``compare_models`` (rl.py:444-463) from the CLI: "Base Model" (bare query),
    "RAG Model" (base + retrieved documents), then each ``--checkpoint`` — a PEFT adapter directory
    (loaded into the base policy) or a full HF model directory. Checkpoints take the reference's
    remaining names in its argument order (RL-finetuned, then Transfer-learned) unless given as
    ``--checkpoint "Name=path"``."""
    from .eval import Evaluator
    from .models import build_model
    from .rewards import RewardModel

    di = _device()
    st = build_stack(cfg, di.device)
    recs = _held_out_records(cfg, st, min(cfg.data.n_queries, 64))
    ev = Evaluator(RewardModel(st["encoder"], cfg.reward), cfg.eval)
    base, tok = st["policy"], st["tokenizer"]
    models = {"Base Model": (base, tok, {"include_docs": False, "prepare": _adapter_view(base, None)}),
              "RAG Model": (base, tok, {"include_docs": True, "prepare": _adapter_view(base, None)})}
    free_names = list(REF_MODEL_NAMES[2:])
    for spec in args.checkpoint or []:
        name, sep, path = spec.partition("=")
        if not sep:
            name, path = (free_names.pop(0) if free_names else os.path.basename(spec.rstrip("/"))), spec
        elif name in free_names:
            free_names.remove(name)
        if is_adapter_dir(path):
            models[name] = (base, tok, {"include_docs": True, "prepare": _adapter_view(base, path)})
        else:
            models[name] = (build_model(path, device=di.device), tok, {"include_docs": True})
    report = ev.compare_models(models, recs)
    write_comparison(report, os.path.join(cfg.out_dir, cfg.name), di.is_main)
    return report


def compare_pipeline_models(cfg, st, policy, run_dir: str, is_main: bool = True):
    """End of ``cli pipeline``: the reference's model comparison (rl.py:444-463, 491-525) over one
    shared set of base weights — "Base Model" (adapters off, bare query), "RAG Model" (adapters
    off, retrieved documents in the prompt), "RL-finetuned Model" (the PPO ``best_model`` adapter),
    "Transfer-learned Model" (the SFT adapter) — written to model_comparison_results.csv. The
    policy's live adapter values are restored afterwards (the PPO trainer keeps using them)."""
    from .eval import Evaluator
    from .rewards import RewardModel

    n = int(getattr(cfg.eval, "compare_items", 0))
    if n <= 0:
        return None
    recs = _held_out_records(cfg, st, n)
    tok = st["tokenizer"]
    lora = list(policy.lora_parameters()) if hasattr(policy, "lora_parameters") else []
    saved = [p.detach().clone() for p in lora]
    rl_dir = os.path.join(run_dir, "best_model_adapter")
    sft_dir = os.path.join(run_dir, "sft_adapter")
    if not lora:  # full fine-tuning: the base weights themselves were trained; only the result is left
        report = Evaluator(RewardModel(st["encoder"], cfg.reward), cfg.eval).compare_models(
            {"RL-finetuned Model": (policy, tok, {"include_docs": True})}, recs)
        write_comparison(report, run_dir, is_main)
        return report
    models = {"Base Model": (policy, tok, {"include_docs": False, "prepare": _adapter_view(policy, None)}),
              "RAG Model": (policy, tok, {"include_docs": True, "prepare": _adapter_view(policy, None)})}
    if is_adapter_dir(rl_dir):
        models["RL-finetuned Model"] = (policy, tok, {"include_docs": True, "prepare": _adapter_view(policy, rl_dir)})
    if is_adapter_dir(sft_dir):
        models["Transfer-learned Model"] = (policy, tok, {"include_docs": True,
                                                          "prepare": _adapter_view(policy, sft_dir)})
    ev = Evaluator(RewardModel(st["encoder"], cfg.reward), cfg.eval)
    try:
        report = ev.compare_models(models, recs)
    finally:
        with torch.no_grad():
            for p, v in zip(lora, saved):
                p.copy_(v)
        if hasattr(policy, "set_lora_enabled"):
            policy.set_lora_enabled(True)
        if lora and hasattr(policy, "refresh_lora"):
            policy.refresh_lora()
    write_comparison(report, run_dir, is_main)
    return report


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
    tr.close()  # the SFT GradSync's post-accumulate hooks on the LoRA parameters go with it
    del tr
    if cfg.sft.full_finetune:
        mio.load_hf_state_dict(policy, mio.read_state_dict(os.path.join(run_dir, "sft_policy")))
        policy.requires_grad_(False)
    else:
        load_adapter(policy, os.path.join(run_dir, "sft_adapter"))
    if policy.embed.is_cuda:
        torch.cuda.empty_cache()
    ppo = cmd_ppo(cfg, args, policy=policy, stack=st)
    from . import parallel

    compare_pipeline_models(cfg, st, policy, run_dir, parallel.info().is_main)
    return ppo


def cmd_serve(cfg, args):
    from .serve import serve

    serve(cfg, host=args.host, port=args.port)


def cmd_bench(cfg, args, rest):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *rest])
    sys.exit(r.returncode)


def cmd_launch(args, rest):
    from .parallel.launch import launch_env, torchrun_cmd

    cmd = torchrun_cmd(args.nproc, ["-m", "rag_tl_domainllm_optimizer_amd", *rest], args.port)
    # the caller's environment (NCCL_* / RCCL_* / HSA_* tuning) passes through to every rank;
    # --env KEY=VALUE adds or overrides entries (e.g. --env NCCL_MIN_NCHANNELS=32)
    try:
        env = launch_env(args.env or [])
    except ValueError as e:
        raise SystemExit(f"launch: {e}")
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
