#!/usr/bin/env python3
"""Headline benchmark: PPO rollout tokens/sec (node) + p50 RAG answer latency, Mistral-7B.

Metric and config from BASELINE.json: Mistral-7B-shaped bf16 policy (random init, LoRA r=16 on all
linear projections — or every weight with --full-ft — value head), 256 rollouts per GPU, all-MiniLM-L6-shaped
retrieval encoder, all-mpnet-base-v2-shaped reward encoder (the reference's default), 100k-doc synthetic
corpus in an HBM-resident IVF index. One process per GPU (torchrun env, RCCL over xGMI), data
parallel; per-GPU work is fixed (weak scaling).

One timed step = one full PPO iteration per rank: retrieve top-k docs for the rank's queries ->
RAG prompts -> rollout generation (prefill + hipGraph-replayed decode, sampling) with reward
scoring overlapped on a side stream -> frozen-reference log-probs -> token GAE -> PPO update
(forward + backward + bucketed RCCL all-reduce + fused AdamW) over all minibatches.
value = generated rollout tokens summed over ranks / max-over-ranks wall time of the K timed steps.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W
``python bench.py --gpus N`` with N > 1 and no torchrun environment starts the N ranks itself
(torch.distributed.run as a child process, parallel/launch.py) and exits with their status;
RAGTL_DIST_BACKEND=gloo rehearses N ranks on one GPU.

Secondary modes (not the headline; each prints its own JSON line):
  --mode sft       BASELINE config 3: RAFT-style LoRA r=16 SFT with distractor docs, tokens/s
  --mode pipeline  BASELINE config 5: RAG index -> LoRA SFT -> PPO on one policy (default
                   --model llama2-13b; --fp8 runs rollouts / reference scoring on e4m3fn weights)
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_LATENCY_S = 2.4  # README.md:38 "RL Optimized" latency (best published); RAG baseline 3.1 s


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--encoder", default="minilm-l6", help="retrieval (bi-encoder / IVF index) encoder")
    ap.add_argument("--reward-encoder", default="mpnet-base",
                    help="reward-model sentence encoder (the reference's RewardModel default is all-mpnet-base-v2, "
                         "rl.py:54-55); 'same' reuses the retrieval encoder")
    ap.add_argument("--rollout-batch", type=int, default=256,
                    help="sequences per GPU per PPO step (default 256, also for --mode pipeline: "
                         "profiles/r4/pipeline13b_rollout_batch.log)")
    ap.add_argument("--new-tokens", type=int, default=128)
    ap.add_argument("--max-prompt", type=int, default=320)
    ap.add_argument("--minibatch", type=int, default=32, help="PPO minibatch (sequences per optimizer step)")
    ap.add_argument("--ref-minibatch", type=int, default=None,
                    help="sequences per reference-scoring forward (default: PPOConfig.ref_minibatch_size)")
    ap.add_argument("--top-k-docs", type=int, default=3)
    ap.add_argument("--ndocs", type=int, default=100_000)
    ap.add_argument("--doc-words", type=int, default=48)
    ap.add_argument("--nlist", type=int, default=512)
    ap.add_argument("--nprobe", type=int, default=16)
    ap.add_argument("--latency-queries", type=int, default=16)
    ap.add_argument("--skip-latency", action="store_true")
    ap.add_argument("--latency-contexts", default="",
                    help="long-context RAG answers: comma list of prompt budgets in tokens (e.g. 1024,2048,4096); "
                         "each retrieves enough documents to fill its budget and reports p50 latency + stages")
    ap.add_argument("--vary-docs", action="store_true",
                    help="1..top-k retrieved docs per query (variable prompt lengths: exercises the varlen "
                         "packed forwards; RAGTL_PACK=0 for the padded comparison)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--tuning", default="",
                    help="kernel-selection overrides for A/B runs, e.g. gemm_group_m=8,gemm_bn128_cost=0.6 (ops.set_tuning; "
                         "recorded in the JSON line)")
    ap.add_argument("--rope-fusion", default="on", choices=["on", "off"],
                    help="A/B: RoPE in the qkv GEMM epilogue and in the attention backward stores (on) or the "
                         "separate rotation passes (off)")
    ap.add_argument("--torch-profile", default=None,
                    help="PPO mode: run one extra (untimed) step under torch.profiler after the warm-up and "
                         "write its per-op table, grouped by Python call site, to this path")
    ap.add_argument("--mode", default="ppo", choices=["ppo", "sft", "pipeline", "serve"])
    ap.add_argument("--serve-concurrency", default="1,4,16",
                    help="--mode serve: closed-loop client counts (one engine, max batch = the largest)")
    ap.add_argument("--serve-requests", type=int, default=64, help="--mode serve: answers per concurrency level")
    ap.add_argument("--serve-engine", default="continuous", choices=["continuous", "dynamic"],
                    help="--mode serve: iteration-level (continuous) or request-group (dynamic) batching")
    ap.add_argument("--fp8", action=argparse.BooleanOptionalAction, default=None,
                    help="fp8 (e4m3fn) weights for no-grad forwards (default: on for --mode pipeline, config 5)")
    ap.add_argument("--fp8-kv", action=argparse.BooleanOptionalAction, default=None,
                    help="fp8 (e4m3fn) rollout K/V cache (default: with --fp8)")
    ap.add_argument("--fp8-train", action=argparse.BooleanOptionalAction, default=None,
                    help="W8A8 frozen-base product in LoRA training forwards (default: with --fp8)")
    ap.add_argument("--sft-batch", type=int, default=64, help="SFT sequences per GPU per step")
    ap.add_argument("--full-ft", action="store_true",
                    help="PPO over every policy weight (the reference's full-parameter mode: bf16 compute copies "
                         "+ fp32 master, frozen reference copy) instead of LoRA r=16")
    ap.add_argument("--old-logp", default="rollout", choices=["rollout", "recompute"],
                    help="PPO ratio's theta_old log-probs: the rollout sampler's (free) or a training-numerics "
                         "forward of the policy beside the reference forward (exact ratio 1 at theta_old)")
    ap.add_argument("--lora-grad-epilogue", default="on", choices=["on", "off"],
                    help="A/B: LoRA adapter gradients accumulated into the flat .grad buffer by one native epilogue "
                         "per projection (on) or returned to autograd (off: zero fill + scale + one add per adapter)")
    ap.add_argument("--kl-in-loss", default="on", choices=["on", "off"],
                    help="frozen-reference KL as a k3 penalty on the update forward's own log-probs (on) or as a "
                         "-beta (old - ref) token reward (off: the pre-round-6 form)")
    ap.add_argument("--defer-splitk", default="on", choices=["on", "off"],
                    help="decode at batch > 64: split-K partials summed by the norm / attention kernels (on) or "
                         "reduced after each GEMM (off; A/B)")
    ap.add_argument("--merged-rollout", default="on", choices=["on", "off"],
                    help="rollouts on the merged bf16 W + s*B*A copy (on) or on the unmerged LoRA K-extension (off)")
    args = ap.parse_args()
    if args.mode == "pipeline" and args.model == "mistral-7b" and "--model" not in sys.argv:
        args.model = "llama2-13b"
    # 256 rollouts per GPU: a decode step streams the weights once whatever the batch, so a larger
    # rollout batch amortises it (Mistral-7B 64 -> 128 -> 256: 4660 -> 5108 -> 6101 tokens/s,
    # profiles/bench_r1_rollout*.log; Llama-2-13B config 5: 3343 -> 3614 -> 4444 tokens/s,
    # profiles/r4/pipeline13b_rollout_batch.log); 288 GB of HBM hold the KV cache
    if args.fp8 is None:
        args.fp8 = args.mode == "pipeline"
    if args.fp8_kv is None:
        args.fp8_kv = bool(args.fp8)
    if args.fp8_train is None:
        args.fp8_train = bool(args.fp8)

    # --gpus N without a torchrun environment: start N ranks (one process per GPU) as a child
    # torch.distributed.run BEFORE anything touches the GPU, relay rank 0's JSON line and exit with
    # the ranks' status (non-zero if any rank fails or the reported world is not N)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        from rag_tl_domainllm_optimizer_amd.parallel.launch import self_launch

        sys.exit(self_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}: refusing to report a "
              f"mislabelled scaling point", file=sys.stderr, flush=True)
        sys.exit(2)

    from rag_tl_domainllm_optimizer_amd import models, parallel
    from rag_tl_domainllm_optimizer_amd.data import SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.generation import SamplingParams
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.rag import RagPipeline
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder, IVFIndex
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    di = parallel.init()
    dev = di.device
    assert di.world == args.gpus, (di.world, args.gpus)
    tuning_over = {}
    if args.tuning:
        from rag_tl_domainllm_optimizer_amd import ops

        for kv in args.tuning.split(","):
            k, v = kv.split("=")
            tuning_over[k.strip()] = float(v) if "." in v else int(v)
        ops.set_tuning(**tuning_over)
        log(f"[bench] tuning overrides: {tuning_over}")
    if args.lora_grad_epilogue == "off":
        import importlib

        importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear").DIRECT_LORA_GRADS = False
        tuning_over["lora_grad_epilogue"] = "off"
    if args.rope_fusion == "off":
        import importlib

        importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear").ROPE_EPILOGUE = False
        importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.attention").ROPE_BWD_FUSED = False
        tuning_over["rope_fusion"] = "off"
    assert dev.type == "cuda", "bench.py needs a GPU"
    # one-shot collective probe (outside every timed region): the bus bandwidth a 168 MiB fp32
    # all-reduce (the LoRA gradient payload) reaches on this job's process group (RCCL over xGMI)
    ar_probe = parallel.allreduce_bandwidth() if di.world > 1 else None
    if ar_probe:
        log(f"[bench] all-reduce probe ({ar_probe['backend']}, world {di.world}): {ar_probe['bytes'] / 1e6:.0f} MB in "
            f"{ar_probe['time_s'] * 1e3:.2f} ms, bus {ar_probe['busbw_GBps']:.1f} GB/s")
    torch.manual_seed(1234)
    t_setup = time.perf_counter()

    # ---- models (identical random init on every rank: same seed) ----
    pcfg = models.resolve_preset(args.model)
    tok = Tokenizer.synthetic(pcfg.vocab_size, pcfg.arch)
    policy = build_model(args.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    policy.defer_splitk = args.defer_splitk == "on"
    if args.defer_splitk == "off":
        tuning_over["defer_splitk"] = "off"
    enc_model = build_model(args.encoder, device=dev, dtype=torch.bfloat16, seed=1, fast_init=True).eval()
    encoder = Encoder(enc_model, Tokenizer.synthetic(enc_model.cfg.vocab_size, enc_model.cfg.arch), max_length=128)
    if args.reward_encoder in ("same", args.encoder):
        reward_encoder = encoder
    else:
        rw_model = build_model(args.reward_encoder, device=dev, dtype=torch.bfloat16, seed=2, fast_init=True).eval()
        reward_encoder = Encoder(rw_model, Tokenizer.synthetic(rw_model.cfg.vocab_size, rw_model.cfg.arch),
                                 max_length=128)
    log(f"[bench] models ready: {args.model} ({pcfg.num_params() / 1e9:.2f} B params) + {args.encoder} (retrieval) + "
        f"{args.reward_encoder} (reward)")

    # ---- corpus + IVF index in HBM ----
    corpus = SyntheticCorpus(tok.words(), n_docs=args.ndocs, doc_words=args.doc_words, seed=7)
    t0 = time.perf_counter()
    emb = encoder.encode(corpus.docs)
    index = IVFIndex(encoder.dim, nlist=args.nlist, metric="ip", device=dev, nprobe=args.nprobe)
    index.train(emb, niter=10)
    index.add(emb)
    del emb
    torch.cuda.synchronize()
    log(f"[bench] indexed {len(corpus)} docs (IVF nlist={index.nlist}) in {time.perf_counter() - t0:.1f}s")

    if args.mode in ("sft", "pipeline"):
        return run_sft_pipeline(args, di, policy, tok, encoder, corpus, index, ar_probe, reward_encoder)
    if args.mode == "serve":
        return run_serve(args, di, policy, tok, encoder, corpus, index)

    # ---- PPO trainer ----
    pc = PPOConfig(max_new_tokens=args.new_tokens, max_prompt_tokens=args.max_prompt, minibatch_size=args.minibatch,
                   lora_r=16, lora_alpha=32.0, seed=0, rollout_chunks=1, overlap_reward=True,
                   full_finetune=args.full_ft, merged_lora_rollout=args.merged_rollout == "on",
                   old_logp=args.old_logp, kl_in_loss=args.kl_in_loss == "on",
                   **({"ref_minibatch_size": args.ref_minibatch} if args.ref_minibatch else {}))
    trainer = PPOTrainer(policy, tok, RewardModel(reward_encoder), pc, max_batch=args.rollout_batch)
    if args.merged_rollout == "off":
        tuning_over["merged_rollout"] = "off"
    if args.old_logp != "rollout":
        tuning_over["old_logp"] = args.old_logp
    if args.kl_in_loss != "on":
        tuning_over["kl_in_loss"] = "off"
    if args.no_graph:
        trainer.gen.use_graph = False
    rng = random.Random(100 + di.rank)

    def make_batch():
        items = corpus.sample_queries(args.rollout_batch, seed=rng.randrange(1 << 30))
        qs = [it.query for it in items]
        _, ids = index.search(encoder.encode(qs), args.top_k_docs)
        docs = [[corpus.docs[i] for i in row if i >= 0] for row in ids.tolist()]
        if args.vary_docs:
            docs = [d[:rng.randint(1, len(d))] if d else d for d in docs]
        return {"query": qs, "retrieved_docs": docs, "ground_truth": [it.ground_truth for it in items]}

    # ---- p50 RAG answer latency (batch 1, retrieve + generate) ----
    lat = None
    if not args.skip_latency:
        rag = RagPipeline(encoder, index, corpus.docs, policy, tok, top_k=args.top_k_docs,
                          sampling=SamplingParams(max_new_tokens=args.new_tokens, temperature=0.7, top_k=50),
                          max_prompt_tokens=args.max_prompt, max_batch=1, use_graph=not args.no_graph)
        qs = [it.query for it in corpus.sample_queries(args.latency_queries + 2, seed=99)]
        lat = rag.latency_stats(qs, warmup=2)
        del rag
        torch.cuda.empty_cache()
        log(f"[bench] RAG latency p50={lat['p50_s']:.3f}s p90={lat['p90_s']:.3f}s "
            f"({lat['mean_new_tokens']:.0f} new tokens) stages={lat['stage_mean_s']}")
    ctx_lat = {}
    for L in [int(x) for x in args.latency_contexts.split(",") if x]:
        # ~50 tokens per synthetic document: retrieve enough to fill the budget, the prompt budget
        # drops the lowest-ranked ones that do not fit
        k = max(args.top_k_docs, L // 40)
        rag = RagPipeline(encoder, index, corpus.docs, policy, tok, top_k=k,
                          sampling=SamplingParams(max_new_tokens=args.new_tokens, temperature=0.7, top_k=50),
                          max_prompt_tokens=L, max_batch=1, use_graph=not args.no_graph)
        qs = [it.query for it in corpus.sample_queries(args.latency_queries + 2, seed=98)]
        st = rag.latency_stats(qs, warmup=2)
        del rag
        torch.cuda.empty_cache()
        ctx_lat[L] = st
        log(f"[bench] RAG latency @ {L}-token budget: p50={st['p50_s']:.3f}s prompt={st['mean_prompt_tokens']:.0f} "
            f"tokens, decode {st['stage_mean_s']['decode_s'] / max(st['mean_new_tokens'] - 1, 1) * 1e3:.2f} "
            f"ms/token, stages={st['stage_mean_s']}")
    log(f"[bench] setup {time.perf_counter() - t_setup:.1f}s")

    if args.steps == 0:  # latency-only (profiling) mode
        if di.is_main:
            print(json.dumps({"p50_rag_latency_s": lat["p50_s"] if lat else None, "rag_stages": lat,
                              "long_context": ctx_lat}), flush=True)
        parallel.shutdown()
        return

    # ---- PPO steps ----
    # KL(pi_theta_old || ref) per sequence of the very first step (LoRA B = 0: policy == reference),
    # measured on the first update minibatch in training numerics; with the KL in the loss this is
    # what the penalty sees at init (the pre-round-6 sampler-vs-training form read 1.83 here)
    kl_init = {}

    def note_init(m):
        if not kl_init:
            kl_init.update(kl_ref_at_init=m["kl_ref_theta_old"], kl_old_ref_at_init=m["kl_old_ref"],
                           clipfrac_first_mb_at_init=m["clipfrac_first_mb"])

    for w in range(args.warmup):
        m = trainer.step(make_batch())
        note_init(m)
        log(f"[bench] warmup {w}: {m['step_time_s']:.2f}s tokens={m['rollout_tokens']:.0f} "
            f"reward={m['reward_mean']:.3f}")
    if args.torch_profile:
        torch_profile_step(trainer, make_batch, args.torch_profile)
    parallel.barrier()
    torch.cuda.synchronize()
    trainer.sync.comm_bytes = 0
    t0 = time.perf_counter()
    tokens = 0.0
    phase = {}
    gaps, egaps, clipf, kls = [], [], [], []
    for s in range(args.steps):
        # inside the timed region: sample the rank's queries, encode them and search the IVF index
        # (retrieval), then the full PPO iteration on the retrieved RAG prompts
        m = trainer.step(make_batch())
        note_init(m)
        kls.append((m["kl_ref"], m["kl_ref_theta_old"], m["kl_old_ref"]))
        tokens += m["rollout_tokens"] * di.world  # reduce_metrics averaged over ranks
        for k, v in m.items():
            if k.startswith("time/"):
                phase[k] = phase.get(k, 0.0) + v
        gaps.append(m["behaviour_logp_gap"])
        egaps.append(m["rollout_engine_logp_gap"])
        clipf.append(m["clipfrac_first_mb"])
        log(f"[bench] step {s}: {m['step_time_s']:.2f}s loss={m['total_loss']:.4f} kl_ref={m['kl_ref']:.4f} "
            f"logp_gap={m['behaviour_logp_gap']:.2e} clipfrac0={m['clipfrac_first_mb']:.4f}")
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0  # this rank's wall time, before waiting for the others
    parallel.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    parallel.all_reduce_(elapsed, "max")
    elapsed = float(elapsed)
    spread = rank_spread(t_local / args.steps, dev)
    comm_bytes = trainer.sync.comm_bytes / args.steps
    value = tokens / elapsed
    res = {
        "metric": "PPO rollout tokens/sec (node) + p50 RAG answer latency, Mistral-7B 1/2/4/8 GPU",
        "value": value,
        "unit": "tokens/s",
        "n_gpus": di.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic (random-init weights, synthetic {args.ndocs}-doc corpus)",
        "config": {"model": args.model, "global_batch": args.rollout_batch * di.world,
                   "seq_len": args.max_prompt + args.new_tokens, "parallelism": f"dp{di.world}",
                   "new_tokens": args.new_tokens, "lora_r": None if args.full_ft else 16,
                   "full_finetune": bool(args.full_ft), "encoder": args.encoder,
                   "reward_encoder": args.reward_encoder if args.reward_encoder != "same" else args.encoder,
                   "ndocs": args.ndocs,
                   "index": f"ivf{index.nlist}/nprobe{args.nprobe}", "minibatch": args.minibatch,
                   **({"docs_per_query": f"1-{args.top_k_docs}",
                       "packed": os.environ.get("RAGTL_PACK", "1") != "0"} if args.vary_docs else {})},
        "backend": di.backend or "none",
        "world": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
        "p50_rag_latency_s": lat["p50_s"] if lat else None,
        "p90_rag_latency_s": lat["p90_s"] if lat else None,
        "rag_latency_vs_baseline": (REF_LATENCY_S / lat["p50_s"]) if lat else None,
        **({"long_context_rag": {str(k): {"p50_s": v["p50_s"], "prompt_tokens": v["mean_prompt_tokens"],
                                          "stage_mean_s": v["stage_mean_s"]} for k, v in ctx_lat.items()}}
           if ctx_lat else {}),
        "phase_s_per_step": {k: v / args.steps for k, v in phase.items()},
        # behaviour / target policy gap: mean |logp_update - old_logp| (nats per response token) and
        # the clip fraction of the first minibatch of each step, scored at theta = theta_old
        "behaviour_logp_gap": sum(gaps) / len(gaps),
        # the rollout engine's sampler log-probs vs the training forward at theta_old (equal to the
        # above unless --old-logp recompute)
        "rollout_engine_logp_gap": sum(egaps) / len(egaps),
        "old_logp_source": args.old_logp,
        "clipfrac_first_mb": sum(clipf) / len(clipf),
        # reference KL (nats / sequence): where the penalty is applied, its value over the timed steps
        # (update forwards vs reference; first minibatch at theta_old), sum_t (old_logp - ref) (the
        # sampler-based quantity the reward used before round 6), and the same at the first step
        "kl_in_loss": args.kl_in_loss == "on",
        "kl_ref": sum(k[0] for k in kls) / len(kls),
        "kl_ref_theta_old": sum(k[1] for k in kls) / len(kls),
        "kl_old_ref": sum(k[2] for k in kls) / len(kls),
        **kl_init,
        # data-parallel diagnostics: gradient payload each rank hands to RCCL per step, and the
        # spread of the per-rank step times (before the closing barrier) in seconds
        "allreduce_bytes_per_step": comm_bytes,
        "rank_step_s": spread,
        "allreduce_probe": ar_probe,
        **({"tuning": tuning_over} if tuning_over else {}),
        **({"zero_state_bytes_per_rank": trainer.opt.state_bytes()} if getattr(trainer.opt, "sharded", False)
           else {}),
    }
    if di.is_main:
        print(json.dumps(res), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(res, f, indent=2)
    parallel.shutdown()


def torch_profile_step(trainer, make_batch, path):
    """One PPO step under torch.profiler (outside the timed region): device time per op, grouped by
    the Python call site that launched it, so small torch glue kernels can be traced to source."""
    from torch.profiler import ProfilerActivity, profile

    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        trainer.step(make_batch())
        torch.cuda.synchronize()
    with open(path, "w") as f:
        f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=80,
                                                            max_name_column_width=60))
    log(f"[bench] torch profile -> {path}")


def rank_spread(step_s: float, dev) -> dict:
    """min / mean / max over ranks of one rank-local per-step wall time."""
    from rag_tl_domainllm_optimizer_amd import parallel

    t = torch.tensor([step_s], dtype=torch.float64, device=dev)
    lo, hi, sm = t.clone(), t.clone(), t.clone()
    parallel.all_reduce_(lo, "min")
    parallel.all_reduce_(hi, "max")
    parallel.all_reduce_(sm, "sum")
    world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    return {"min": float(lo), "mean": float(sm) / world, "max": float(hi)}


def _timed(di, fn, steps):
    """Run ``fn`` ``steps`` times between barriers + device syncs; returns (max-over-ranks wall
    seconds, outputs, per-rank step-time spread)."""
    from rag_tl_domainllm_optimizer_amd import parallel

    parallel.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = [fn(i) for i in range(steps)]
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0
    parallel.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=di.device)
    parallel.all_reduce_(el, "max")
    return float(el), out, rank_spread(t_local / max(steps, 1), di.device)


def run_serve(args, di, policy, tok, encoder, corpus, index):
    """RAG answer serving with dynamic request batching (serve.BatchingEngine): closed-loop clients
    at each concurrency level; answers/s, generated tokens/s and per-request latency percentiles."""
    import threading

    import numpy as np

    from rag_tl_domainllm_optimizer_amd import parallel
    from rag_tl_domainllm_optimizer_amd.generation import SamplingParams
    from rag_tl_domainllm_optimizer_amd.rag import RagPipeline
    from rag_tl_domainllm_optimizer_amd.serve import BatchingEngine, ContinuousEngine

    levels = [int(c) for c in args.serve_concurrency.split(",") if c]
    if args.fp8:
        policy.set_fp8(True)
    policy.kv_fp8 = bool(args.fp8_kv)
    rag = RagPipeline(encoder, index, corpus.docs, policy, tok, top_k=args.top_k_docs,
                      sampling=SamplingParams(max_new_tokens=args.new_tokens, temperature=0.7, top_k=50),
                      max_prompt_tokens=args.max_prompt, max_batch=max(levels), use_graph=not args.no_graph)
    qs = [it.query for it in corpus.sample_queries(args.serve_requests * len(levels) + 32, seed=17)]
    rows = []
    eng_cls = ContinuousEngine if args.serve_engine == "continuous" else BatchingEngine
    with eng_cls(rag) as eng:
        eng.answer_many(qs[:32])  # warm-up: graph capture at the batch sizes the levels produce
        for li, c in enumerate(levels):
            mine = qs[32 + li * args.serve_requests: 32 + (li + 1) * args.serve_requests]
            lat, ntok, bsz = [], [], []
            lock = threading.Lock()

            def client(part):
                for q in part:
                    a = eng.answer(q, timeout=600)
                    with lock:
                        lat.append(a.timings["total_s"])
                        ntok.append(a.timings["new_tokens"])
                        bsz.append(a.timings.get("batch_size", 0))

            ts = [threading.Thread(target=client, args=(mine[i::c],)) for i in range(c)]
            t0 = time.perf_counter()
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            el = time.perf_counter() - t0
            la = np.array(lat)
            rows.append({"concurrency": c, "answers_per_s": len(lat) / el, "tokens_per_s": float(sum(ntok)) / el,
                         "p50_latency_s": float(np.percentile(la, 50)), "p90_latency_s": float(np.percentile(la, 90)),
                         "mean_batch": float(np.mean(bsz)), "requests": len(lat)})
            log(f"[bench] serve c={c}: {rows[-1]['answers_per_s']:.2f} answers/s {rows[-1]['tokens_per_s']:.0f} tok/s "
                f"p50 {rows[-1]['p50_latency_s']:.3f}s p90 {rows[-1]['p90_latency_s']:.3f}s batch {rows[-1]['mean_batch']:.1f}")
    best = max(rows, key=lambda r: r["tokens_per_s"])
    res = {"metric": f"RAG answer serving tokens/sec ({args.serve_engine} batching), " + args.model,
           "value": best["tokens_per_s"],
           "unit": "tokens/s", "n_gpus": di.world, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "fp8-e4m3fn" if args.fp8 else "bf16", "data": "synthetic (random-init weights, synthetic corpus)",
           "config": {"model": args.model, "new_tokens": args.new_tokens, "index": f"ivf{args.nlist}/nprobe{args.nprobe}",
                      "top_k_docs": args.top_k_docs, "max_batch": max(levels)},
           "levels": rows}
    if di.is_main:
        print(json.dumps(res), flush=True)
    parallel.shutdown()


def run_sft_pipeline(args, di, policy, tok, encoder, corpus, index, ar_probe=None, reward_encoder=None):
    """config 3 (--mode sft) and config 5 (--mode pipeline) on synthetic data / random weights."""
    import random

    from rag_tl_domainllm_optimizer_amd import parallel
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.train import SFTConfig, SFTTrainer, build_raft_examples
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    rng = random.Random(200 + di.rank)
    items = corpus.sample_queries(args.sft_batch * (args.steps + args.warmup), seed=rng.randrange(1 << 30))
    ex = build_raft_examples([{"query": i.query, "ground_truth": i.ground_truth, "gold_doc": i.gold_doc}
                              for i in items], corpus.docs)
    sft = SFTTrainer(policy, tok, SFTConfig(batch_size=args.sft_batch, lora_r=16, max_seq=args.max_prompt + 64,
                                            warmup_steps=0, lr_schedule="constant"))
    B = args.sft_batch
    sft_f8 = bool(args.mode == "pipeline" and args.fp8 and args.fp8_train)
    if sft_f8:  # config 5: the SFT stage's frozen-base forwards on W8A8 as well
        policy.set_fp8(True, train=True)
    for w in range(args.warmup):
        m = sft.step(ex[w * B:(w + 1) * B])
        log(f"[bench] sft warmup {w}: {m['step_time_s']:.2f}s loss={m['loss']:.3f}")
    seq_tok = []

    def sft_step(i):
        batch = ex[(args.warmup + i) * B:(args.warmup + i + 1) * B]
        ids, start, _ = sft.encode([e["prompt"] for e in batch], [e["answer"] for e in batch])
        seq_tok.append(int((ids.shape[1] - start).sum()))
        return sft.step(batch)

    sft.sync.comm_bytes = 0
    el, ms, sft_spread = _timed(di, sft_step, args.steps)
    sft_bytes = sft.sync.comm_bytes / max(args.steps, 1)
    sft_tok = sum(seq_tok) * di.world
    res = {"metric": "RAFT LoRA SFT tokens/sec (node), " + args.model, "value": sft_tok / el, "unit": "tokens/s",
           "n_gpus": di.world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "fp8-e4m3fn frozen-base forwards / bf16 adapters and backward" if sft_f8 else "bf16",
           "data": "synthetic (random-init weights, synthetic corpus)",
           "config": {"model": args.model, "global_batch": B * di.world, "seq_len": args.max_prompt + 64,
                      "parallelism": f"dp{di.world}", "lora_r": 16, "raft_distractors": 3},
           "final_loss": ms[-1]["loss"] if ms else None,
           "world": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
           "allreduce_bytes_per_step": sft_bytes, "rank_step_s": sft_spread, "allreduce_probe": ar_probe}
    if args.mode == "sft":
        if di.is_main:
            print(json.dumps(res), flush=True)
        parallel.shutdown()
        return
    # ---- config 5: the SFT-adapted policy continues into PPO (same adapters, fp8 inference and,
    # with --fp8-train, fp8 frozen-base forwards in the update) ----
    if args.fp8:
        policy.set_fp8(True, train=args.fp8_train)
    policy.kv_fp8 = bool(args.fp8_kv)
    pc = PPOConfig(max_new_tokens=args.new_tokens, max_prompt_tokens=args.max_prompt, minibatch_size=args.minibatch,
                   lora_r=16, lora_alpha=32.0, seed=0)
    ppo = PPOTrainer(policy, tok, RewardModel(reward_encoder or encoder), pc, max_batch=args.rollout_batch)

    def make_batch():
        its = corpus.sample_queries(args.rollout_batch, seed=rng.randrange(1 << 30))
        qs = [it.query for it in its]
        _, ids = index.search(encoder.encode(qs), args.top_k_docs)
        return {"query": qs, "retrieved_docs": [[corpus.docs[i] for i in row if i >= 0] for row in ids.tolist()],
                "ground_truth": [it.ground_truth for it in its]}

    for w in range(args.warmup):
        ppo.step(make_batch())
    # retrieval (query encode + IVF search) inside the timed region, as in the headline mode
    ppo.sync.comm_bytes = 0
    el2, pm, ppo_spread = _timed(di, lambda i: ppo.step(make_batch()), args.steps)
    ppo_bytes = ppo.sync.comm_bytes / max(args.steps, 1)
    toks = sum(m["rollout_tokens"] for m in pm) * di.world
    res2 = {"metric": "RAG -> LoRA SFT -> PPO pipeline, " + args.model, "value": toks / el2, "unit": "tokens/s",
            "n_gpus": di.world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": el2 / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": ("fp8-e4m3fn inference + frozen-base training forwards / bf16 adapters and backward"
                      if args.fp8_train else "fp8-e4m3fn inference / bf16 training") if args.fp8 else "bf16",
            "data": "synthetic (random-init weights, synthetic corpus)",
            "config": {"model": args.model, "global_batch": args.rollout_batch * di.world,
                       "seq_len": args.max_prompt + args.new_tokens, "parallelism": f"dp{di.world}",
                       "lora_r": 16, "fp8": bool(args.fp8), "fp8_kv": bool(args.fp8_kv),
                       "fp8_train": bool(args.fp8 and args.fp8_train)},
            "sft": res, "ppo_phase_s_per_step": {k: sum(m[k] for m in pm) / len(pm) for k in pm[0]
                                                  if k.startswith("time/")},
            "world": res["world"], "allreduce_bytes_per_step": ppo_bytes, "rank_step_s": ppo_spread,
            "allreduce_probe": ar_probe}
    if di.is_main:
        print(json.dumps(res2), flush=True)
    parallel.shutdown()


if __name__ == "__main__":
    main()
