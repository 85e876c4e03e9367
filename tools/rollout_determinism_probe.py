"""Rollout determinism probe (found the fused decode-attention clamped-key race): builds a fresh
tiny PPO stack per repetition and prints token / log-prob / value sums, which must be identical.
MODE: keep (previous trainer alive while the next is built), poison (NaN-fill freed memory first),
nograph (eager decode)."""
import os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
from test_pipeline_gpu import _tiny_stack
from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

def poison():
    x = torch.full((1 << 28,), float("nan"), device="cuda")
    del x
    torch.cuda.synchronize()

mode = os.environ.get("MODE", "")
for rep in range(6):
    if "poison" in mode:
        poison()
    pol, tok, enc, corpus = _tiny_stack(5)
    items = corpus.sample_queries(8, seed=1)
    batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
             "ground_truth": [i.ground_truth for i in items]}
    tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=8, max_prompt_tokens=96, minibatch_size=4,
                    lora_r=8, overlap_reward=True, seed=3), max_batch=8)
    if "nograph" in mode:
        tr.gen.use_graph = False
    ro = tr.rollout(batch)
    torch.cuda.synchronize()
    print(mode, rep, ro.resp.sum().item(), ro.old_logp.sum().item(), ro.old_values.sum().item(), flush=True)
    if "keep" not in mode:
        del tr, ro
