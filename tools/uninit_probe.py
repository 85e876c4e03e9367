"""Uninitialised-memory probe: poison the caching allocator's free blocks (NaN / large values)
before building the tiny PPO stack and running rollout + prepare; results that change with the
poison come from a kernel reading memory nothing wrote."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


def poison(val):
    bufs = [torch.full((1 << 24,), val, dtype=torch.float32, device="cuda") for _ in range(64)]  # 4 GiB
    bufs += [torch.full((1 << s,), val, dtype=torch.float32, device="cuda") for s in range(8, 22) for _ in range(8)]
    torch.cuda.synchronize()
    del bufs


def main():
    from test_pipeline_gpu import _tiny_stack
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    os.environ["RAGTL_PACK"] = sys.argv[1] if len(sys.argv) > 1 else "0"
    mode = sys.argv[2] if len(sys.argv) > 2 else "prep"
    for val in (0.0, float("nan"), 3.0e4, 0.0, -1.0e30):
        poison(val)
        pol, tok, enc, corpus = _tiny_stack(5)
        items = corpus.sample_queries(8, seed=1)
        batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
                 "ground_truth": [i.ground_truth for i in items]}
        tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=8, max_prompt_tokens=96,
                                                              minibatch_size=4, lora_r=8, seed=3), max_batch=8)
        if mode == "prep":
            tr.prepare(tr.rollout(batch))
        elif mode == "roll":
            tr.rollout(batch)
        torch.cuda.synchronize()
        poison(val)
        ro = tr.rollout(batch)
        tr.prepare(ro)
        torch.cuda.synchronize()
        print(f"mode={mode} poison={val}: resp={int(ro.resp.sum())} lens={ro.resp_len.tolist()} "
              f"oldlp={float(ro.old_logp.sum()):.6f} reflp={float(ro.ref_logp.sum()):.6f} "
              f"score={float(ro.scores.sum()):.6f}", flush=True)
        del tr, pol, enc, ro
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
