"""Consecutive generations with / without a device sync between them, plus a rollout/prepare
sequence with and without syncs: which schedule changes the sampled tokens?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


def main():
    from test_pipeline_gpu import _tiny_stack
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    def sig(ro):
        return f"resp={int(ro.resp.sum())} lens={ro.resp_len.tolist()} oldlp={float(ro.old_logp.sum()):.5f}"

    for sched in ("R P s R", "R s P s R", "R s R", "R R", "R P s R", "R s P s R"):
        pol, tok, enc, corpus = _tiny_stack(5)
        items = corpus.sample_queries(8, seed=1)
        batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
                 "ground_truth": [i.ground_truth for i in items]}
        tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=8, max_prompt_tokens=96,
                                                              minibatch_size=4, lora_r=8, seed=3), max_batch=8)
        ros = []
        for op in sched.split():
            if op == "R":
                ros.append(tr.rollout(batch))
            elif op == "P":
                tr.prepare(ros[-1])
            else:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print(f"{sched:12s}: first {sig(ros[0])} | last {sig(ros[-1])} off={int(tr.gen.rng_offset)}", flush=True)


if __name__ == "__main__":
    main()
