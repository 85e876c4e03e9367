"""Determinism probe for the reward / reference overlap: the same PPO rollout + prepare with
overlap_reward True / False (and RAGTL_PACK 0 / 1), printing checksums of each stage."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


def main():
    from test_pipeline_gpu import _tiny_stack
    from rag_tl_domainllm_optimizer_amd import ops
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    for pack in ("1", "0", "1", "0"):
        os.environ["RAGTL_PACK"] = pack
        for overlap in (True, False, True):
            pol, tok, enc, corpus = _tiny_stack(5)
            items = corpus.sample_queries(8, seed=1)
            batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
                     "ground_truth": [i.ground_truth for i in items]}
            tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=8, max_prompt_tokens=96,
                                                                  minibatch_size=4, lora_r=8, overlap_reward=overlap,
                                                                  seed=3), max_batch=8)
            C = ops.native()

            def dirty(tag):
                torch.cuda.synchronize()
                ws = tr.gen.workspace
                att = int((ws[2] != 0).sum()) if ws is not None else -1
                print(f"   {tag}: gemm_ws_dirty={C.decode_ws_dirty_tickets()} attn_dirty={att}", flush=True)

            ro0 = tr.rollout(batch)
            dirty("rollout0")
            tr.prepare(ro0)
            dirty("prepare0")
            ro = tr.rollout(batch)
            dirty("rollout1")
            tr.prepare(ro)
            dirty("prepare1")
            print(f"pack={pack} overlap={overlap}: resp={int(ro.resp.sum())} lens={ro.resp_len.tolist()} "
                  f"oldlp={float(ro.old_logp.sum()):.6f} reflp={float(ro.ref_logp.sum()):.6f} "
                  f"scores={[round(float(x), 5) for x in ro.scores]}", flush=True)


if __name__ == "__main__":
    main()
