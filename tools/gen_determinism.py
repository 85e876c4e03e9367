"""Generation determinism probe: the same sampled generation from fresh Generators (graph / eager)
and from one reused Generator; prints per-run checksums of tokens and log-probs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


def main():
    from test_pipeline_gpu import _tiny_stack
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.rag.prompt import build_prompt

    pol, tok, enc, corpus = _tiny_stack(5)
    pol.add_lora(8, 16.0, None, seed=1)
    pol.refresh_lora()
    items = corpus.sample_queries(8, seed=1)
    prompts = [tok.encode(build_prompt(i.query, [corpus.docs[i.gold_doc]]))[-96:] for i in items]
    sp = SamplingParams(max_new_tokens=8, temperature=0.7, top_k=50)
    ref = None
    for mode in ("graph", "eager", "graph"):
        for rep in range(4):
            gen = Generator(pol, 8, 96 + 16, torch.device("cuda"))
            gen.use_graph = mode == "graph"
            outs = [gen.generate(prompts, sp, pad_id=tok.pad_token_id, eos_ids=[tok.eos_token_id]) for _ in range(2)]
            torch.cuda.synchronize()
            for k, o in enumerate(outs):
                sig = (o.tokens.cpu().tolist(), o.lengths.cpu().tolist())
                lp = float(o.logprobs.float().sum())
                same = ref is None or sig == ref[0]
                if ref is None:
                    ref = (sig, lp)
                print(f"{mode} rep{rep} call{k}: same_tokens={same} lens={sig[1]} lp={lp:.6f} dlp={lp - ref[1]:.2e}",
                      flush=True)


if __name__ == "__main__":
    main()
