"""CLI, config system and serving on CPU (config-1 plumbing scale)."""
import json

import pytest

from rag_tl_domainllm_optimizer_amd import cli
from rag_tl_domainllm_optimizer_amd import config as C


def test_config_overrides_and_presets(tmp_path):
    cfg = C.load(preset="config1_cpu_plumbing", overrides=["--ppo.lr=1e-4", "--reward.long_words=200",
                                                           "--ppo.lora_targets=['q_proj','v_proj']"])
    assert cfg.model.policy == "opt-125m:random" and cfg.retrieval.index == "flat"
    assert cfg.ppo.lr == 1e-4 and cfg.reward.long_words == 200
    assert cfg.ppo.lora_targets == ("q_proj", "v_proj")
    # reference defaults
    d = C.RunConfig()
    assert (d.ppo.clip_range, d.ppo.value_coef, d.ppo.entropy_coef, d.ppo.max_grad_norm, d.ppo.lam) == \
        (0.2, 0.5, 0.01, 0.5, 0.95)
    assert d.reward.weights == {"factual_accuracy": 0.5, "relevance": 0.3, "conciseness": 0.2}
    y = tmp_path / "c.yaml"
    y.write_text("ppo:\n  clip_range: 0.1\ndata:\n  batch_size: 4\n")
    cfg = C.load(str(y))
    assert cfg.ppo.clip_range == 0.1 and cfg.data.batch_size == 4
    with pytest.raises(KeyError):
        C.load(overrides=["--ppo.nope=1"])


def _tiny(tmp_path):
    return ["--model.policy=tiny-llama:random", "--model.encoder=tiny-bert:random", "--data.synthetic_docs=64",
            "--data.doc_words=16", "--retrieval.index=flat", f"--out_dir={tmp_path}", "--data.n_queries=16",
            "--data.batch_size=8", "--ppo.max_new_tokens=6", "--ppo.max_prompt_tokens=96", "--ppo.minibatch_size=4",
            "--sft.batch_size=4", "--sft.lora_r=4", "--ppo.lora_r=4"]


def test_cli_rag_and_index(tmp_path, capsys):
    cli.main(["index", *_tiny(tmp_path), f"--retrieval.index_path={tmp_path / 'idx'}"])
    cli.main(["rag", *_tiny(tmp_path), f"--retrieval.index_path={tmp_path / 'idx'}", "--query", "what is it ?"])
    lines = [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert lines[0]["ntotal"] == 64
    assert "answer" in lines[-1] and len(lines[-1]["doc_ids"]) == 3


def test_cli_pipeline_sft_then_ppo(tmp_path):
    cli.main(["pipeline", *_tiny(tmp_path)])
    import os

    run = tmp_path / "run"
    assert os.path.isdir(run / "sft_adapter") and os.path.isdir(run / "best_model_adapter")
    assert os.path.exists(run / "metrics.jsonl")
    # the reference's comparison report (rl.py:444-463, 521-525): four models, seven metric keys
    import pandas as pd

    from rag_tl_domainllm_optimizer_amd.eval import METRIC_KEYS

    rep = pd.read_csv(run / "model_comparison_results.csv", index_col=0)
    assert list(rep.columns) == ["Base Model", "RAG Model", "RL-finetuned Model", "Transfer-learned Model"]
    assert sorted(rep.index) == sorted(METRIC_KEYS)
    assert rep.notna().all().all()


def test_cli_eval_adapter_checkpoints(tmp_path, capsys):
    """cmd_eval takes PEFT adapter directories (loaded into the base policy) and names the columns
    after the reference's models."""
    import pandas as pd

    cli.main(["pipeline", *_tiny(tmp_path)])
    run = tmp_path / "run"
    rep = cli.main(["eval", *_tiny(tmp_path), "--checkpoint", str(run / "best_model_adapter"),
                    "--checkpoint", f"Transfer-learned Model={run / 'sft_adapter'}"])
    assert list(rep.columns) == ["Base Model", "RAG Model", "RL-finetuned Model", "Transfer-learned Model"]
    assert "Model Comparison Report:" in capsys.readouterr().out
    # different adapters give different answers than the base on at least one metric
    assert not rep["Base Model"].equals(rep["RL-finetuned Model"]) or not rep["RAG Model"].equals(
        rep["Transfer-learned Model"])
    assert (pd.read_csv(run / "model_comparison_results.csv", index_col=0).shape[1]) == 4


def test_serve_app():
    from fastapi.testclient import TestClient

    from rag_tl_domainllm_optimizer_amd.serve import create_app

    class FakePipe:
        docs = ["a", "b"]
        top_k = 2
        max_batch = 4

        def answer(self, qs, top_ks=None):
            from rag_tl_domainllm_optimizer_amd.rag import RagAnswer

            return [RagAnswer(q, "ans", [0], ["a"], [1.0], {"total_s": 0.1}) for q in qs]

    c = TestClient(create_app(FakePipe()))
    assert c.get("/health").json()["docs"] == 2
    r = c.post("/answer", json={"query": "q"}).json()
    assert r["answer"] == "ans" and r["doc_ids"] == [0]
    assert r["timings"]["batch_size"] == 1 and c.get("/stats").json()["requests"] == 1


def test_cli_ppo_resume_from_latest(tmp_path, capsys):
    args = _tiny(tmp_path) + ["--data.epochs=1"]
    cli.main(["ppo", *args])
    cli.main(["ppo", *[a for a in args if not a.startswith("--data.epochs")], "--data.epochs=2", "--resume"])
    out = capsys.readouterr().out
    assert "Resumed from" in out and "Epoch 2/2" in out and "Epoch 1/2" not in out
    assert (tmp_path / "run" / "epoch_2_trainer_state").is_dir()


def test_cli_pipeline_full_finetune_sft(tmp_path):
    """Full-parameter SFT writes no adapter: the pipeline hands the SFT-trained weights to PPO
    through the saved HF policy (sft_policy), and the index is built once."""
    import os

    import torch

    from rag_tl_domainllm_optimizer_amd.models import io as mio

    calls = []
    real = cli.build_stack

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)
    cli.build_stack = counting
    try:
        tr = cli.main(["pipeline", *_tiny(tmp_path), "--sft.full_finetune=True", "--sft.lr=1e-3"])
    finally:
        cli.build_stack = real
    assert len(calls) == 1
    run = tmp_path / "run"
    assert os.path.isdir(run / "sft_policy") and not os.path.isdir(run / "sft_adapter")
    # the PPO policy started from the SFT weights on disk (PPO then trains LoRA on top of them)
    sd = mio.read_state_dict(str(run / "sft_policy"))
    w = sd["model.layers.0.mlp.down_proj.weight"]
    base = tr.policy.layers[0].down_w.detach().float()
    torch.testing.assert_close(base, w.float())


def test_cli_sft_resume_and_epoch_checkpoints(tmp_path, capsys):
    args = _tiny(tmp_path) + ["--data.epochs=1", "--sft.save_every=1"]
    cli.main(["sft", *args])
    ck = tmp_path / "run" / "sft_ckpt"
    assert (ck / "epoch_1_adapter").is_dir() and (ck / "best_model_trainer_state").is_dir()
    cli.main(["sft", *[a for a in args if not a.startswith("--data.epochs")], "--data.epochs=2", "--resume"])
    out = capsys.readouterr().out
    assert "[sft] resumed from" in out and "Epoch 2/2" in out and "Epoch 1/2" not in out
    assert (ck / "epoch_2_trainer_state").is_dir()
    # a PPO resume in the same run directory must not pick up an SFT checkpoint
    assert cli.latest_checkpoint(str(tmp_path / "run")) is None


def test_held_out_eval_records_disjoint_from_training(tmp_path):
    """Evaluation items never repeat a training query (the synthetic fact set is finite, so a
    second sampling seed alone would)."""
    cfg = C.load(overrides=_tiny(tmp_path) + ["--data.n_queries=48"])
    st = cli.build_stack(cfg, cli._device().device, need_policy=False)
    train = {r["query"] for r in cli._records(cfg, st, cfg.data.n_queries)}
    held = cli._held_out_records(cfg, st, 16)
    assert held and not ({r["query"] for r in held} & train)
    assert len({r["query"] for r in held}) == len(held)
