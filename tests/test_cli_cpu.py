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


def test_serve_app():
    from fastapi.testclient import TestClient

    from rag_tl_domainllm_optimizer_amd.serve import create_app

    class FakePipe:
        docs = ["a", "b"]
        top_k = 2

        def answer(self, qs):
            from rag_tl_domainllm_optimizer_amd.rag import RagAnswer

            return [RagAnswer(q, "ans", [0], ["a"], [1.0], {"total_s": 0.1}) for q in qs]

    c = TestClient(create_app(FakePipe()))
    assert c.get("/health").json()["docs"] == 2
    r = c.post("/answer", json={"query": "q"}).json()
    assert r["answer"] == "ans" and r["doc_ids"] == [0]


def test_cli_ppo_resume_from_latest(tmp_path, capsys):
    args = _tiny(tmp_path) + ["--data.epochs=1"]
    cli.main(["ppo", *args])
    cli.main(["ppo", *[a for a in args if not a.startswith("--data.epochs")], "--data.epochs=2", "--resume"])
    out = capsys.readouterr().out
    assert "Resumed from" in out and "Epoch 2/2" in out and "Epoch 1/2" not in out
    assert (tmp_path / "run" / "epoch_2_trainer_state").is_dir()
