"""PEFT / TRL checkpoint formats on CPU: adapter key names and shapes,
adapter_config.json fields, adapter round trip, merge == adapter forward, unmerge restores the base,
merge-and-drop leaves a plain model, value-head layouts (reference rl.py:150,365-370)."""
import json

import torch

from rag_tl_domainllm_optimizer_amd import models
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
from rag_tl_domainllm_optimizer_amd.models.lora import (adapter_state_dict, load_adapter, merge_and_drop_lora,
                                                        merge_lora, save_adapter)

TARGETS = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


def _model(seed=1):
    m = models.CausalLM(PRESETS["tiny-mistral"], dtype=torch.float32, seed=seed)
    m.add_lora(4, 8.0, "all", seed=3)
    with torch.no_grad():
        for p in m.lora_parameters():
            p.normal_(0, 0.05)
    m.refresh_lora()
    return m


def test_adapter_keys_shapes_and_config(tmp_path):
    from safetensors.torch import load_file

    m = _model()
    cfg = m.cfg
    sd = adapter_state_dict(m)
    pre = "base_model.model.model.layers"
    assert sd[f"{pre}.0.self_attn.q_proj.lora_A.weight"].shape == (4, cfg.hidden_size)
    assert sd[f"{pre}.0.self_attn.k_proj.lora_B.weight"].shape == (cfg.num_kv_heads * cfg.head_dim, 4)
    assert sd[f"{pre}.1.mlp.down_proj.lora_A.weight"].shape == (4, cfg.intermediate_size)
    assert sd[f"{pre}.1.mlp.gate_proj.lora_B.weight"].shape == (cfg.intermediate_size, 4)
    assert len(sd) == 2 * len(TARGETS) * cfg.num_layers
    save_adapter(m, str(tmp_path / "ad"))
    c = json.load(open(tmp_path / "ad" / "adapter_config.json"))
    assert c["peft_type"] == "LORA" and c["task_type"] == "CAUSAL_LM" and c["r"] == 4 and c["lora_alpha"] == 8.0
    assert c["bias"] == "none" and c["fan_in_fan_out"] is False and sorted(c["target_modules"]) == sorted(TARGETS)
    assert set(load_file(str(tmp_path / "ad" / "adapter_model.safetensors"))) == set(sd)


def test_adapter_roundtrip_merge_unmerge(tmp_path):
    m = _model()
    ids = torch.randint(3, m.cfg.vocab_size, (2, 12))
    with torch.no_grad():
        y = m(ids)
    save_adapter(m, str(tmp_path / "ad"))
    m2 = models.CausalLM(m.cfg, dtype=torch.float32, seed=1)  # same base weights, no adapters
    load_adapter(m2, str(tmp_path / "ad"))
    with torch.no_grad():
        torch.testing.assert_close(m2(ids), y, rtol=1e-5, atol=1e-5)
    base = {n: p.detach().clone() for n, p in m.named_parameters() if "lora" not in n}
    merge_lora(m)
    m.set_lora_enabled(False)
    with torch.no_grad():
        torch.testing.assert_close(m(ids), y, rtol=1e-4, atol=1e-4)
    merge_lora(m, sign=-1.0)
    for n, p in m.named_parameters():
        if n in base:
            torch.testing.assert_close(p.detach(), base[n], rtol=1e-5, atol=1e-6)
    # merge-and-drop: a plain model computing the adapted function
    m.set_lora_enabled(True)
    merge_and_drop_lora(m)
    assert getattr(m, "lora_config", None) is None and not m.lora_parameters()
    with torch.no_grad():
        torch.testing.assert_close(m(ids), y, rtol=1e-4, atol=1e-4)


def test_value_head_layouts():
    vh = models.ValueHead(16, seed=2)
    lin = torch.nn.Linear(16, 1)
    lin.load_state_dict(vh.reference_state_dict())  # exactly torch.nn.Linear(H, 1)'s state dict
    h = torch.randn(3, 16)
    torch.testing.assert_close(vh(h), lin(h).squeeze(-1))
    assert set(vh.trl_state_dict()) == {"v_head.summary.weight", "v_head.summary.bias"}
