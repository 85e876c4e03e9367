"""fp8 K/V cache (config 5) on the CPU reference path: storage layout, quantisation, and a decode
step over the quantised cache against fp32 attention on the dequantised one."""
import math

import torch

from rag_tl_domainllm_optimizer_amd import ops
from rag_tl_domainllm_optimizer_amd.ops import reference as ref


def test_kperm_is_a_permutation_grouping_lane_chunks():
    from rag_tl_domainllm_optimizer_amd.ops.attention import fp8_kv_perm

    p = fp8_kv_perm(128)
    assert sorted(p.tolist()) == list(range(128))
    # lane group g of the MFMA kernel reads elements 32 s + 8 g + e (s = 0..3): bytes [32 g, 32 g + 32)
    for g in range(4):
        els = [32 * s + 8 * g + e for s in range(4) for e in range(8)]
        assert sorted(p[els].tolist()) == list(range(32 * g, 32 * g + 32))


def test_quantize_roundtrip_error_bound():
    torch.manual_seed(0)
    x = torch.randn(3, 5, 7, 128) * torch.logspace(-2, 2, 7)[None, None, :, None]
    for permute in (False, True):
        q, s = ops.kv_quantize_rows(x, permute)
        assert q.dtype == torch.uint8 and s.shape == x.shape[:-1]
        xd = ops.kv_dequantize(q, s, permute)
        # e4m3: 3 mantissa bits -> relative error <= 2^-4 of the value (normals), plus the
        # subnormal floor amax / 448 * 2^-9
        err = (xd - x).abs()
        bound = x.abs() * 2 ** -4 + x.abs().amax(-1, keepdim=True) / 448 * 2 ** -9
        assert (err <= bound + 1e-12).all()


def test_decode_step_fp8kv_cpu_matches_dequantised_attention():
    torch.manual_seed(1)
    B, Hq, Hkv, D, Smax = 2, 8, 2, 128, 40
    W = (Hq + 2 * Hkv) * D
    S = 24
    prompt = torch.randn(B * S, W).to(torch.bfloat16)
    kc = torch.zeros(B, Hkv, Smax, D, dtype=torch.uint8)
    vc = torch.zeros_like(kc)
    ks = torch.zeros(B, Hkv, 48)
    vs = torch.zeros_like(ks)
    ops.kv_store_fp8(prompt, kc, vc, ks, vs, B, S, Hq)
    k_ref = prompt[:, Hq * D:(Hq + Hkv) * D].float().reshape(B, S, Hkv, D).transpose(1, 2)
    kd = ops.kv_dequantize(kc[:, :, :S], ks[:, :, :S], True)
    assert ((kd - k_ref).abs().max() / k_ref.abs().max()).item() < 0.07
    slot = torch.tensor([S, S], dtype=torch.int32)
    attn_len = slot + 1
    pos = slot.clone()
    cos, sin = ref.rope_tables(D, 256, 10000.0, "cpu")
    qkv = torch.randn(B, W).to(torch.bfloat16)
    out = ops.decode_step_attention(qkv, kc, vc, slot, attn_len, Hq, pos, cos, sin, None, 0, k_scale=ks, v_scale=vs)
    # reference: rotate, quantise the new token into a copy of the dequantised caches, fp32 attention
    q = ops.rope_qkv_(qkv.clone(), pos, cos, sin, Hq, Hkv, D, S=1)
    kn = ops.kv_dequantize(*ops.kv_quantize_rows(q[:, Hq * D:(Hq + Hkv) * D].reshape(B, Hkv, D), True), True)
    vn = ops.kv_dequantize(*ops.kv_quantize_rows(q[:, (Hq + Hkv) * D:].reshape(B, Hkv, D), False), False)
    kfull = ops.kv_dequantize(kc, ks[..., :Smax], True)
    vfull = ops.kv_dequantize(vc, vs[..., :Smax], False)
    assert torch.allclose(kfull[:, :, S], kn) and torch.allclose(vfull[:, :, S], vn)
    o_ref = ref.decode_attention(q.float(), kfull, vfull, attn_len, Hq, None, 0, 1.0 / math.sqrt(D))
    assert (out.float() - o_ref).abs().max().item() < 2e-2 * o_ref.abs().max().item() + 1e-3
