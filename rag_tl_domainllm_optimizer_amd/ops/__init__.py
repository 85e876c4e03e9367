"""Public op API. One entry per native kernel; GPU tensors run the gfx950 HIP kernels, CPU tensors
the eager reference implementations (:mod:`.reference`, also the test oracles)."""
from ._ext import get_tuning, native, native_available, on_gpu, set_tuning, tuning  # noqa: F401
from .linear import (  # noqa: F401
    ACT_DSWIGLU, ACT_IDS, ACT_SWIGLU, KMAJ, ROW, FoldCache, LoRAGroup, ShufCache, SplitK, gemm, gemm_big, gemm_decode, gemm_nn, gemm_tn, linear,
    swiglu_mlp, gemm_rope, linear_rope, rope_fusable,
    refresh_lora_batched,
    linear_deferred, batch_invariant)
from .norm import layer_norm, rms_norm  # noqa: F401
from .attention import (  # noqa: F401
    attention, decode_attention, decode_step_attention, decode_workspace, flash_attention_packed, gather_rows, packed_inverse, scatter_rows,
    flash_attention_qkv, rope_qkv, rope_qkv_, FP8_KV_D, kv_dequantize, kv_quantize_rows, kv_store_fp8,
)
from .misc import (embedding, gae, ivf_scan, ppo_advantages, pool_normalize, ppo_loss, row_dot, sample, segment_mean,  # noqa: F401
                   swiglu, token_logprobs, topk)
from .optim import FlatParams, FusedAdamW, MixedFlatParams, flat_params  # noqa: F401
from .fp8 import Fp8Cache, dequantize_fp8, gemm_fp8, quantize_fp8  # noqa: F401
from . import reference  # noqa: F401
