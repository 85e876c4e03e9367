"""rag_tl_domainllm_optimizer_amd — an MI355X-native (gfx950 / CDNA4) retrieve -> generate ->
LoRA-finetune -> PPO-optimize framework.

Subpackages: ops (HIP kernels + oracles), models, tokenizer, generation, retrieval, rag, rewards,
metrics, train (PPO, RAFT SFT, checkpoints), eval, parallel (RCCL data parallel), runtime, utils,
serve, compat (reference API), cli.
"""
__version__ = "0.1.0"
