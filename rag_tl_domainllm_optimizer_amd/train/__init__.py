"""Training: PPO after RAG (config 4), RAFT LoRA SFT (config 3), checkpointing, schedules."""
from .common import lr_at, masked_mean, masked_whiten, response_mask, score_sequences  # noqa: F401
from .raft import RaftConfig, build_raft_examples  # noqa: F401
from .sft import SFTConfig, SFTTrainer  # noqa: F401
from .ppo import PPOConfig, PPOTrainer, Rollout  # noqa: F401
from .checkpoint import load_checkpoint, save_checkpoint  # noqa: F401
