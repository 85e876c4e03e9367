"""Scalar value head V(s) = w·h + b on the final (post-norm) hidden state.

Same parameterisation and file layout as the reference's ``torch.nn.Linear(hidden_size, 1)``
(reinforcement_learning_optimization_after_rag.py:150, saved as ``{tag}_value_head.pt`` with keys
weight [1, H] / bias [1], rl.py:368), kept in fp32.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class ValueHead(nn.Module):
    def __init__(self, hidden_size: int, device=None, seed: int = 0):
        super().__init__()
        self.linear = nn.Linear(hidden_size, 1, device=device, dtype=torch.float32)
        # explicit CPU generator: identical init on every DP rank and in every run
        g = torch.Generator(device="cpu").manual_seed(seed)
        with torch.no_grad():
            self.linear.weight.copy_(torch.randn(1, hidden_size, generator=g) / (hidden_size ** 0.5))
            self.linear.bias.zero_()

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        # a row dot product (memory-bound, one pass over h), not a library GEMV; on the GPU one
        # wave per row in a fixed order (ops.row_dot): a row's value is independent of the batch
        from .. import ops

        return ops.row_dot(h, self.linear.weight[0], self.linear.bias)

    def reference_state_dict(self):
        """{"weight": [1, H], "bias": [1]} exactly as torch.nn.Linear(H, 1).state_dict()."""
        return {"weight": self.linear.weight.detach().cpu().clone(), "bias": self.linear.bias.detach().cpu().clone()}

    def load_reference_state_dict(self, sd):
        with torch.no_grad():
            self.linear.weight.copy_(sd["weight"])
            self.linear.bias.copy_(sd["bias"])

    def trl_state_dict(self):
        """TRL AutoModelForCausalLMWithValueHead naming (v_head.summary.*)."""
        sd = self.reference_state_dict()
        return {"v_head.summary.weight": sd["weight"], "v_head.summary.bias": sd["bias"]}
