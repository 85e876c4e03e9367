"""Failure detection and fault injection.

* ``check_finite`` — non-finite loss guard (the fused AdamW also skips non-finite grad norms on
  device and counts them).
* ``maybe_inject_fault(step)`` — raises at the step named by RAGTL_FAULT_AT_STEP, so tests can
  assert that resume-from-checkpoint reproduces an uninterrupted run.
The reference has no error handling at all."""
from __future__ import annotations

import math
import os


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(step: int):
    at = os.environ.get("RAGTL_FAULT_AT_STEP")
    if at is not None and int(at) == step:
        raise InjectedFault(f"injected fault at step {step}")


def check_finite(name: str, value: float) -> bool:
    return value is not None and math.isfinite(float(value))
