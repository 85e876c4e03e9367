"""Metrics sink: JSONL on rank 0 (runs/<name>/metrics.jsonl), optional wandb forwarding when the
package is importable (the reference logs to wandb, reinforcement_learning_optimization_after_rag.py:268,340-351)."""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Optional


class MetricsSink:
    def __init__(self, run_dir: Optional[str] = None, enabled: bool = True, use_wandb: bool = False,
                 project: str = "rl-after-rag", config: Optional[dict] = None, stdout: bool = False):
        self.enabled = enabled
        self.stdout = stdout
        self.path = None
        self._wandb = None
        self.history = []
        if enabled and run_dir:
            os.makedirs(run_dir, exist_ok=True)
            self.path = os.path.join(run_dir, "metrics.jsonl")
            if config is not None:
                with open(os.path.join(run_dir, "config.json"), "w") as f:
                    json.dump(config, f, indent=2, default=str)
        if enabled and use_wandb:
            try:
                import wandb  # noqa: F401

                wandb.init(project=project, config=config)
                self._wandb = wandb
            except Exception:
                self._wandb = None

    def log(self, metrics: dict, step: Optional[int] = None):
        if not self.enabled:
            return
        rec = {"time": time.time(), **({"step": step} if step is not None else {}), **metrics}
        self.history.append(rec)
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        if self.stdout:
            print(json.dumps(rec, default=float), file=sys.stderr, flush=True)
        if self._wandb is not None:
            self._wandb.log(metrics, step=step)

    def finish(self):
        if self._wandb is not None:
            self._wandb.finish()
