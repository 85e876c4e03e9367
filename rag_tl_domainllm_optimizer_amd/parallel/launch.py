"""Start one process per GPU from a plain ``python script.py --gpus N`` invocation.

``bench.py --gpus N`` (and ``cli launch``) must not run N GPUs' worth of work in ONE process: the
parent builds a ``torch.distributed.run`` command (single node, rendezvous on 127.0.0.1, a free
port), starts it as a CHILD process before anything touches the GPU (the parent never initialises
HIP, so no exec-after-GPU-init hazard), relays the children's stdout line by line, and reports the
children's exit status. The reference runs on one device only
(reinforcement_learning_optimization_after_rag.py:165-168); this is the launcher of the DP path.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from typing import Dict, Iterable, List, Optional, Sequence


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 (the rendezvous port of the child launch)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def torchrun_cmd(nproc: int, target: Sequence[str], port: int, python: Optional[str] = None) -> List[str]:
    """``python -m torch.distributed.run`` over ``nproc`` local ranks running ``target`` (a script
    path followed by its arguments, or ``["-m", module, ...]``)."""
    if nproc < 1:
        raise ValueError(f"nproc must be >= 1, got {nproc}")
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", *target]


def launch_env(extra: Iterable[str] = (), base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """The ranks' environment: the caller's (NCCL_* / RCCL_* / HSA_* tuning and RAGTL_* switches
    pass through), dmabuf IPC for RCCL (``HSA_ENABLE_IPC_MODE_LEGACY=0``), plus KEY=VALUE entries.
    Launcher variables inherited from an enclosing torchrun are dropped so the children get their
    own rank / world."""
    env = dict(os.environ if base is None else base)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
              "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for kv in extra:
        k, sep, v = kv.partition("=")
        if not sep or not k:
            raise ValueError(f"--env expects KEY=VALUE, got {kv!r}")
        env[k] = v
    return env


def strip_arg(argv: Sequence[str], name: str) -> List[str]:
    """``argv`` without ``name VALUE`` / ``name=VALUE`` (e.g. to re-pass --gpus explicitly)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == name:
            skip = True
            continue
        if a.startswith(name + "="):
            continue
        out.append(a)
    return out


def last_json_line(lines: Iterable[str]) -> Optional[dict]:
    """The last stdout line that parses as a JSON object (rank 0's result line)."""
    res = None
    for ln in lines:
        ln = ln.strip()
        if ln.startswith("{") and ln.endswith("}"):
            try:
                res = json.loads(ln)
            except ValueError:
                pass
    return res


def run_children(cmd: Sequence[str], env: Dict[str, str], expect_world: Optional[int] = None,
                 out=None) -> int:
    """Run the launch command, echo its stdout as it arrives, and return its exit code — or 3 when it
    succeeded but rank 0's JSON line reports a world size other than ``expect_world`` (a mislabelled
    scaling point is a failure, not a result)."""
    out = out or sys.stdout
    proc = subprocess.Popen(list(cmd), env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    seen: List[str] = []
    assert proc.stdout is not None
    for ln in proc.stdout:
        out.write(ln)
        out.flush()
        seen.append(ln)
    rc = proc.wait()
    if rc != 0:
        print(f"[launch] ranks exited with code {rc}", file=sys.stderr, flush=True)
        return rc
    if expect_world is not None:
        res = last_json_line(seen)
        world = None if res is None else res.get("world", res.get("n_gpus"))
        if world != expect_world:
            print(f"[launch] expected world {expect_world}, rank 0 reported {world}", file=sys.stderr, flush=True)
            return 3
    return 0


def self_launch(nproc: int, script: str, argv: Sequence[str], gpus_flag: str = "--gpus",
                extra_env: Iterable[str] = ()) -> int:
    """Re-run ``script`` under torch.distributed.run with ``nproc`` ranks (``argv`` keeps every
    other flag; ``--gpus N`` is passed explicitly) and return the combined exit code."""
    target = [os.path.abspath(script), *strip_arg(argv, gpus_flag), gpus_flag, str(nproc)]
    cmd = torchrun_cmd(nproc, target, free_port())
    print(f"[launch] {nproc} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return run_children(cmd, launch_env(extra_env), expect_world=nproc)
