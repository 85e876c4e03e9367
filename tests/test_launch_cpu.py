"""The self-launching multi-rank path of bench.py / cli launch (parallel/launch.py): command and
environment construction, stdout relay, world-size check, and bench.py's refusal to report a
mislabelled scaling point. Runs on CPU (gloo ranks)."""
import io
import json
import os
import subprocess
import sys
import textwrap

import pytest

from rag_tl_domainllm_optimizer_amd.parallel import launch as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_torchrun_cmd_shape():
    cmd = L.torchrun_cmd(8, ["/x/bench.py", "--steps", "3"], 29611, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-port=29611" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert cmd[-3:] == ["/x/bench.py", "--steps", "3"]
    with pytest.raises(ValueError):
        L.torchrun_cmd(0, ["x"], 1)


def test_strip_arg_forms():
    argv = ["--gpus", "4", "--steps", "2", "--gpus=8", "--warmup", "1"]
    assert L.strip_arg(argv, "--gpus") == ["--steps", "2", "--warmup", "1"]


def test_launch_env_drops_parent_rank_vars_and_adds_overrides():
    base = {"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3", "MASTER_PORT": "1", "NCCL_DEBUG": "WARN", "PATH": "/bin"}
    env = L.launch_env(["NCCL_MIN_NCHANNELS=32", "A=b=c"], base=base)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        assert k not in env
    assert env["NCCL_DEBUG"] == "WARN" and env["PATH"] == "/bin"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert env["NCCL_MIN_NCHANNELS"] == "32" and env["A"] == "b=c"
    with pytest.raises(ValueError):
        L.launch_env(["NOVALUE"], base={})


def test_free_port_is_bindable():
    import socket

    p = L.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


def test_last_json_line():
    lines = ["[log]\n", '{"a": 1}\n', "noise {\n", '{"world": 2, "value": 5}\n', "tail\n"]
    assert L.last_json_line(lines) == {"world": 2, "value": 5}
    assert L.last_json_line(["x"]) is None


_RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch.distributed as dist
    dist.init_process_group("gloo")
    w = dist.get_world_size()
    report = int(sys.argv[1]) if len(sys.argv) > 1 else w
    if dist.get_rank() == 0:
        print("[rank0] hello", flush=True)
        print(json.dumps({"world": report, "value": 1.0}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if os.environ.get("FAIL_RANK") == os.environ["RANK"]:
        sys.exit(7)
""")


def _script(tmp_path):
    p = tmp_path / "rank_script.py"
    p.write_text(_RANK_SCRIPT)
    return str(p)


def test_run_children_relays_rank0_json_and_checks_world(tmp_path):
    scr = _script(tmp_path)
    out = io.StringIO()
    rc = L.run_children(L.torchrun_cmd(2, [scr], L.free_port()), L.launch_env(), expect_world=2, out=out)
    assert rc == 0
    lines = out.getvalue().splitlines()
    assert "[rank0] hello" in lines
    assert L.last_json_line(lines)["world"] == 2
    # rank 0 reports a different world -> the launcher fails the run (mislabelled scaling point)
    rc = L.run_children(L.torchrun_cmd(2, [scr, "1"], L.free_port()), L.launch_env(), expect_world=2,
                        out=io.StringIO())
    assert rc == 3
    # a failing rank fails the launch
    rc = L.run_children(L.torchrun_cmd(2, [scr], L.free_port()), L.launch_env(["FAIL_RANK=1"]), expect_world=2,
                        out=io.StringIO())
    assert rc != 0


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "mislabelled" in r.stderr


def test_bench_gpus_n_starts_n_ranks(tmp_path):
    """``python bench.py --gpus 2`` without torchrun env launches two ranks itself. On this CPU box
    the ranks initialise a gloo world of 2 and then stop at the GPU requirement; the launch must
    report the ranks' failure (non-zero), and each rank must have seen world 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert "[launch] 2 ranks" in r.stderr
    assert "--nproc-per-node=2" in r.stderr
    assert r.returncode != 0
    assert "bench.py needs a GPU" in r.stderr


def test_bench_json_line_shape_from_launcher():
    """The parent relays the child's JSON line unchanged: json.loads of the last stdout line."""
    sample = json.dumps({"metric": "m", "value": 1.0, "n_gpus": 2, "world": 2})
    assert L.last_json_line(["[bench] x", sample]) == json.loads(sample)
