"""bench.py --gpus N without torchrun: the parent spawns
one child process per rank with torchrun's environment and never touches the
GPU itself; rank 0's stdout is the job's stdout, and the first failing rank
ends the job with its exit code. CPU only (children are stand-in scripts)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = """
import json, os, sys, time
r = int(os.environ["RANK"])
mode = sys.argv[1]
if mode == "fail" and r == 2:
    sys.exit(3)
if mode == "fail":
    time.sleep(60)
print(json.dumps({"rank": r, "world": os.environ["WORLD_SIZE"], "local": os.environ["LOCAL_RANK"],
                  "addr": os.environ["MASTER_ADDR"], "port": os.environ["MASTER_PORT"]}))
"""


def test_rank_envs_without_cuda():
    envs = bench.rank_envs(8, 29555, base={"PATH": "/usr/bin", "WORLD_SIZE_X": "1"})
    assert [e["RANK"] for e in envs] == [str(r) for r in range(8)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(r) for r in range(8)]
    assert {e["WORLD_SIZE"] for e in envs} == {"8"}
    assert {(e["MASTER_ADDR"], e["MASTER_PORT"]) for e in envs} == {("127.0.0.1", "29555")}
    assert {e["HSA_ENABLE_IPC_MODE_LEGACY"] for e in envs} == {"0"}
    assert all(e["PATH"] == "/usr/bin" for e in envs)
    assert not torch.cuda.is_initialized()


def test_launch_ranks_rank0_stdout(tmp_path, capfd):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    envs = bench.rank_envs(3, bench.free_port())
    rc = bench.launch_ranks(3, [sys.executable, str(script), "ok"], envs, poll_s=0.05)
    out, err = capfd.readouterr()
    assert rc == 0
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and '"rank": 0' in lines[0] and '"world": "3"' in lines[0]
    assert err.count('"rank":') == 2  # ranks 1 and 2 write to stderr
    assert not torch.cuda.is_initialized()


def test_launch_ranks_first_failure_ends_job(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    envs = bench.rank_envs(4, bench.free_port())
    t0 = time.time()
    rc = bench.launch_ranks(4, [sys.executable, str(script), "fail"], envs, poll_s=0.05)
    assert rc == 3
    assert time.time() - t0 < 40  # the sleeping ranks were terminated, not waited for


def test_maybe_launch_only_outside_torchrun(monkeypatch):
    class A:
        gpus = 1
    assert bench.maybe_launch(A) is None
    A.gpus = 4
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.maybe_launch(A) is None  # under torchrun: run in this process
