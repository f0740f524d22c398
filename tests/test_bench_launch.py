"""bench.py's N > 1 launch (VERDICT r05 "do this" 1): plain `python bench.py
--gpus N` with no WORLD_SIZE starts its N ranks itself as a child
torch.distributed.run, and the N > 1 headline is C4 (12.5 GB per GPU, nReduce
64, BASELINE.json configs[3]) with the C5 E(P) sub-run."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def _line(stdout: str) -> dict:
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_self_launch_dry_run():
    """--gpus 2 without a launcher: two gloo ranks come up (the child launcher),
    rank 0 alone prints, the workload defaults to C4 at R = 64, host threads
    are split over the node's ranks; no GPU is touched (--dry-run)."""
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _line(res.stdout)
    assert d["n_gpus"] == 2 and d["ranks"] == [0, 1]
    assert d["workload"] == "c4" and d["nreduce"] == 64 and d["input_bytes_per_gpu"] == 12_500_000_000
    assert d["scaling_workload"] == "c5"
    assert d["host_threads"] == max(1, min(16, (os.cpu_count() or 1) // 2))


def test_single_gpu_default_is_c2():
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"],
                         capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _line(res.stdout)
    assert d["n_gpus"] == 1 and d["workload"] == "c2" and d["nreduce"] == 10
    assert d["input_bytes_per_gpu"] == 10_000_000_000


def test_self_launch_forwards_exit_code(monkeypatch):
    """The parent runs the launcher as a child (never an exec) with the same
    arguments and returns the child's exit status."""
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    assert bench.self_launch(["--gpus", "8", "--steps", "3"], 8) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3"][-4:]
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1"


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_self_launched_rehearsal_line():
    """`bench.py --gpus 2 --rehearsal` on a one-GPU box (shrunk splits): the
    self-launched ranks share the device (no RCCL exchange, flagged), and rank
    0 prints ONE line with n_gpus 2, C4 at R = 64, the multi_gpu fields, the
    C5 sub-run and the per-phase wall seconds."""
    args = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearsal",
            "--files", "2", "--file-mb", "50", "--scaling-files", "2", "--steps", "2", "--warmup", "1",
            "--scaling-steps", "1", "--no-cpu-baseline", "--no-pcie", "--no-pipelined"]
    res = subprocess.run(args, capture_output=True, text=True, timeout=280, env=_env(), cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _line(res.stdout)
    assert d["n_gpus"] == 2 and d["rehearsal"] is True
    assert d["config"]["workload"].startswith("C4") and d["config"]["nreduce"] == 64
    assert d["config"]["parallelism"] == "dp2"
    m = d["multi_gpu"]
    for k in ("exchange_ms", "exchange_a2a_ms", "shuffle_bytes_per_gpu", "xgmi_frac", "weak_scaling_efficiency",
              "rccl_nranks", "ranks"):
        assert k in m, k
    assert [r["rank"] for r in m["ranks"]] == [0, 1]
    s = d["multi_gpu_scaling_workload"]
    assert s["nreduce"] == 64 and s["checks"]["sorted_unique"] and s["checks"]["partition_ok"]
    assert s["checks"]["total_words_match"]
    assert d["checks"]["sorted_unique"] and d["checks"]["total_words_match"]
    assert d["checks"]["exact_vs_oracle"]  # each rank's own split (no exchange in a rehearsal)
    assert {"generate", "upload", "warmup_and_timed_steps", "scaling_subrun", "total"} <= set(d["wall_s"])
