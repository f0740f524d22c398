"""Host code under AddressSanitizer / UBSan (the analogue of the
reference's `go build -race`; GPU code is not instrumented — GPU ASan is not
available on this pool):

* the oracle's restatements (oracle/mroracle.c, oracle/mrcount.c) on the golden
  edge cases and a synthetic UTF-8 corpus: the partitioned oracle, the threaded
  counter (1 and 3 threads) and the merge of per-file outputs must agree;
* the coordinator (build/mrcoord_gpu_asan) driven through the task protocol
  by fake workers (tests/test_coordinator.py's CPU test, same binary built with
  -fsanitize=address,undefined).
"""
from __future__ import annotations

import os
import subprocess

import pytest

import cases
import test_coordinator as TC
from mrgpu import corpus as C
from mrgpu.lib import BUILD_DIR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def asan_builds():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "distributed-systems-implemented_amd"), "asan"], check=True)


def test_oracle_under_asan(asan_builds, tmp_path):
    exe = os.path.join(ROOT, "oracle", "_build", "asan_driver")
    files = []
    for name, fs in sorted(cases.edge_cases().items()):
        for i, f in enumerate(fs):
            p = tmp_path / f"{name}-{i}.txt"
            p.write_bytes(f)
            files.append(str(p))
    for i, f in enumerate(cases.synthetic(C.KIND_UTF8, 5000, [200_000, 150_001], 51, 0.001)):
        p = tmp_path / f"syn-{i}.txt"
        p.write_bytes(f)
        files.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    for pat, R in (("distributed", 10), ("e", 3), ("κόσμε", 7)):
        r = subprocess.run([exe, pat, str(R)] + files, capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-3000:]


def test_coordinator_protocol_under_asan(asan_builds, tmp_path, monkeypatch):
    exe = os.path.join(BUILD_DIR, "mrcoord_gpu_asan")
    monkeypatch.setattr(TC, "COORD", exe)
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=0")  # the HIP runtime it links keeps allocations to exit
    TC.test_handout_order_wait_reissue_and_done(tmp_path)
