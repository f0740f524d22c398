"""CPU test of the shuffle's send / receive layout (csrc/mrgpu_exch.h), the plan
mrg_exchange hands to ncclAllToAllv (replacing mr/worker.go:80-122's mr-X-Y
files): a simulated P-rank all-to-all with empty segments, a rank that sends
nothing and one that receives nothing (tests/native/exch_plan_sim.cpp)."""
from __future__ import annotations

import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "exch_plan_sim.cpp")


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("exch") / "exch_plan_sim")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-fsanitize=address,undefined", "-o", exe, SRC],
                   check=True)
    return exe


@pytest.mark.parametrize("P,seed", [(1, 1), (2, 2), (3, 3), (8, 4), (8, 5), (8, 6), (16, 7), (64, 8)])
def test_exchange_plan_all_to_all(sim, P, seed):
    r = subprocess.run([sim, str(P), str(seed)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith(f"ok {P} ")
