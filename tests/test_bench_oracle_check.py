"""bench.py's full-size exact check (oracle_exact_check) on the CPU: one rank,
and two gloo ranks whose oracle partitions travel to their owners (r % N) and
are merged there (mr/worker.go:123-146 over every split's intermediates).  The
"GPU output" here is the single-process oracle's, restricted to each rank's
owned partitions, so a routing or merge bug makes the check fail; a corrupted
partition must be reported."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent(r'''
    import json, os, sys
    root = sys.argv[1]
    sys.path.insert(0, root); sys.path.insert(0, os.path.join(root, "tests"))
    import numpy as np
    import torch.distributed as dist
    import bench, cases, _oracle as O
    from mrgpu import corpus as C
    world = int(os.environ.get("WORLD_SIZE", "1")); rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    res = {}
    for app, w in (("wc", bench.WORKLOADS["c2u"]), ("grep:distributed", bench.WORKLOADS["c3"])):
        if app == "wc":
            splits = [b"\n".join(cases.synthetic(C.KIND_UTF8, 30000, [400_000, 300_000], 60 + i, 0.001)) for i in range(world)]
        else:
            splits = [b"\n".join(cases.synthetic_grep(30000, [500_000], 70 + i)) for i in range(world)]
        R = 10
        want = O.c_partitioned(app, splits, R)
        gpu = [want[r] if r % world == rank else b"" for r in range(R)]
        host = np.frombuffer(splits[rank], dtype=np.uint8)
        ok = bench.oracle_exact_check(w, host, gpu, R, rank, world)["exact_vs_oracle"]
        bad = list(gpu)
        mine = [r for r in range(R) if r % world == rank]
        bad[mine[0]] = bad[mine[0]][:-1]  # a truncated partition
        caught = not bench.oracle_exact_check(w, host, bad, R, rank, world)["exact_vs_oracle"]
        res[app] = [ok, caught]
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()
''')


def _run(tmp_path, nproc):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if nproc == 1:
        cmd = [sys.executable, str(script), ROOT]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", "29527", str(script), ROOT]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [l for l in res.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_bench_oracle_check_one_rank(tmp_path):
    r = _run(tmp_path, 1)
    assert r == {"wc": [True, True], "grep:distributed": [True, True]}


def test_bench_oracle_check_two_ranks_gloo(tmp_path):
    r = _run(tmp_path, 2)
    assert r == {"wc": [True, True], "grep:distributed": [True, True]}
