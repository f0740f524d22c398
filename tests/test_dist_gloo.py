"""N > 1 on CPU: the multi-rank protocol with gloo, world_size 2.

Each rank maps its own shard of the input files (the oracle stands in for the
device map — no GPU here), builds per-key partials with partition =
ihash(key) % R, sends every key to rank (partition % world) as MRGI bytes
(mrgpu.intermediate, the mrg_parts_export format) through the counts-then-payload
all-to-all of mrgpu.dist, merges what it owns and formats its partitions.  The
union over ranks must equal the single-rank oracle's mr-out-r exactly, and
non-owned partitions must be empty.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent(r'''
    import json, os, sys, collections
    sys.path.insert(0, os.path.join(sys.argv[1], "distributed-systems-implemented_amd"))
    sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
    import torch.distributed as dist
    import _oracle as O, cases
    from mrgpu import dist as D, intermediate as I
    from mrgpu import corpus as C
    dist.init_process_group("gloo")
    rank, world, _ = D.env_ranks()
    R = 10
    files = cases.synthetic(C.KIND_UTF8, 20000, [120_000, 90_000, 150_001, 70_000, 40_000], 41, 0.001)
    mine = [f for i, f in enumerate(files) if i % world == rank]          # shard: files round-robin
    counts = collections.Counter()
    for f in mine:                                                        # map (oracle stand-in)
        counts.update(O.mr_oracle.wc_map(f))
    send = []
    for dst in range(world):                                              # pack per owner
        keys = [k for k in counts if D.owner_of(O.c_ihash(k) % R, world) == dst]
        send.append(I.encode(1, R, keys, [counts[k] for k in keys], [O.c_ihash(k) % R for k in keys]))
    recv = D.alltoallv_bytes(send)                                        # shuffle
    merged = collections.Counter()
    for b in recv:                                                        # merge owned partials
        d = I.decode(b)
        for k, c, p in zip(d["keys"], d["count"], d["kpart"]):
            assert D.owner_of(int(p), world) == rank
            merged[k] += int(c)
    out = {}
    for r in range(R):                                                    # reduce owned partitions
        keys = sorted(k for k in merged if O.c_ihash(k) % R == r)
        out[r] = b"".join(k + b" " + str(merged[k]).encode() + b"\n" for k in keys).hex()
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        want = O.c_partitioned("wc", files, R)
        ok = True
        for r in range(R):
            own = D.owner_of(r, world)
            for q in range(world):
                got = bytes.fromhex(gathered[q][r])
                ok &= got == (want[r] if q == own else b"")
        print(json.dumps({"ok": bool(ok), "max_t": D.max_over_ranks(1.0)}))
    else:
        D.max_over_ranks(2.0)
    dist.destroy_process_group()
''')


def test_two_rank_shuffle_gloo(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", "29517", str(script), ROOT],
                         capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [l for l in res.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert r["ok"] and r["max_t"] == 2.0


def test_intermediate_codec_roundtrip():
    sys.path.insert(0, os.path.join(ROOT, "distributed-systems-implemented_amd"))
    from mrgpu import intermediate as I
    keys = [b"a", b"abcdefghijklmnop", b"abcdefghijklmnopq", "κόσμε".encode(), b"x" * 100]
    b = I.encode(1, 10, keys, [1, 2, 3, 4, 5], [0, 1, 2, 3, 4])
    d = I.decode(b)
    assert d["keys"] == keys and list(d["count"]) == [1, 2, 3, 4, 5] and list(d["kpart"]) == [0, 1, 2, 3, 4]
    with pytest.raises(ValueError):
        I.decode(b[:-1])


MULTI = textwrap.dedent(r'''
    import json, os, sys
    sys.path.insert(0, sys.argv[1])
    import torch.distributed as dist
    dist.init_process_group("gloo")
    import bench
    rank, world = dist.get_rank(), dist.get_world_size()
    # per-step stats as mrg_get_stats reports them after an RCCL exchange
    st = {"exchange_ms": 3.0 + rank, "exchange_a2a_ms": 2.0 + rank, "exchange_unpack_ms": 1.0,
          "shuffle_send_bytes": 1.0e9 * (rank + 1), "rccl_nranks": world, "rccl_rank": rank, "device": rank}
    m = bench.multi_fields([st, st], t_max=0.02, t1=0.016, world=world, shared=False, ndev=world)
    if rank == 0:
        print(json.dumps(m))
    dist.destroy_process_group()
''')


def test_multi_gpu_fields_gloo(tmp_path):
    """bench.py's N > 1 fields on two gloo ranks: the exchange split into its
    all-to-all and the owner's unpack + re-aggregation (max over ranks), the rank
    count RCCL reported and each rank's device, gathered to rank 0; the xGMI
    rate is taken over the all-to-all time only."""
    script = tmp_path / "multi.py"
    script.write_text(MULTI)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", "29518", str(script), ROOT],
                         capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    m = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
    assert m["exchange_ms"] == 4.0 and m["exchange_a2a_ms"] == 3.0 and m["exchange_unpack_ms"] == 1.0
    assert m["rccl_nranks"] == [2]
    assert [(r["rank"], r["rccl_rank"], r["device"]) for r in m["ranks"]] == [(0, 0, 0), (1, 1, 1)]
    assert m["shuffle_bytes_per_gpu"] == 2_000_000_000
    # rank 0's own rate: 1e9 bytes over its 2 ms all-to-all; 1 link at P = 2
    assert m["xgmi_achieved_GBps"] == 500.0 and m["xgmi_peak_GBps"] == 153.0
    assert m["weak_scaling_efficiency"] == 0.8
