"""Ablation probe for wc_map_kernel (benchmark-only; map_mode != 0 gives wrong results).

Times the map kernel over the C2 (or C5: --workload c5) corpus with phases switched off:
  mode 1 = read input only, 2 = tokenize only, 4 = + key extraction (no table), 0 = full;
  mode 128 = aggregator reads + hashes its records only (agg_ms).
usage: python tools/mapprobe.py [--gb 10] [--modes 1,2,4,0] [--grids 256,512] [--workload c2|c5]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # the repo root (bench.py's corpus generator)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from mrgpu import MRG_APP_WC, Context  # noqa: E402
from mrgpu import corpus as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10)
    ap.add_argument("--modes", default="1,2,4,0")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="context option name=value (repeatable)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c2u", "c5"])
    a = ap.parse_args()
    nfiles = max(1, int(a.gb * 4))
    if a.workload in ("c5", "c2u"):
        import bench
        buf = bench.gen_corpus(bench.WORKLOADS[a.workload], 0, 250, nfiles)
    else:
        voc = C.Vocab(C.KIND_ASCII, 1.07, 10**6, 2)
        sizes = [250_000_000] * nfiles
        buf = np.empty(sum(sizes), dtype=np.uint8)
        voc.fill_files(sizes, [2 + i for i in range(nfiles)], C.wc_params(), out=buf)
    ctx = Context(0)
    for o in a.opt:
        k, v = o.split("=")
        ctx.set_option(k, int(v))
    d = ctx.device_alloc(buf.size)
    for off in range(0, buf.size, 1 << 30):
        n = min(1 << 30, buf.size - off)
        ctx.h2d(d + off, buf[off:off + n], n)
    res = []
    for g in [int(x) for x in a.grids.split(",")]:
        ctx.set_option("map_grid", g)
        for m in [int(x, 0) for x in a.modes.split(",")]:
            ctx.set_option("map_mode", m)
            ts = []
            for _ in range(a.reps):
                p = ctx.map(MRG_APP_WC, None, device_ptr=d, nbytes=buf.size, nreduce=10)
                st = ctx.stats()
                ts.append(st["map_kernel_ms"])
                p.free()
            r = {"grid": g, "mode": m, "map_kernel_ms": min(ts), "all_ms": [round(x, 3) for x in ts],
                 "GBps": buf.size / min(ts) / 1e6,
                 "map_total_ms": st["map_total_ms"], "agg_ms": st["agg_ms"], "long_ms": st["long_ms"],
                 "collect_ms": st["collect_ms"], "spilled": st["lds_overflow"], "agg_miss": st["agg_miss"],
                 "dict_ms": st["dict_ms"], "dict_hits": st["dict_hits"],
                 "spill_record_bytes": st.get("spill_record_bytes", 0)}
            print(json.dumps(r), flush=True)
            res.append(r)
    ctx.set_option("map_mode", 0)
    ctx.device_free(d)
    ctx.close()


if __name__ == "__main__":
    main()
