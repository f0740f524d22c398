"""Time the P > 1 shuffle's device work on ONE GPU: P contexts on device 0 each
map a C2-shaped split (same generator as bench.py, seed per rank), then
mrg_exchange_group moves the records (peer copies instead of RCCL) and every
owner re-aggregates; then each owner reduces its partitions.  The RCCL transfer
itself is not here (RCCL refuses two ranks on one device); what is here is the
count / pack / unpack / re-aggregation work every rank does around it, i.e. the
part of T(P) - T(1) that does not depend on xGMI.

usage: python tools/exchprobe.py [--P 8] [--mb 1250] [--nreduce 10] [--reps 3]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

from mrgpu import corpus as C  # noqa: E402
from mrgpu.lib import Context, MRG_APP_WC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--mb", type=int, default=1250)
    ap.add_argument("--nreduce", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    voc = C.Vocab(C.KIND_ASCII, 1.07, 1_000_000, 42)
    ctxs = [Context(0) for _ in range(a.P)]
    dptrs = []
    n = a.mb * 1_000_000
    for r in range(a.P):
        buf = np.empty(n, dtype=np.uint8)
        voc.fill_files([n], [42 + 1000 * r], C.wc_params(), threads=16, out=buf)
        d = ctxs[r].device_alloc(n)
        ctxs[r].h2d(d, buf)
        dptrs.append(d)
    for c in ctxs:
        c.sync()
    for rep in range(a.reps):
        t0 = time.perf_counter()
        local = [ctxs[r].map(MRG_APP_WC, device_ptr=dptrs[r], nbytes=n, nreduce=a.nreduce) for r in range(a.P)]
        for c in ctxs:
            c.sync()
        t1 = time.perf_counter()
        owned = Context.exchange_group(ctxs, local)
        for c in ctxs:
            c.sync()
        t2 = time.perf_counter()
        nrec_local = sum(p.info()[0] for p in local)
        nrec_owned = sum(p.info()[0] for p in owned)
        outs = [ctxs[r].reduce_all(owned[r]) for r in range(a.P)]
        for c in ctxs:
            c.sync()
        t3 = time.perf_counter()
        nbytes_out = sum(len(b) for o in outs for b in o)
        for p in local + owned:
            p.free()
        print({"P": a.P, "split_MB": a.mb, "rep": rep, "map_all_ms": round((t1 - t0) * 1e3, 2),
               "exchange_group_ms": round((t2 - t1) * 1e3, 2),
               "exchange_per_rank_ms": round((t2 - t1) * 1e3 / a.P, 3),
               "reduce_all_ms": round((t3 - t2) * 1e3, 2), "records_local": nrec_local,
               "records_owned": nrec_owned, "out_bytes": nbytes_out}, flush=True)


if __name__ == "__main__":
    main()
