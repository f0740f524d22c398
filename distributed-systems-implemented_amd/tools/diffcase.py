"""Debug helper: run one wc case through the library and list the keys whose
counts differ from the oracle (tests/_oracle.py), per partition.
    python tools/diffcase.py [--opt name=value ...]"""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "distributed-systems-implemented_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa
import _oracle as O, cases
from mrgpu import Context, MRG_APP_WC
from mrgpu import corpus as C

ap = argparse.ArgumentParser()
ap.add_argument("--opt", action="append", default=[])
ap.add_argument("--case", default="coord")
a = ap.parse_args()
if a.case == "coord":
    files = cases.synthetic(C.KIND_UTF8, 20000, [300_000, 200_000, 250_000, 1_000, 90_000], 61, 0.001)
else:
    files = cases.edge_cases()[a.case]
R = 10
with Context(0) as ctx:
    for o in a.opt:
        k, v = o.split("=")
        ctx.set_option(k, int(v))
    for fi, f in enumerate(files):
        got = ctx.run_job(MRG_APP_WC, f, nreduce=R)
        want = O.c_partitioned("wc", [f], R)
        if got == want:
            print(f"file {fi}: ok ({len(f)} bytes)")
            continue
        def parse(parts):
            d = {}
            for p in parts:
                for l in p.split(b"\n")[:-1]:
                    k, v = l.rsplit(b" ", 1)
                    d[k] = int(v)
            return d
        g, w = parse(got), parse(want)
        bad = [(k, g.get(k), w.get(k)) for k in set(g) | set(w) if g.get(k) != w.get(k)]
        print(f"file {fi}: {len(bad)} keys differ ({len(f)} bytes); gpu stats {ctx.stats()['spill_buckets']}")
        for k, x, y in sorted(bad, key=lambda t: -(t[2] or 0))[:25]:
            print("   ", k, len(k), "gpu", x, "oracle", y)
