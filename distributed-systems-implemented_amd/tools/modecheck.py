"""Exactness of wc_map_kernel variants selected by map_mode (benchmark knobs
that must keep results exact) on a 64 MB C2-style corpus vs the C oracle.
usage: python tools/modecheck.py 0x20000 0x40000 ..."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

import _oracle as O  # noqa: E402
from mrgpu import MRG_APP_WC, Context  # noqa: E402
from mrgpu import corpus as C  # noqa: E402


def main():
    voc = C.Vocab(C.KIND_ASCII, 1.07, 10**6, 2)
    files = [bytes(f) for f in voc.fill_files([16_000_000] * 4, [3000 + i for i in range(4)], C.wc_params())]
    want = O.c_partitioned("wc", files, 10)
    joined = b"\n".join(files)
    ctx = Context(0)
    ok = True
    for m in [int(x, 0) for x in sys.argv[1:]] or [0]:
        ctx.set_option("map_mode", m)
        got = ctx.run_job(MRG_APP_WC, joined, nreduce=10)
        st = ctx.stats()
        good = got == want
        ok &= good
        print(f"mode {m:#x}: {'exact' if good else 'MISMATCH'} dict_hits {st['dict_hits']} spilled {st['lds_overflow']}",
              flush=True)
    ctx.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
