"""Pin the C1 substitute corpus (mrgpu.corpus.c1_files, seed 1) and the
oracle's outputs on it: SHA-256 of every file, of mrsequential's mr-out-0 and
of every mr-out-r at nReduce = 10.  Re-run:  python tests/golden/make_c1_manifest.py"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "distributed-systems-implemented_amd"))

import _oracle as O  # noqa: E402
from mrgpu import corpus as C  # noqa: E402


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    files = C.c1_files(1)
    man = {"generator": "mrgpu.corpus.c1_files(seed=1)", "sizes": [len(f) for f in files],
           "files": [sha(f) for f in files],
           "mr_out_0": sha(O.c_mrsequential("wc", files)),
           "mr_out_r10": [sha(p) for p in O.c_partitioned("wc", files, 10)]}
    with open(os.path.join(HERE, "c1_manifest.json"), "w") as f:
        json.dump(man, f, indent=1)
    print("wrote c1_manifest.json")


if __name__ == "__main__":
    main()
