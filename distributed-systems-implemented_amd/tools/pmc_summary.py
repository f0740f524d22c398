"""Summarize rocprofv3 --pmc CSVs per kernel (sum over dimensions per dispatch,
then mean over dispatches of the same kernel).

usage: python tools/pmc_summary.py [--each] <dir with *_counter_collection.csv> [kernel-substring ...]
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads (MI355X_MICROARCH.md §HBM), so `hbm_read_bytes_x2`
doubles it.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, separate=False):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f, r["Dispatch_Id"])
            names[key] = r["Kernel_Name"].split("(")[0]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = collections.Counter()
    for key in sorted(per, key=lambda k: (k[0], int(k[1]))):
        nm = names[key]
        if separate:
            nm = f"{nm}#{seen[nm]}"
            seen[names[key]] += 1
        for c, v in per[key].items():
            out[nm][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def main():
    args = sys.argv[1:]
    separate = "--each" in args  # one entry per dispatch (name#k) instead of the mean per kernel name
    args = [a for a in args if a != "--each"]
    d = args[0]
    want = args[1:] or ["wc_map_kernel", "wc_agg_kernel"]
    res = {}
    for k, cs in load(d, separate).items():
        if any(w in k for w in want):
            if "FETCH_SIZE" in cs:
                cs["hbm_read_bytes_x2"] = cs["FETCH_SIZE"] * 1024 * 2
            if "WRITE_SIZE" in cs:
                cs["hbm_write_bytes"] = cs["WRITE_SIZE"] * 1024
            res[k] = cs
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
