"""Diagnostic: run the two-worker coordinator wc case and print the differing
lines against the oracle (tests/test_coordinator.py::test_coordinator_two_gpu_workers)."""
import os, subprocess, sys, tempfile
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _oracle as O
import cases
from mrgpu import corpus as C
from mrgpu.lib import BUILD_DIR

workers = int(sys.argv[1]) if len(sys.argv) > 1 else 2
files = cases.synthetic(C.KIND_UTF8, 20000, [300_000, 200_000, 250_000, 1_000, 90_000], 61, 0.001)
d = tempfile.mkdtemp()
paths = []
for i, f in enumerate(files):
    p = os.path.join(d, f"pg-{i}.txt")
    open(p, "wb").write(f)
    paths.append(p)
R = 10
r = subprocess.run([os.path.join(BUILD_DIR, "mrcoord_gpu"), "-n", str(R), "-w", str(workers), "--sock", os.path.join(d, "s"), "wc"] + paths,
                   cwd=d, capture_output=True, timeout=240)
print("rc", r.returncode, r.stderr.decode()[-500:])
want = O.c_partitioned("wc", files, R)
for k in range(R):
    got = open(os.path.join(d, f"mr-out-{k}"), "rb").read()
    if got != want[k]:
        g, w = set(got.split(b"\n")), set(want[k].split(b"\n"))
        print(k, "extra", sorted(g - w)[:8], "missing", sorted(w - g)[:8], len(g - w), len(w - g))
