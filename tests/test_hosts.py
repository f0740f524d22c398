"""The reference's own end-to-end check (MapReduce/main/test-mr.sh:26-60) on the
C++ hosts: mrseq_gpu (mrsequential.go) produces mr-out-0; mrjob_gpu (worker map
tasks -> mr-X-Y intermediates -> reduce tasks) produces mr-out-*; then
`sort mr-out* | grep .` must equal `sort mr-out-0` — and, stricter, both must
equal the oracle byte for byte."""
from __future__ import annotations

import glob
import os
import subprocess

import pytest

import _oracle as O
import cases
from mrgpu import corpus as C
from mrgpu.lib import BUILD_DIR

pytestmark = pytest.mark.gpu


def _run(exe, args, cwd):
    subprocess.run([os.path.join(BUILD_DIR, exe)] + args, cwd=cwd, check=True, timeout=120)


@pytest.mark.parametrize("app", ["wc", "grep:distributed"])
def test_test_mr_sh_equivalent(tmp_path, app):
    if app == "wc":
        files = cases.synthetic(C.KIND_UTF8, 20000, [300_000, 500_000, 200_000, 1_000], 31, 0.001)
    else:
        files = cases.synthetic_grep(20000, [400_000, 300_000], 32, match_rate=0.03)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"pg-{i}.txt"
        p.write_bytes(f)
        paths.append(str(p))
    seq = tmp_path / "seq"
    job = tmp_path / "job"
    seq.mkdir()
    job.mkdir()
    _run("mrseq_gpu", [app] + paths, seq)
    _run("mrjob_gpu", ["-n", "10", app] + paths, job)
    out0 = (seq / "mr-out-0").read_bytes()
    assert out0 == O.c_mrsequential(app, files)
    parts = [(job / f"mr-out-{r}").read_bytes() for r in range(10)]
    assert parts == O.c_partitioned(app, files, 10)
    assert not glob.glob(str(job / "mr-*-*[0-9]")) or all("out" in g for g in glob.glob(str(job / "mr-*")))
    all_lines = sorted(l for p in parts for l in p.split(b"\n") if l)  # sort mr-out* | grep .
    assert all_lines == sorted(l for l in out0.split(b"\n") if l)


def test_c1_substitute_corpus_hosts(tmp_path):
    """C1's plumbing run on the GPU hosts: mrseq_gpu (mrsequential.go) and
    mrjob_gpu -n 10 on the pinned Gutenberg substitute (tests/test_c1.py),
    byte-exact against the oracle and against each other as test-mr.sh checks."""
    files = C.c1_files(1)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"pg-{i}.txt"
        p.write_bytes(f)
        paths.append(str(p))
    (tmp_path / "seq").mkdir()
    (tmp_path / "job").mkdir()
    _run("mrseq_gpu", ["wc"] + paths, tmp_path / "seq")
    _run("mrjob_gpu", ["-n", "10", "wc"] + paths, tmp_path / "job")
    out0 = (tmp_path / "seq" / "mr-out-0").read_bytes()
    assert out0 == O.c_mrsequential("wc", files)
    parts = [(tmp_path / "job" / f"mr-out-{r}").read_bytes() for r in range(10)]
    assert parts == O.c_partitioned("wc", files, 10)
    assert sorted(l for p in parts for l in p.split(b"\n") if l) == sorted(l for l in out0.split(b"\n") if l)
