"""C1 (BASELINE.json configs[0]): main/mrsequential.go + mrapps/wc on the
Gutenberg texts, CPU only — plumbing, no GPU.

The reference's pg-*.txt are not bundled (.gitignore:36), so the
input is the committed-by-seed substitute mrgpu.corpus.c1_files() (8 files of
0.1-0.6 MB English-like prose with CRLF line ends, punctuation, quotes,
apostrophes, hyphens and digits), pinned by tests/golden/c1_manifest.json.

* oracle/_build/mrseq (the single-process restatement of mrsequential.go) and
  oracle/_build/mrcpu (coordinator + 3 worker processes, nReduce = 10, the
  test-mr.sh layout) must pass the reference's own check
  (main/test-mr.sh:30-31,52-53): `sort mr-out* | grep .` == `sort mr-out-0`;
* their outputs are pinned by the manifest;
* the pure-Python restatement agrees on the first files.
The GPU hosts run the same corpus in tests/test_hosts.py.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess

import pytest

import _oracle as O
from mrgpu import corpus as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAN = json.load(open(os.path.join(ROOT, "tests", "golden", "c1_manifest.json")))


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def c1_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("c1")
    files = C.c1_files(1)
    paths = []
    for i, f in enumerate(files):
        p = d / f"pg-{i}.txt"
        p.write_bytes(f)
        paths.append(str(p))
    return d, files, paths


def test_c1_corpus_pinned(c1_dir):
    _, files, _ = c1_dir
    assert [len(f) for f in files] == MAN["sizes"] == C.C1_SIZES
    assert [sha(f) for f in files] == MAN["files"]
    for f in files:
        f.decode("ascii")
        assert f.endswith(b"\r\n") and b"\r\n\r\n" in f and b"CHAPTER" in f
        assert any(ch in f for ch in (b"'", b'"', b"-", b",", b";")) and any(bytes([d]) in f for d in b"0123456789")


def test_c1_mrsequential_vs_distributed_cpu(c1_dir):
    """The reference's test-mr.sh on the CPU restatements (no GPU)."""
    d, files, paths = c1_dir
    O.build_oracle()
    seq = d / "seq"
    job = d / "job"
    seq.mkdir(exist_ok=True)
    job.mkdir(exist_ok=True)
    subprocess.run([os.path.join(ROOT, "oracle", "_build", "mrseq"), "--app", "wc"] + paths, cwd=seq, check=True,
                   capture_output=True, timeout=300)
    subprocess.run([os.path.join(ROOT, "oracle", "_build", "mrcpu"), "--app", "wc", "--nreduce", "10", "--workers", "3",
                    "--dir", str(job)] + paths, check=True, capture_output=True, timeout=300)
    out0 = (seq / "mr-out-0").read_bytes()
    parts = [(job / f"mr-out-{r}").read_bytes() for r in range(10)]
    assert sha(out0) == MAN["mr_out_0"]
    assert [sha(p) for p in parts] == MAN["mr_out_r10"]
    lines = sorted(l for p in parts for l in p.split(b"\n") if l)  # sort mr-out* | grep .
    assert lines == sorted(l for l in out0.split(b"\n") if l)
    assert out0 == O.c_mrsequential("wc", files)
    assert len(list(job.glob("mr-*-*"))) == 10  # intermediates removed (worker.go:151-154): only mr-out-*


def test_c1_python_restatement_agrees(c1_dir):
    _, files, _ = c1_dir
    sub = files[:2]
    assert O.mr_oracle.mrsequential("wc", sub) == O.c_mrsequential("wc", sub)
    assert O.mr_oracle.mr_partitioned("wc", sub, 10) == O.c_partitioned("wc", sub, 10)
