"""The coordinator-driven mode (build/mrcoord_gpu):
task handout restating mr/coordinator.go:43-114 over the rpc.go fields.

CPU tests drive the real coordinator binary with protocol-level fake workers
(no GPU): map tasks first, reduce tasks only after every map task completed,
status 2 while tasks are in flight, re-issue of a task held past the timeout
(coordinator.go:70-77), completions counted once per task, status 3 and exit
when every reduce task is done.  The GPU worker processes run in the -m gpu
tests below (P = 2 workers on one GPU, output byte-exact vs the oracle).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import subprocess
import time

import pytest

import _oracle as O
import cases
from mrgpu import corpus as C
from mrgpu.lib import BUILD_DIR

MAGIC = 0x4D52434F
REQ = struct.Struct("<IIq")        # magic, method, TaskNumber
REP = struct.Struct("<IiiiiiI")    # magic, TaskStatus, NMap, CMap, NReduce, CReduce, len(Filename)
REQUEST, MAP_DONE, REDUCE_DONE = 1, 2, 3
MAP, REDUCE, WAIT, DONE = 0, 1, 2, 3
COORD = os.path.join(BUILD_DIR, "mrcoord_gpu")


def call(sock: str, method: int, task: int = 0):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(sock)
    s.sendall(REQ.pack(MAGIC, method, task))
    buf = b""
    while len(buf) < REP.size:
        chunk = s.recv(REP.size - len(buf))
        assert chunk
        buf += chunk
    magic, status, nmap, cmap, nreduce, creduce, fl = REP.unpack(buf)
    name = b""
    while len(name) < fl:
        name += s.recv(fl - len(name))
    s.close()
    assert magic == MAGIC
    return status, nmap, cmap, nreduce, creduce, name.decode()


def start(tmp_path, files, R, timeout_s="1"):
    if not os.path.exists(COORD):
        pytest.skip("mrcoord_gpu not built")
    sock = str(tmp_path / "coord.sock")
    p = subprocess.Popen([COORD, "-n", str(R), "-w", "0", "--sock", sock, "--task-timeout", timeout_s, "wc"]
                         + [str(f) for f in files], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    for _ in range(200):
        if os.path.exists(sock):
            break
        time.sleep(0.01)
    return p, sock


def test_handout_order_wait_reissue_and_done(tmp_path):
    files = [tmp_path / f"pg-{i}.txt" for i in range(3)]
    for f in files:
        f.write_bytes(b"x\n")
    p, sock = start(tmp_path, files, 2, "1")
    try:
        got = [call(sock, REQUEST) for _ in range(3)]
        assert [g[0] for g in got] == [MAP] * 3 and [g[2] for g in got] == [0, 1, 2]
        assert [g[5] for g in got] == [str(f) for f in files] and all(g[3] == 2 for g in got)
        assert call(sock, REQUEST)[0] == WAIT            # every map task in progress
        assert call(sock, MAP_DONE, 0)[2] == 1           # completion accepted: CMap = 1
        assert call(sock, MAP_DONE, 0)[2] == 0           # a duplicate completion counts once, not accepted
        call(sock, MAP_DONE, 1)
        assert call(sock, REQUEST)[0] == WAIT            # map 2 not completed: no reduce task yet
        time.sleep(1.3)                                  # map 2 held past the timeout -> untouched again
        st = call(sock, REQUEST)
        assert st[0] == MAP and st[2] == 2
        call(sock, MAP_DONE, 2)
        r0, r1 = call(sock, REQUEST), call(sock, REQUEST)
        assert (r0[0], r0[4], r1[0], r1[4]) == (REDUCE, 0, REDUCE, 1) and r0[1] == 3
        assert call(sock, REQUEST)[0] == WAIT
        # a client that connects and never sends must not stall the coordinator
        # (accepted sockets time out after 0.5 s)
        idle = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        idle.connect(sock)
        t0 = time.time()
        assert call(sock, REDUCE_DONE, 1)[4] == 1        # accepted: the worker may remove its inputs
        assert call(sock, REDUCE_DONE, 1)[4] == 0        # a late duplicate: it must not
        assert time.time() - t0 < 3
        idle.close()
        call(sock, REDUCE_DONE, 0)
        assert call(sock, REQUEST)[0] == DONE
        out, err = p.communicate(timeout=10)
        assert p.returncode == 0, err
        info = json.loads(out.decode().strip().splitlines()[-1])
        assert info["reissued"] == 1 and info["nmap"] == 3 and info["nreduce"] == 2 and info["done"]
    finally:
        if p.poll() is None:
            p.kill()


# ---------------------------------------------------------------- GPU workers
def _write(tmp_path, files):
    paths = []
    for i, f in enumerate(files):
        q = tmp_path / f"pg-{i}.txt"
        q.write_bytes(f)
        paths.append(str(q))
    return paths


@pytest.mark.gpu
@pytest.mark.parametrize("app,fmt", [("wc", "mrgi"), ("wc", "json"), ("grep:distributed", "mrgi")])
def test_coordinator_two_gpu_workers(tmp_path, app, fmt):
    """mrcoord_gpu -w 2: two worker processes on one GPU pull map and reduce
    tasks; mr-out-* must equal the oracle, and test-mr.sh's check must hold."""
    if app == "wc":
        files = cases.synthetic(C.KIND_UTF8, 20000, [300_000, 200_000, 250_000, 1_000, 90_000], 61, 0.001)
    else:
        files = cases.synthetic_grep(20000, [300_000, 200_000, 150_000], 62, match_rate=0.03)
    paths = _write(tmp_path, files)
    R = 10
    args = [COORD, "-n", str(R), "-w", "2", "--sock", str(tmp_path / "s")] + (["--json"] if fmt == "json" else [])
    r = subprocess.run(args + [app] + paths, cwd=tmp_path, capture_output=True, timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    parts = [(tmp_path / f"mr-out-{k}").read_bytes() for k in range(R)]
    assert parts == O.c_partitioned(app, files, R)
    assert not list(tmp_path.glob("mr-[0-9]*-[0-9]*"))  # intermediates removed (worker.go:150-154)


@pytest.mark.gpu
def test_coordinator_reissues_a_crashed_workers_task(tmp_path):
    """A worker dies holding a task (no completion RPC); after the re-issue
    timeout the coordinator hands the task to the surviving worker
    (coordinator.go:70-77) and the output is still exact."""
    files = cases.synthetic(C.KIND_ASCII, 5000, [200_000, 150_000, 100_000, 120_000], 63)
    paths = _write(tmp_path, files)
    sock = str(tmp_path / "s")
    coord = subprocess.Popen([COORD, "-n", "4", "-w", "0", "--sock", sock, "--task-timeout", "2", "wc"] + paths,
                             cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    for _ in range(300):
        if os.path.exists(sock):
            break
        time.sleep(0.01)
    wk = os.path.join(BUILD_DIR, "mrworker_gpu")
    env = dict(os.environ, MRG_WORKER_CRASH_AFTER="1")
    bad = subprocess.run([wk, "--sock", sock, "wc"], cwd=tmp_path, env=env, capture_output=True, timeout=120)
    assert bad.returncode == 3  # took one task, completed it, died holding the second
    good = subprocess.run([wk, "--sock", sock, "wc"], cwd=tmp_path, capture_output=True, timeout=180)
    assert good.returncode == 0, good.stderr.decode()[-2000:]
    out, err = coord.communicate(timeout=30)
    assert coord.returncode == 0, err.decode()
    assert json.loads(out.decode().strip().splitlines()[-1])["reissued"] >= 1
    assert [(tmp_path / f"mr-out-{k}").read_bytes() for k in range(4)] == O.c_partitioned("wc", files, 4)


@pytest.mark.gpu
def test_coordinator_forked_worker_crash_still_succeeds(tmp_path):
    """-w 2 with forked worker 0 dying while it holds its second task: the task
    is re-issued to worker 1 (coordinator.go:70-77); the job's status follows
    Done(), so it exits 0 and reports the crash as information."""
    # (16 map and 8 reduce tasks: with 4 + 4, worker 1 sometimes finished every
    # task before worker 0 asked for its second, and nothing crashed)
    files = cases.synthetic(C.KIND_ASCII, 5000, [200_000, 150_000, 100_000, 120_000] * 4, 64)
    paths = _write(tmp_path, files)
    env = dict(os.environ, MRG_WORKER_CRASH_AFTER="1", MRG_WORKER_CRASH_INDEX="0")
    r = subprocess.run([COORD, "-n", "8", "-w", "2", "--sock", str(tmp_path / "s"), "--task-timeout", "2", "wc"]
                       + paths, cwd=tmp_path, env=env, capture_output=True, timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    info = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert info["done"] and info["workers_failed"] == 1 and info["reissued"] >= 1
    assert [(tmp_path / f"mr-out-{k}").read_bytes() for k in range(8)] == O.c_partitioned("wc", files, 8)
    assert not list(tmp_path.glob("mr-*.tmp-*"))  # unique temp files, all renamed


@pytest.mark.gpu
def test_worker_fails_on_unreadable_reduce_input(tmp_path):
    """A reduce input that exists but cannot be read (here a directory: EISDIR
    even for root) is a fatal worker error (log.Fatalf, worker.go:60-64), not a
    task abandoned as 'removed by a duplicate' — abandoning it made the
    coordinator re-issue the task forever.  Only a missing input
    (ENOENT) abandons the task."""
    files = cases.synthetic(C.KIND_ASCII, 5000, [200_000], 65)
    paths = _write(tmp_path, files)
    sock = str(tmp_path / "s")
    coord = subprocess.Popen([COORD, "-n", "2", "-w", "0", "--sock", sock, "--task-timeout", "2", "wc"] + paths,
                             cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        for _ in range(300):
            if os.path.exists(sock):
                break
            time.sleep(0.01)
        wk = os.path.join(BUILD_DIR, "mrworker_gpu")
        env = dict(os.environ, MRG_WORKER_CRASH_AFTER="1")
        first = subprocess.run([wk, "--sock", sock, "wc"], cwd=tmp_path, env=env, capture_output=True, timeout=120)
        assert first.returncode == 3  # did the map task, died holding a reduce task
        inter = tmp_path / "mr-0-0"
        assert inter.exists()
        inter.unlink()
        inter.mkdir()  # opens, but every read fails
        bad = subprocess.run([wk, "--sock", sock, "wc"], cwd=tmp_path, capture_output=True, timeout=120)
        assert bad.returncode != 0
        assert b"cannot read" in bad.stderr and b"mr-0-0" in bad.stderr
    finally:
        coord.kill()
        coord.communicate(timeout=30)
