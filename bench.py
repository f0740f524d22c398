#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on its configs[1] workload.

metric : word-count input GB/s (map+shuffle+reduce) at 1/2/4/8 MI355X; % HBM roofline
step   : one whole wc job over one GPU's input split, device-resident in HBM:
         map (tokenize + LDS combine + HBM hash aggregation) -> [RCCL all-to-all
         shuffle keyed by ihash % nReduce when N > 1] -> reduce (sort, format
         every mr-out-r) -> output bytes copied to host.
workload (configs[1] = SURVEY.md §8d C2): 10 GB synthetic Zipf(s=1.07, V=1e6)
         ASCII corpus (40 files x 250 MB) per GPU, nReduce = 10.  Weak scaling:
         every rank maps its own 10 GB (seed per rank); value = all ranks' input
         bytes x steps / max-over-ranks time.

Other §8d workloads (evidence runs; the default is C2):
  --workload c2u wc on 10 GB of mixed ASCII/UTF-8 Zipf text (north_star's mixed corpus: the
                 tokenizer's non-ASCII path), nReduce = 10
  --workload c3  grep "distributed" over 10 GB of valid mixed ASCII/UTF-8 lines
  --workload c4  wc, 12.5 GB per GPU, nReduce = 64 (the 8-GPU 100 GB config)
  --workload c5  wc, 25 GB per GPU, Zipf(s=0.8, V=1e7) with every vocabulary word
                 once up front (>= 1e7 distinct keys), nReduce = 64

Run:  python bench.py [--gpus N --steps K --warmup W]
      N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
             --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
      or plain `python bench.py --gpus N`: with no WORLD_SIZE in the environment
      it starts those N ranks itself, as a child torch.distributed.run (before
      any GPU call; the parent forwards rank 0's line and the child's exit code).
      N > 1 defaults to C4 (12.5 GB per GPU, nReduce = 64, the 8-GPU 100 GB
      config) with the C5 weak-scaling sub-run (E(P) at 25 GB per GPU).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-systems-implemented_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before mrgpu: one shared HIP runtime)
import torch.distributed as dist  # noqa: E402

from mrgpu import MRG_APP_GREP, MRG_APP_WC, Context, ihash  # noqa: E402
from mrgpu import corpus as C  # noqa: E402

METRIC = "word-count input GB/s (map+shuffle+reduce) at 1/2/4/8 MI355X; % HBM roofline"
GREP_METRIC = "grep input GB/s (map+shuffle+reduce) at 1/2/4/8 MI355X; % HBM roofline"

# SURVEY.md §8d workloads: app, corpus kind, Zipf s, vocabulary V, seed, files x MB, nReduce
WORKLOADS = {
    "c2": dict(app="wc", kind=C.KIND_ASCII, s=1.07, V=10**6, seed=2, files=40, file_mb=250, nreduce=10,
               desc="C2: wc, Zipf s=1.07 over 1e6 ASCII words"),
    "c2u": dict(app="wc", kind=C.KIND_UTF8, s=1.07, V=10**6, seed=6, files=40, file_mb=250, nreduce=10,
                desc="C2u: wc, Zipf s=1.07 over 1e6 mixed-script words (~30 % non-ASCII: Greek, Cyrillic, CJK, "
                     "Deseret, CJK ext. B), valid UTF-8"),
    "c3": dict(app="grep", kind=C.KIND_UTF8, s=1.07, V=10**6, seed=3, files=40, file_mb=250, nreduce=10,
               desc="C3: grep 'distributed' (0.5 % of lines, 20 % of those repeated), valid UTF-8, "
                    "~30 % non-ASCII words, lines 40-120 B"),
    "c4": dict(app="wc", kind=C.KIND_ASCII, s=1.07, V=10**6, seed=4, files=50, file_mb=250, nreduce=64,
               desc="C4: wc, Zipf s=1.07 over 1e6 ASCII words, 12.5 GB per GPU"),
    "c5": dict(app="wc", kind=C.KIND_ASCII, s=0.8, V=10**7, seed=5, files=100, file_mb=250, nreduce=64,
               desc="C5: wc, Zipf s=0.8 over 1e7 ASCII words, every word once up front"),
}
PATTERN = b"distributed"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0  # measured copy bandwidth (secondary reference)
XGMI_LINK_GBS = 153.0  # per xGMI link (7 links x ~153 GB/s per GPU)


def host_threads() -> int:
    """Host threads per rank for generation and the oracle checks: the box's
    cores split over the ranks of this node (8 ranks x 16 threads would
    oversubscribe a node whose ranks all generate and check at once)."""
    per_node = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return max(1, min(16, (os.cpu_count() or 1) // max(1, per_node)))


def self_launch(argv: list[str], n: int) -> int:
    """`bench.py --gpus N` (N > 1) with no launcher around it: run the N ranks
    as a child `torch.distributed.run` on 127.0.0.1 and return its exit code.
    A child, never an exec: this process must not replace itself (nothing here
    has touched the GPU yet, but the rule is kept everywhere).  The ranks inherit
    stdout, so rank 0's JSON line is this command's line."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    log(f"--gpus {n} without WORLD_SIZE: starting {n} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


class Wall:
    """Wall seconds of the run's host-side phases (generation, upload, timed
    steps, checks, sub-runs), reported in the line: the N = 8 run must fit the
    driver's time limit (DESIGN.md §7 budget)."""

    def __init__(self):
        self.t0 = time.time()
        self.phases: dict[str, float] = {}

    def add(self, name: str, t_start: float):
        self.phases[name] = round(self.phases.get(name, 0.0) + time.time() - t_start, 1)

    def as_dict(self):
        return {**self.phases, "total": round(time.time() - self.t0, 1)}


def log(msg):
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


class heartbeat:
    """A progress line every `every` s while a long host-side step runs (the
    full-size oracle check of C5 takes minutes; a silent GPU box command is
    taken to be hung)."""

    def __init__(self, what: str, every: float = 30.0):
        import threading
        self.what, self.every, self.stop = what, every, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(self.every):
            log(f"{self.what}: {time.time() - t0:.0f} s")

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()


def file_params(w: dict, i: int, nfiles: int):
    if w["app"] == "grep":
        return C.grep_params(PATTERN)
    if w["V"] > 10**6:  # C5: file i emits its share of the vocabulary once, up front
        return C.wc_params(vocab_lo=w["V"] * i // nfiles, vocab_hi=w["V"] * (i + 1) // nfiles)
    return C.wc_params()


def file_seed(w: dict, rank: int, split: int, i: int) -> int:
    """Seed of file i of split `split` on `rank`: every (rank, split) is a distinct
    input (split 0 keeps the seeds of earlier rounds' single-split bench lines)."""
    return w["seed"] + 1000 * rank + 100_000 * split + i


def gen_corpus(w: dict, rank: int, file_mb: int, nfiles: int, split: int = 0):
    """nfiles generated files back to back in one buffer.  Every file ends with '\n',
    so the concatenation is word-for-word the same input as separate splits."""
    voc = C.Vocab(w["kind"], w["s"], w["V"], w["seed"])
    buf = np.empty(nfiles * file_mb * 1_000_000, dtype=np.uint8)
    sz = file_mb * 1_000_000
    uniform = w["app"] == "grep" or w["V"] <= 10**6
    if uniform:
        seeds = [file_seed(w, rank, split, i) for i in range(nfiles)]
        voc.fill_files([sz] * nfiles, seeds, file_params(w, 0, nfiles), threads=host_threads(), out=buf)
    else:
        from concurrent.futures import ThreadPoolExecutor  # the C generator releases the GIL

        def one(i):
            voc.fill_files([sz], [file_seed(w, rank, split, i)], file_params(w, i, nfiles), threads=1,
                           out=buf[i * sz:(i + 1) * sz])
        with ThreadPoolExecutor(host_threads()) as ex:
            list(ex.map(one, range(nfiles)))
    return buf


def check_output(parts: list[bytes], nreduce: int, app: str = "wc", sample: int = 20000) -> dict:
    """Size-independent properties of the full-size output: every partition sorted
    bytewise with unique keys, every sampled key in the right partition; wc: counts
    sum to the word total; grep: every line is "L L" and L holds the pattern."""
    ok_sorted = ok_part = ok_form = True
    total = 0
    rng = np.random.default_rng(0)
    for r, p in enumerate(parts):
        lines = p.split(b"\n")[:-1] if p else []
        if app == "grep":
            keys = [l[:(len(l) - 1) // 2] for l in lines]
            total += len(lines)
            for i in rng.integers(0, len(keys), size=min(sample // nreduce, len(keys))) if keys else []:
                l, k = lines[i], keys[i]
                if len(l) % 2 == 0 or l != k + b" " + k or PATTERN not in k:
                    ok_form = False
        else:
            keys = [l.rsplit(b" ", 1)[0] for l in lines]
            total += sum(int(l.rsplit(b" ", 1)[1]) for l in lines)
        if any(keys[i] >= keys[i + 1] for i in range(len(keys) - 1)):
            ok_sorted = False
        if keys:
            for i in rng.integers(0, len(keys), size=min(sample // nreduce, len(keys))):
                if ihash(keys[i]) % nreduce != r:
                    ok_part = False
    out = {"sorted_unique": ok_sorted, "partition_ok": ok_part}
    if app == "grep":
        out.update(lines_format_ok=ok_form, matching_lines=total)
    else:
        out["total_words"] = total
    return out


def ascii_word_count(dev) -> int | None:
    """Independent word count of a device-resident ASCII split with plain torch
    ops (no libmrgpu code): Go's FieldsFunc(!IsLetter) words in ASCII text are
    the maximal runs of [A-Za-z].  None when the split holds a byte >= 0x80."""
    total, prev, step = 0, False, 1 << 30
    for off in range(0, dev.numel(), step):
        x = dev[off:off + step]
        if int(x.max()) >= 0x80:
            return None
        y = x | 32
        let = (y >= 97) & (y <= 122)
        total += int((let[1:] & ~let[:-1]).sum()) + int(bool(let[0]) and not prev)
        prev = bool(let[-1])
        del x, y, let
    return total


def _cpu_files(w: dict, sample_files: int, sample_mb: int, tmp: str):
    voc = C.Vocab(w["kind"], w["s"], w["V"], w["seed"])
    files, paths = [], []
    for i in range(sample_files):
        f = voc.fill_files([sample_mb * 1_000_000], [w["seed"] + i], file_params(w, i, w["files"]))[0]
        p = os.path.join(tmp, f"pg-{i}.txt")
        f.tofile(p)
        files.append(f)
        paths.append(p)
    return files, paths


def cpu_baseline(w: dict, sample_files: int, sample_mb: int, seq_files: int, nreduce: int, ctx: Context) -> dict | None:
    """The oracle's restatements of the reference on a bounded sample of the same
    workload, on this host's cores: oracle/_build/mrcpu = mrcoordinator + N mrworker
    processes (mr/coordinator.go, mr/worker.go: JSON-lines mr-X-Y shuffle, one
    write(2) per KV), and oracle/_build/mrseq = main/mrsequential.go (one process).
    The GPU's output is compared with mrcpu's on the same sample."""
    exe = os.path.join(ROOT, "oracle", "_build", "mrcpu")
    seq_exe = os.path.join(ROOT, "oracle", "_build", "mrseq")
    if not os.path.exists(exe):
        log("cpu_baseline skipped: oracle/_build/mrcpu not built")
        return None
    workers = min(16, os.cpu_count() or 1)
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = tempfile.mkdtemp(prefix="mrcpu-", dir=base)
    try:
        files, paths = _cpu_files(w, sample_files, sample_mb, tmp)
        wdir = os.path.join(tmp, "work")
        os.makedirs(wdir)
        app_args = ["--app", "grep", "--pattern", PATTERN.decode()] if w["app"] == "grep" else ["--app", "wc"]
        res = subprocess.run([exe] + app_args + ["--nreduce", str(nreduce), "--workers", str(workers), "--dir", wdir]
                             + paths, capture_output=True, text=True, timeout=900)
        if res.returncode != 0:
            log(f"mrcpu failed: {res.stderr[-500:]}")
            return None
        info = json.loads(res.stdout.strip().splitlines()[-1])
        cpu_out = [open(os.path.join(wdir, f"mr-out-{r}"), "rb").read() for r in range(nreduce)]
        joined = b"\n".join(bytes(f) for f in files)
        if w["app"] == "grep":
            gpu_out = ctx.run_job(MRG_APP_GREP, joined, pattern=PATTERN, nreduce=nreduce)
        else:
            gpu_out = ctx.run_job(MRG_APP_WC, joined, nreduce=nreduce)
        out = {"value": round(info["bytes"] / info["seconds"] / 1e9, 4), "unit": "GB/s", "cores": workers,
               "kind": "port",
               "sample": f"{sample_files} files x {sample_mb} MB of the same corpus generator "
                         f"({info['bytes'] / 1e9:.2f} GB); oracle/_build/mrcpu = restated mrcoordinator + {workers} "
                         f"mrworker processes, JSON-lines mr-X-Y shuffle with one write(2) per KV as "
                         f"worker.go:84-89, nReduce={nreduce}; {info['seconds']:.1f} s",
               "gpu_output_identical": gpu_out == cpu_out}
        if os.path.exists(seq_exe) and seq_files > 0:
            sdir = os.path.join(tmp, "seq")
            os.makedirs(sdir)
            r2 = subprocess.run([seq_exe] + app_args + ["--out", os.path.join(sdir, "mr-out-0")] + paths[:seq_files],
                                capture_output=True, text=True, timeout=900)
            if r2.returncode == 0:
                si = json.loads(r2.stdout.strip().splitlines()[-1])
                out["mrseq"] = {"value": round(si["bytes"] / si["seconds"] / 1e9, 4), "unit": "GB/s", "cores": 1,
                                "sample": f"{seq_files} x {sample_mb} MB; oracle/_build/mrseq = restated "
                                          f"main/mrsequential.go (one process, every KV resident, one sort, one "
                                          f"write(2) per key); {si['seconds']:.1f} s"}
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _oracle():
    """The C oracle (tests/_oracle.py -> oracle/_build/liboracle.so): the checker
    of the full-size output, used outside the timed region only."""
    tdir = os.path.join(ROOT, "tests")
    if tdir not in sys.path:
        sys.path.insert(0, tdir)
    import _oracle as O
    return O


def oracle_exact_check(w: dict, host: np.ndarray, gpu_parts: list[bytes], nreduce: int, rank: int, world: int,
                       local_reduce: bool = False) -> dict:
    """Byte equality of every mr-out-r of the full-size job with the C oracle's
    (oracle/mrcount.c: the reference's wc / grep job restated, counted by host
    threads over the same split; main/mrsequential.go:59-84, mrapps/wc.go:21-34,
    mrapps/dgrep.go:18-46).  N > 1: every rank counts its own split, the
    partitions travel to their owners (r % N) over gloo and are merged there
    (the reduce over all splits' intermediates, worker.go:123-146), and each
    owner compares its partitions; non-owned partitions must be empty.
    local_reduce (a rehearsal: ranks share a device, no exchange, every rank
    reduced all partitions of its own split): each rank against its own count."""
    O = _oracle()
    app = "wc" if w["app"] == "wc" else "grep:" + PATTERN.decode()
    threads = host_threads()
    t0 = time.time()
    mine = O.c_count_mt(app, host, nreduce, threads)
    own = (lambda r: True) if local_reduce or world == 1 else (lambda r: r % world == rank)
    if world > 1 and not local_reduce:
        from mrgpu import dist as D
        send = []
        for o in range(world):
            blob = b"".join(len(mine[r]).to_bytes(8, "little") + mine[r] if r % world == o else (0).to_bytes(8, "little")
                            for r in range(nreduce))
            send.append(blob)
        recv = D.alltoallv_bytes(send)
        outs = []
        for b in recv:
            parts, off = [], 0
            for r in range(nreduce):
                n = int.from_bytes(b[off:off + 8], "little")
                parts.append(b[off + 8:off + 8 + n])
                off += 8 + n
            outs.append(parts)
        want = O.c_merge_parts(app, outs)
    else:
        want = mine
    bad = [r for r in range(nreduce) if gpu_parts[r] != (want[r] if own(r) else b"")]
    ok = not bad
    res = {"exact_vs_oracle": ok, "oracle_s": round(time.time() - t0, 1), "oracle_threads": threads,
           "oracle_output_bytes": sum(len(want[r]) for r in range(nreduce) if own(r))}
    if bad:
        res["mismatched_partitions"] = bad[:16]
    if world > 1:
        t = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(t)
        res["exact_vs_oracle"] = int(t.item()) == 0
        res["exact_vs_oracle_rank_failures"] = int(t.item())
    return res


def upload(host: np.ndarray, local: int):
    """The split, resident in HBM before the timed region (a torch tensor: the
    independent word count reads it with plain torch ops)."""
    nbytes = int(host.size)
    dev = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{local}")
    step = 1 << 30
    for off in range(0, nbytes, step):
        n = min(step, nbytes - off)
        dev[off:off + n].copy_(torch.from_numpy(host[off:off + n]))
    torch.cuda.synchronize()
    return dev


def download(dev) -> np.ndarray:
    """A resident split back to host memory (the oracle check reads it there; the
    host copies are not kept while several splits are resident)."""
    return dev.cpu().numpy()


def timed_steps(ctx: Context, run_step, steps: int, warmup: int, world: int, nsplits: int = 1):
    """W untimed warmup steps (the first one's wall time is reported as the cold
    split: fresh dictionary, first allocations), then exactly K steps between a
    barrier + synchronize on both sides; step i maps resident split i % nsplits
    (run_step(split)), so every timed step meets a split other than the one the
    context's kept state (dictionary, spill layout, segment capacities) came
    from, as a worker's next map task does.  Returns (max-over-ranks seconds,
    per-step stats, cold ms, cold stats)."""
    cold_ms, cold_st = None, None
    for i in range(warmup):
        ctx.sync()
        t0 = time.perf_counter()
        run_step(i % nsplits)
        ctx.sync()
        if i == 0:
            cold_ms = (time.perf_counter() - t0) * 1e3
            cold_st = ctx.stats()
    stats = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.sync()
    t_start = time.perf_counter()
    for i in range(steps):
        run_step((warmup + i) % nsplits)
        stats.append(ctx.stats())
    ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    t_max = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
    return t_max, stats, cold_ms, cold_st


def no_shuffle_time(ctx: Context, run_step, steps: int, shared: bool, nsplits: int = 1) -> float:
    """T(1) of the weak-scaling efficiency: the same per-GPU splits with no
    shuffle (every partition reduced locally), in this process; max over ranks."""
    ctx.set_option("skip_exchange", 1)
    dist.barrier()
    ctx.sync()
    t1 = time.perf_counter()
    for i in range(steps):
        run_step(i % nsplits)
    ctx.sync()
    t1 = time.perf_counter() - t1
    dist.barrier()
    ctx.set_option("skip_exchange", 1 if shared else 0)
    v = torch.tensor([t1], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


def multi_fields(stats: list[dict], t_max: float, t1: float, world: int, shared: bool, ndev: int) -> dict:
    def mean(k):
        return sum(st[k] for st in stats) / len(stats)
    ex_ms, a2a_ms, unp_ms = mean("exchange_ms"), mean("exchange_a2a_ms"), mean("exchange_unpack_ms")
    snd = mean("shuffle_send_bytes")
    v = torch.tensor([ex_ms, a2a_ms, unp_ms, snd], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    ex_max, a2a_max, unp_max, snd_max = (float(x) for x in v)
    # what RCCL itself saw, and each rank's device (gathered to every rank)
    me = {"rank": int(os.environ.get("RANK", "0")), "rccl_nranks": int(stats[-1]["rccl_nranks"]),
          "rccl_rank": int(stats[-1]["rccl_rank"]), "device": int(stats[-1]["device"]),
          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    links = min(world - 1, 7)
    # the xGMI rate is taken over the all-to-alls alone (the unpack and the
    # owner's re-aggregation are HBM work, reported separately)
    per_gpu_bw = snd / (a2a_ms / 1e3) / 1e9 if a2a_ms > 0 else 0.0
    m = {"exchange_ms": round(ex_max, 3), "exchange_a2a_ms": round(a2a_max, 3),
         "exchange_unpack_ms": round(unp_max, 3), "shuffle_bytes_per_gpu": int(snd_max),
         "rccl_nranks": sorted({r["rccl_nranks"] for r in ranks}), "ranks": ranks,
         "xgmi_achieved_GBps": round(per_gpu_bw, 2), "xgmi_peak_GBps": links * XGMI_LINK_GBS,
         "xgmi_frac": round(per_gpu_bw / (links * XGMI_LINK_GBS), 4),
         "t1_ms_per_step": round(t1 / len(stats) * 1e3, 3), "tP_ms_per_step": round(t_max / len(stats) * 1e3, 3),
         "weak_scaling_efficiency": round(t1 / t_max, 4)}
    if shared:
        m["rehearsal"] = f"{world} ranks shared {ndev} device(s): no RCCL exchange ran (not a measurement)"
    return m


def scaling_subrun(wname: str, args, rank: int, world: int, local: int, shared: bool, ndev: int) -> dict:
    """SURVEY.md §8(d) defines E(P) on C5 (25 GB per GPU, 1e7 distinct keys,
    R = 64): the same timed-step / T(1) measurement on that workload, in this
    run, after the headline workload's buffers are released (args.scaling_splits
    resident splits per rank, rotated as in the headline)."""
    w = WORKLOADS[wname]
    nsplits = max(1, args.scaling_splits)
    devs = []
    t0 = time.time()
    with heartbeat(f"[{wname}] generating the splits"):
        for sp in range(nsplits):
            host = gen_corpus(w, rank, w["file_mb"], args.scaling_files or w["files"], sp)
            devs.append(upload(host, local))
            del host
    nbytes = int(devs[0].numel())
    log(f"[{wname}] generated {nsplits} x {nbytes / 1e9:.2f} GB in {time.time() - t0:.1f} s")
    ctx = Context(local)
    for o in args.opt:
        k, v = o.split("=")
        ctx.set_option(k, int(v))
    if not shared:
        obj = [Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx.comm_init(obj[0], world, rank)
    else:
        ctx.set_option("skip_exchange", 1)
    dptrs = [d.data_ptr() for d in devs]

    def run_step(sp=0):
        return ctx.run_job(MRG_APP_WC, device_ptr=dptrs[sp], nbytes=nbytes, nreduce=w["nreduce"], copy_out=False)

    steps = max(1, args.scaling_steps)
    t_max, stats, _, _ = timed_steps(ctx, run_step, steps, 1, world, nsplits)
    p, n, offs = run_step(0)
    import ctypes
    out = ctypes.string_at(p, n) if n else b""
    parts = [out[offs[i]:offs[i + 1]] for i in range(w["nreduce"])]
    chk = check_output(parts, w["nreduce"], "wc")
    owned_ok = all(not parts[r] for r in range(w["nreduce"]) if r % world != rank) or shared
    # Σ counts over every owner's partitions = an independent count of every
    # rank's split 0 (plain torch ops on the resident input)
    indep = ascii_word_count(devs[0])
    tw = torch.tensor([chk["total_words"], -(1 << 40) if indep is None else indep], dtype=torch.int64)
    dist.all_reduce(tw)
    t1 = no_shuffle_time(ctx, run_step, steps, shared, nsplits)
    res = {"workload": f"{w['desc']}; {nbytes / 1e9:.2f} GB per GPU", "nreduce": w["nreduce"],
           "splits_per_gpu": nsplits,
           "value": round(nbytes * world * steps / t_max / 1e9, 3), "unit": "GB/s", "steps": steps,
           "ms_per_step": round(t_max / steps * 1e3, 3),
           **multi_fields(stats, t_max, t1, world, shared, ndev),
           "checks": {"sorted_unique": chk["sorted_unique"], "partition_ok": chk["partition_ok"],
                      "non_owned_empty": owned_ok, "total_words": int(tw[0]),
                      "total_words_match": int(tw[0]) == int(tw[1])}}
    ctx.close()
    del devs
    torch.cuda.empty_cache()
    return res


def group_rehearsal(args) -> dict:
    """The owner side of C5's weak-scaling shuffle at C5's key counts, on ONE GPU:
    P contexts (ranks) in this process, each mapping its own C5 split (Zipf s=0.8
    over 1e7 words, every vocabulary word once up front: >= 1e7 distinct keys per
    rank, the splits shrunk so P of them fit one device), R = 64, then
    mrg_exchange_group (the same count / pack / unpack / exact re-aggregation code
    as the RCCL path, with peer copies in place of ncclAllToAllv) and every owner's
    reduce (partitions r % P).  Checked byte for byte against the C oracle: each
    rank's split counted by oracle/mrcount.c, merged per partition (the reduce
    over every split's intermediates, worker.go:123-146).  Reports what E(P) must
    absorb on each owner: the unpack + re-aggregation of P ranks' records and the
    owner's reduce.  NOT an RCCL or xGMI measurement (no communicator exists)."""
    w = WORKLOADS["c5"]
    P, R = args.group_ranks, w["nreduce"]
    O = _oracle()
    threads = min(16, os.cpu_count() or 1)
    devs, want_parts = [], []
    t0 = time.time()
    with heartbeat("group rehearsal: splits + oracle counts"):
        for g in range(P):
            host = gen_corpus(w, g, args.group_file_mb, args.group_files, 0)
            devs.append(upload(host, 0))
            want_parts.append(O.c_count_mt("wc", host, R, threads))
            del host
    with heartbeat("group rehearsal: oracle merge"):
        want = O.c_merge_parts("wc", want_parts)
    del want_parts
    nbytes = [int(d.numel()) for d in devs]
    log(f"[group] {P} splits of {nbytes[0] / 1e9:.2f} GB + oracle in {time.time() - t0:.1f} s")
    ctxs = [Context(0) for _ in range(P)]
    steps = []
    outs = None
    try:
        for step in range(max(1, args.group_steps)):
            local = [ctxs[g].map(MRG_APP_WC, None, device_ptr=devs[g].data_ptr(), nbytes=nbytes[g], nreduce=R)
                     for g in range(P)]
            mst = [c.stats() for c in ctxs]
            torch.cuda.synchronize()
            te = time.perf_counter()
            owned = Context.exchange_group(ctxs, local)
            te = time.perf_counter() - te
            est = [c.stats() for c in ctxs]
            recv = [o.info()[0] for o in owned]
            outs, rst = [], []
            for g in range(P):
                outs.append(ctxs[g].reduce_all(owned[g]))
                rst.append(ctxs[g].stats())
            steps.append({
                "distinct_keys_per_rank": [int(s["distinct_keys"]) for s in mst],
                "map_kernel_ms": [round(s["map_kernel_ms"], 3) for s in mst],
                "map_total_ms": [round(s["map_total_ms"], 3) for s in mst],
                "keys_per_owner_after_reaggregation": [int(x) for x in recv],
                "records_received_per_owner": [int(s["shuffle_recv_records"]) for s in est],
                "exchange_unpack_ms": [round(s["exchange_unpack_ms"], 3) for s in est],
                "shuffle_send_bytes": [int(s["shuffle_send_bytes"]) for s in est],
                "owner_reduce_ms": [round(s["reduce_ms"], 3) for s in rst],
                "exchange_group_wall_ms": round(te * 1e3, 3)})
            for q in local + owned:
                q.free()
    finally:
        for c in ctxs:
            c.close()
    bad = [(g, r) for g in range(P) for r in range(R) if outs[g][r] != (want[r] if r % P == g else b"")]
    last = steps[-1]
    res = {"metric": "group rehearsal of the P-rank shuffle at C5 key counts (one GPU, peer copies; not RCCL)",
           "ranks": P, "nreduce": R, "split_bytes_per_rank": nbytes[0],
           "workload": f"{w['desc']}; {args.group_files} files x {args.group_file_mb} MB per rank (seed per rank)",
           "steps": len(steps),
           "min_distinct_keys_per_rank": min(last["distinct_keys_per_rank"]),
           "exchange_unpack_ms_max": max(last["exchange_unpack_ms"]),
           "exchange_unpack_ms_mean": round(sum(last["exchange_unpack_ms"]) / P, 3),
           "owner_reduce_ms_max": max(last["owner_reduce_ms"]),
           "owner_reduce_ms_mean": round(sum(last["owner_reduce_ms"]) / P, 3),
           "keys_per_owner_after_reaggregation": last["keys_per_owner_after_reaggregation"],
           "records_received_per_owner": last["records_received_per_owner"],
           "per_step": steps,
           "checks": {"exact_vs_oracle": not bad, "mismatched": bad[:16],
                      "oracle_output_bytes": sum(len(x) for x in want)},
           "note": "P contexts on one device drive mrg_exchange_group: owner counts, per-owner packing, peer "
                   "copies (where mrg_exchange calls ncclAllToAllv), unpack and exact re-aggregation on each owner "
                   "(exchange_unpack_ms, from the owner's own unpack start), then the owner's reduce of partitions "
                   "r % P.  No RCCL communicator exists here, so no xGMI rate or E(P) is measured: those need the "
                   "driver's 8-GPU node."}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="default: c2 (configs[1]) on one GPU, c4 (configs[3]: 12.5 GB per GPU, nReduce = 64) for N > 1")
    ap.add_argument("--file-mb", type=int, default=None, help="override the workload's file size (MB)")
    ap.add_argument("--files", type=int, default=None, help="override the workload's file count")
    ap.add_argument("--nreduce", type=int, default=None, help="override the workload's nReduce")
    ap.add_argument("--cpu-sample-files", type=int, default=16)
    ap.add_argument("--cpu-sample-mb", type=int, default=64)
    ap.add_argument("--cpu-seq-files", type=int, default=2, help="files of the sample the single-process mrseq times")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host-input) job")
    ap.add_argument("--no-oracle", action="store_true", help="skip the full-size exact check against the C oracle")
    ap.add_argument("--scaling-workload", default="c5", help="N > 1: workload of the E(P) sub-run ('none' to skip)")
    ap.add_argument("--scaling-steps", type=int, default=2)
    ap.add_argument("--scaling-files", type=int, default=None,
                    help="override the E(P) workload's file count (rehearsals: ranks sharing one device's HBM)")
    ap.add_argument("--no-pipelined", action="store_true", help="skip the pipelined-jobs measurement")
    ap.add_argument("--splits", type=int, default=0,
                    help="distinct splits resident per rank, rotated over the timed steps (0: 3 at N=1, 2 at N>1)")
    ap.add_argument("--scaling-splits", type=int, default=2, help="resident splits per rank in the E(P) sub-run")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices, no RCCL exchange: not a measurement)")
    ap.add_argument("--opt", action="append", default=[], help="library option name=value (experiments; repeatable)")
    ap.add_argument("--group-rehearsal", action="store_true",
                    help="one GPU: P contexts at C5 key counts through mrg_exchange_group (not RCCL; prints its own line)")
    ap.add_argument("--group-ranks", type=int, default=8)
    ap.add_argument("--group-files", type=int, default=100, help="C5 files per rank (all of them: every word once)")
    ap.add_argument("--group-file-mb", type=int, default=10)
    ap.add_argument("--group-steps", type=int, default=2)
    ap.add_argument("--dry-run", action="store_true",
                    help="resolve ranks, workload and sizes, print them from rank 0 and exit (no GPU call)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.group_rehearsal:
        sys.exit(self_launch(sys.argv[1:], args.gpus))
    if args.group_rehearsal:
        torch.zeros(1, device="cuda:0").add_(1)
        torch.cuda.synchronize()
        print(json.dumps(group_rehearsal(args)), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"--gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # N > 1: the headline is C4, the 8-GPU config (12.5 GB per GPU, R = 64:
    # 64 partitions spread evenly over 2, 4 or 8 owners); E(P) comes from the
    # C5 sub-run below
    args.workload = args.workload or ("c4" if world > 1 else "c2")
    w = WORKLOADS[args.workload]
    args.file_mb = args.file_mb or w["file_mb"]
    args.files = args.files or w["files"]
    args.nreduce = args.nreduce or w["nreduce"]
    grep = w["app"] == "grep"
    wall = Wall()
    if world > 1:
        import datetime
        # control plane only (the shuffle is RCCL inside libmrgpu); a lost rank
        # ends the job in minutes rather than gloo's default half hour
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
    if args.dry_run:
        info = {"rank": rank, "n_gpus": world, "workload": args.workload, "nreduce": args.nreduce,
                "input_bytes_per_gpu": args.files * args.file_mb * 1_000_000, "host_threads": host_threads(),
                "scaling_workload": args.scaling_workload if world > 1 else None}
        if world > 1:
            allinfo = [None] * world
            dist.all_gather_object(allinfo, info)
            info = {**info, "ranks": [i["rank"] for i in allinfo]}
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_run": True, **info}), flush=True)
        return
    # one GPU per rank; more ranks than devices only as an explicit rehearsal of
    # the N > 1 path on a smaller box (the driver's N-GPU runs have one each)
    ndev = max(1, torch.cuda.device_count())
    shared = world > ndev  # rehearsal: RCCL refuses two ranks on one device, so no exchange
    if shared and not args.rehearsal:
        log(f"{world} ranks but {ndev} visible GPU(s): refusing (pass --rehearsal to run without the RCCL exchange)")
        sys.exit(2)
    local = local % ndev
    torch.cuda.set_device(local)
    # torch initializes its CUDA runtime lazily on first use; do it now, so it can
    # never overlap a timed step (seen: one 57 ms map kernel in the first step)
    torch.zeros(1, device=f"cuda:{local}").add_(1)
    torch.cuda.synchronize()

    # S distinct splits resident in HBM (seeds per rank and split); the timed
    # steps rotate over them, so the context's kept state never meets the split
    # it was derived from.  The host copies are dropped after the upload (read
    # back for the oracle check) to keep host memory at one split per rank.
    nsplits = args.splits if args.splits > 0 else (3 if world == 1 else 2)
    t0 = time.time()
    devs = []
    with heartbeat("generating the splits"):
        for sp in range(nsplits):
            tg = time.time()
            host = gen_corpus(w, rank, args.file_mb, args.files, sp)
            wall.add("generate", tg)
            tg = time.time()
            devs.append(upload(host, local))
            wall.add("upload", tg)
            del host
    nbytes = int(devs[0].numel())
    log(f"generated {nsplits} x {nbytes / 1e9:.2f} GB in {time.time() - t0:.1f} s")

    ctx = Context(local)
    for o in args.opt:
        k, v = o.split("=")
        ctx.set_option(k, int(v))
    if world > 1 and not shared:
        obj = [Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx.comm_init(obj[0], world, rank)
    if shared:
        log(f"{world} ranks on {ndev} device(s): rehearsal without the RCCL exchange")
        ctx.set_option("skip_exchange", 1)
    dptrs = [d.data_ptr() for d in devs]
    ctx.sync()

    def run_step(sp=0):
        if grep:
            return ctx.run_job(MRG_APP_GREP, pattern=PATTERN, device_ptr=dptrs[sp], nbytes=nbytes,
                               nreduce=args.nreduce, copy_out=False)
        return ctx.run_job(MRG_APP_WC, device_ptr=dptrs[sp], nbytes=nbytes, nreduce=args.nreduce, copy_out=False)

    tg = time.time()
    t_max, stats, cold_ms, cold_st = timed_steps(ctx, run_step, args.steps, args.warmup, world, nsplits)
    wall.add("warmup_and_timed_steps", tg)
    kern_ms = [st["map_kernel_ms"] for st in stats]
    log("map kernel ms per timed step: " + " ".join(f"{k:.2f}" for k in kern_ms))
    log("aggregation ms per timed step: " + " ".join(f"{st['agg_ms']:.2f}" for st in stats))
    # the same K steps re-mapping ONE split (the rounds-1-3 measurement), for comparison
    same = None
    if nsplits > 1:
        t_same, st_same, _, _ = timed_steps(ctx, lambda sp: run_step(0), args.steps, 1, world, 1)
        same = {"value": round(nbytes * world * args.steps / t_same / 1e9, 3),
                "ms_per_step": round(t_same / args.steps * 1e3, 3),
                "map_kernel_ms": round(sum(x["map_kernel_ms"] for x in st_same) / len(st_same), 3),
                "agg_ms": round(sum(x["agg_ms"] for x in st_same) / len(st_same), 3),
                "dict_ms": round(sum(x["dict_ms"] for x in st_same) / len(st_same), 3)}

    # The output (grep C3: ~78 MB, C5: ~110 MB) crosses PCIe after the whole job:
    # the same K jobs pipelined two deep (mrg_run_job_async: each job's output
    # transfer overlaps the next job's map, as a worker's successive map tasks
    # can), reported beside the serial steps above (`value` stays serial)
    pipelined = None
    if not args.no_pipelined:
        def run_async(sp):
            if grep:
                ctx.run_job_async(MRG_APP_GREP, pattern=PATTERN, device_ptr=dptrs[sp], nbytes=nbytes,
                                  nreduce=args.nreduce)
            else:
                ctx.run_job_async(MRG_APP_WC, device_ptr=dptrs[sp], nbytes=nbytes, nreduce=args.nreduce)
        # untimed: both queue slots once (their pinned output buffers are allocated
        # on first use, ~10 ms per 100 MB)
        run_async(0)
        run_async(1 % nsplits)
        ctx.job_wait(copy_out=False)
        ctx.job_wait(copy_out=False)
        if world > 1:
            dist.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        run_async(0)
        d2h = []
        for i in range(1, args.steps):
            run_async(i % nsplits)
            ctx.job_wait(copy_out=False)
            d2h.append(ctx.stats()["d2h_ms"])
        ctx.job_wait(copy_out=False)
        d2h.append(ctx.stats()["d2h_ms"])
        ctx.sync()
        t_pipe = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([t_pipe], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t_pipe = float(tt.item())
        serial_ms = t_max / args.steps * 1e3
        pipe_ms = t_pipe / args.steps * 1e3
        d2h_ms = sum(st["d2h_ms"] for st in stats) / len(stats)
        pipelined = {"value": round(nbytes * world * args.steps / t_pipe / 1e9, 3), "ms_per_step": round(pipe_ms, 3),
                     "d2h_ms": round(sum(d2h) / len(d2h), 3),
                     "d2h_visible_ms": round(max(0.0, pipe_ms - (serial_ms - d2h_ms)), 3),
                     "note": "the same K jobs queued two deep with mrg_run_job_async / mrg_job_wait: a job's output "
                             "transfer (second stream, pinned buffer) overlaps the next job's map; d2h_visible_ms = "
                             "pipelined step - (serial step - serial d2h)"}

    # output of one more step per split (context-owned buffer) -> checks at full
    # size, outside the timed region: every resident split against the oracle
    import ctypes
    checks = {}
    per_split = []
    tchk = time.time()
    for sp in range(nsplits):
        p, n, offs = run_step(sp)
        out = ctypes.string_at(p, n) if n else b""
        parts = [out[offs[i]:offs[i + 1]] for i in range(args.nreduce)]
        with heartbeat(f"output checks of split {sp}"):
            ck = check_output(parts, args.nreduce, w["app"])
        if sp == 0:
            ck["deterministic"] = hashlib.sha256(out).hexdigest() == hashlib.sha256(
                ctypes.string_at(*run_step(0)[:2])).hexdigest()
        if not grep:
            # Σ counts of the output must equal an independent count of the input's words
            indep = ascii_word_count(devs[sp])
            ck["total_words_independent"] = indep
            ck["total_words_match"] = None if indep is None else indep == ck["total_words"]
        if world > 1:
            key = "matching_lines" if grep else "total_words"
            tw = torch.tensor([ck[key]], dtype=torch.int64)
            dist.all_reduce(tw)
            ck[key] = int(tw.item())
            if not grep and ck.get("total_words_independent") is not None:
                ti = torch.tensor([ck["total_words_independent"]], dtype=torch.int64)
                dist.all_reduce(ti)
                ck["total_words_independent"] = int(ti.item())
                ck["total_words_match"] = ck["total_words_independent"] == ck[key]
        if not args.no_oracle:
            with heartbeat(f"oracle check of split {sp}"):
                host = download(devs[sp])
                ck.update(oracle_exact_check(w, host, parts, args.nreduce, rank, world, local_reduce=shared))
            del host
        del out, parts
        per_split.append(ck)
    checks.update(per_split[0])
    for k in ("sorted_unique", "partition_ok", "total_words_match", "exact_vs_oracle", "lines_format_ok"):
        vals = [c.get(k) for c in per_split if c.get(k) is not None]
        if vals:
            checks[k] = all(vals)
    if nsplits > 1:
        checks["per_split"] = per_split
    wall.add("output_and_oracle_checks", tchk)

    # N > 1: the shuffle's share and the weak-scaling efficiency against the
    # same ranks running their splits with no shuffle (T(1) of the same per-GPU
    # work, measured in this process, every partition reduced locally)
    multi = None
    if world > 1:
        tg = time.time()
        t1 = no_shuffle_time(ctx, run_step, args.steps, shared, nsplits)
        wall.add("no_shuffle_steps", tg)
        multi = multi_fields(stats, t_max, t1, world, shared, ndev)
        multi["note"] = ("shuffle bytes = wire bytes a rank sends to the other ranks (max over ranks of the mean over "
                         "timed steps; 24-byte wire records + long-key bytes); xgmi_frac = those bytes / all-to-all time "
                         "(exchange_a2a_ms; exchange_ms adds the owner's unpack + exact re-aggregation) / "
                         "(min(P-1,7) x 153 GB/s); E(P) = T(1) / T(P), T(1) = the same per-GPU splits run with no "
                         "shuffle in this process")

    total_bytes = nbytes * world * args.steps
    value = total_bytes / t_max / 1e9
    avg_kern = sum(kern_ms) / len(kern_ms)
    # Map + partition (north_star's 50 % target): the map kernel, the dictionary
    # pass and the spill aggregation — every launch between the split and the
    # partitioned, aggregated records
    map_total_avg = sum(st["map_total_ms"] for st in stats) / len(stats)
    achieved = nbytes / (avg_kern / 1e3) / 1e9
    last = stats[-1]

    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("input_bytes") == nbytes and tj.get("workload", "c2") == args.workload:
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = (f"profiled, not this run: {os.path.relpath(tpath, ROOT)} (rocprofv3 --pmc FETCH_SIZE / "
                               f"WRITE_SIZE passes over the same launch, {tj.get('round', '?')})")
        except Exception:
            traffic = None

    # PCIe-inclusive rate (never `value`): one whole job with the split in pageable
    # host memory, so the H2D copy is inside the job (mrg_run_job, MRG_INPUT_HOST)
    pcie = None
    step = 1 << 30
    if world == 1 and not args.no_pcie:
        dev = devs[0]
        host = download(dev)
        ctx.sync()
        t0 = time.perf_counter()  # the copy alone (pageable host -> HBM), for comparison
        for off in range(0, nbytes, step):
            n = min(step, nbytes - off)
            dev[off:off + n].copy_(torch.from_numpy(host[off:off + n]))
        torch.cuda.synchronize()
        th2d = time.perf_counter() - t0
        ctx.sync()
        t0 = time.perf_counter()
        if grep:
            ctx.run_job(MRG_APP_GREP, host, pattern=PATTERN, nreduce=args.nreduce, copy_out=False)
        else:
            ctx.run_job(MRG_APP_WC, host, nreduce=args.nreduce, copy_out=False)
        ctx.sync()
        th = time.perf_counter() - t0
        pcie = {"value": round(nbytes / th / 1e9, 3), "unit": "GB/s", "ms": round(th * 1e3, 3),
                "h2d_only": round(nbytes / th2d / 1e9, 3), "ratio_to_h2d_only": round(th2d / th, 4),
                "note": "one job with the input in pageable host memory (pieces copied on a second stream while "
                        "the map runs); h2d_only = the same bytes copied with nothing else running"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        tg = time.time()
        cpu = cpu_baseline(w, args.cpu_sample_files, args.cpu_sample_mb, args.cpu_seq_files, args.nreduce, ctx)
        wall.add("cpu_baseline", tg)

    ctx.close()
    dev = host = None
    del devs, dev, host
    torch.cuda.empty_cache()
    scaling = None
    if world > 1 and args.scaling_workload not in ("", "none") and args.scaling_workload != args.workload:
        if shared and args.scaling_files is None:
            # a rehearsal: world ranks' C5 splits (2 x 25 GB each, plus their spill
            # pools) do not fit one device's HBM; shrink them (not a measurement)
            args.scaling_files = max(2, WORKLOADS[args.scaling_workload]["files"] * ndev // (4 * world))
            log(f"rehearsal: the {args.scaling_workload} sub-run uses {args.scaling_files} files per split")
        tg = time.time()
        scaling = scaling_subrun(args.scaling_workload, args, rank, world, local, shared, ndev)
        wall.add("scaling_subrun", tg)
    # the slowest rank's phases (the run ends when it does)
    wall_s = wall.as_dict()
    if world > 1:
        allw = [None] * world
        dist.all_gather_object(allw, wall_s)
        wall_s = {k: max(x.get(k, 0.0) for x in allw) for k in allw[0]}

    if rank == 0:
        line = {
            "metric": GREP_METRIC if grep else METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic Zipf corpus from csrc/corpus.c; reference pg-*.txt not bundled)",
            "config": {"workload": f"{w['desc']}; {nbytes / 1e9:.2f} GB per GPU ({args.files} files x "
                                   f"{args.file_mb} MB), device-resident input; {nsplits} distinct splits per GPU "
                                   f"resident, timed steps rotate over them",
                       "splits_per_gpu": nsplits,
                       "nreduce": args.nreduce, "input_bytes_per_gpu": nbytes, "parallelism": f"dp{world}", **({"options": args.opt} if args.opt else {}),
                       "shuffle": "RCCL all-to-all" if world > 1 else "none (single GPU)"},
            **({"rehearsal": True} if shared else {}),
            "roofline": {"bound": "hbm", "kernel": "grep_map_kernel" if grep else "wc_map_kernel",
                         "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                         "map_kernel_ms_median": round(sorted(kern_ms)[len(kern_ms) // 2], 3),
                         "frac_map_partition": round(nbytes / (map_total_avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "note": "achieved = input bytes per launch / mean HIP-event duration of the map kernel "
                                 "on the library stream over the timed steps; frac_of_measured_copy = achieved / "
                                 "6.29 TB/s (SURVEY.md 8(d)); frac_map_partition = input bytes / mean map_total (map kernel + "
                                 "dictionary + aggregation, the Map+partition phase north_star's 50 % is stated on) "
                                 "/ peak"},
            "phases_ms": {"map_kernel": round(avg_kern, 3), "map_total": round(last["map_total_ms"], 3),
                          "dict": round(last["dict_ms"], 3), "agg": round(last["agg_ms"], 3),
                          "exchange": round(last["exchange_ms"], 3), "reduce": round(last["reduce_ms"], 3),
                          "d2h": round(last["d2h_ms"], 3)},
            "same_split_value": same,
            **({"pipelined": pipelined} if pipelined else {}),
            "cold_split": {"ms": round(cold_ms, 3) if cold_ms is not None else None,
                           "dict_ms": round(cold_st["dict_ms"], 3) if cold_st else None,
                           "map_kernel_ms": round(cold_st["map_kernel_ms"], 3) if cold_st else None,
                           "note": "the first warmup step: a fresh context (dictionary built from the split's "
                                   "sample, first allocations); the timed steps then rotate over the resident "
                                   "splits with the context's buffers kept, as a worker's later map tasks do; "
                                   "same_split_value = the same steps re-mapping split 0 only"},
            "staged_input_bytes": int(last["staged_bytes"]),
            "distinct_keys": int(last["distinct_keys"]),
            "dict_hit_words": int(last["dict_hits"]),
            "spilled_words": int(last["lds_overflow"]),
            "spill_record_bytes": int(last.get("spill_record_bytes", 0)),
            "spill_region_full_words": int(last["spill_ovf"]),
            "aggregator_miss_words": int(last["agg_miss"]),
            "aggregation_rounds": int(last["agg_rounds"]),
            "spill_buckets": int(last["spill_buckets"]),
            "output_bytes": int(last["output_bytes"]),
            "checks": checks,
            "pcie_inclusive": pcie,
            "multi_gpu": multi,
            "multi_gpu_scaling_workload": scaling,
            "cpu_baseline": cpu,
            "wall_s": wall_s,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
