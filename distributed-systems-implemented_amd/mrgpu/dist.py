"""Multi-rank plumbing around the C ABI (one process per GPU).

The data path of the shuffle is RCCL inside libmrgpu (mrg_exchange: ncclAllToAll
of per-owner counts, then ncclAllToAllv of the packed partials).  What lives
here is the host-side protocol shared by bench.py and the CPU tests:

* ownership: partition r (= ihash(key) % nReduce) is owned by rank r % nranks;
* the RCCL unique id travels out of band (torch.distributed broadcast here; a
  file or env var for the Go integration — the coordinator RPC stays unchanged);
* a byte all-to-all over torch.distributed (gloo on CPU) with the same
  counts-then-payload shape as mrg_exchange, used to exercise the protocol
  without GPUs (tests/test_dist_gloo.py);
* max-over-ranks timing.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_ranks() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def owner_of(part: int, nranks: int) -> int:
    return part % nranks


def owned_partitions(nreduce: int, rank: int, nranks: int) -> list[int]:
    return [r for r in range(nreduce) if owner_of(r, nranks) == rank]


def broadcast_bytes(payload: bytes | None, src: int = 0) -> bytes:
    obj = [payload]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def alltoallv_bytes(send: list[bytes]) -> list[bytes]:
    """send[j] goes to rank j; returns recv[i] from rank i.  Counts first, then payload
    (the shape of mrg_exchange's ncclAllToAll + ncclAllToAllv)."""
    world = dist.get_world_size()
    assert len(send) == world
    scounts = torch.tensor([len(b) for b in send], dtype=torch.int64)
    rcounts = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(rcounts, scounts)
    sbuf = torch.frombuffer(bytearray(b"".join(send)) or bytearray(1), dtype=torch.uint8)
    rtotal = int(rcounts.sum())
    rbuf = torch.empty(max(rtotal, 1), dtype=torch.uint8)
    if sum(len(b) for b in send) == 0:
        sbuf = torch.empty(0, dtype=torch.uint8)
    dist.all_to_all_single(rbuf[:rtotal], sbuf[:sum(len(b) for b in send)], rcounts.tolist(), scounts.tolist())
    out, off = [], 0
    raw = rbuf[:rtotal].numpy().tobytes()
    for c in rcounts.tolist():
        out.append(raw[off:off + c])
        off += c
    return out


def max_over_ranks(x: float) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
