"""Host codec of the intermediate-partials format "MRGI" (mrg_parts_export/import).

Replaces the reference's per-occurrence JSON lines in mr-X-Y
(MapReduce/mr/worker.go:80-92 write, :100-122 read) with one record per distinct
key: the map side has already combined counts (every wc value is "1").

Layout (little endian), identical to csrc/mrgpu_api.hip `IHdr` + SoA arrays:
  u32 magic "MRGI", u32 app, u32 nreduce, u32 part (0xFFFFFFFF = all), u64 n, u64 arena_n
  u64 k0[n], u64 k1[n], u64 count[n], u64 koff[n], u32 len[n], u32 part[n], u8 arena[arena_n]
k0/k1 hold the first 16 key bytes zero-padded; keys longer than 16 bytes (and
grep lines) live in the arena at koff (koff = 2**64-1 for inline keys).
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = 0x4947524D
HDR = struct.Struct("<IIIIQQ")
INLINE = np.uint64(0xFFFFFFFFFFFFFFFF)


def decode(data: bytes) -> dict:
    """MRGI bytes -> {"app", "nreduce", "part", "keys": [bytes], "count": np.ndarray, "kpart": np.ndarray}."""
    magic, app, nreduce, part, n, arena_n = HDR.unpack_from(data, 0)
    if magic != MAGIC or HDR.size + n * 40 + arena_n != len(data):
        raise ValueError("not an MRGI buffer")
    off = HDR.size

    def arr(dt, cnt):
        nonlocal off
        a = np.frombuffer(data, dtype=dt, count=cnt, offset=off)
        off += a.nbytes
        return a

    k0, k1, cnt, koff = arr("<u8", n), arr("<u8", n), arr("<u8", n), arr("<u8", n)
    ln, kp = arr("<u4", n), arr("<u4", n)
    arena = data[off:off + arena_n]
    keys = []
    for i in range(n):
        L = int(ln[i])
        if koff[i] == INLINE:
            keys.append((int(k0[i]).to_bytes(8, "little") + int(k1[i]).to_bytes(8, "little"))[:L])
        else:
            o = int(koff[i])
            keys.append(bytes(arena[o:o + L]))
    return {"app": app, "nreduce": nreduce, "part": part, "keys": keys, "count": np.array(cnt),
            "kpart": np.array(kp)}


def encode(app: int, nreduce: int, keys: list[bytes], counts, parts, part: int = 0xFFFFFFFF) -> bytes:
    """Records -> MRGI bytes (keys <= 16 bytes without NUL bytes inline, others in the arena)."""
    n = len(keys)
    k0 = np.zeros(n, "<u8")
    k1 = np.zeros(n, "<u8")
    koff = np.full(n, INLINE, "<u8")
    ln = np.zeros(n, "<u4")
    arena = bytearray()
    for i, k in enumerate(keys):
        ln[i] = len(k)
        pad = (k[:16] + b"\0" * 16)[:16]
        k0[i] = int.from_bytes(pad[:8], "little")
        k1[i] = int.from_bytes(pad[8:], "little")
        if len(k) > 16 or b"\0" in k or app != 1:
            koff[i] = len(arena)
            arena += k
    hdr = HDR.pack(MAGIC, app, nreduce, part, n, len(arena))
    return b"".join([hdr, k0.tobytes(), k1.tobytes(), np.asarray(counts, "<u8").tobytes(), koff.tobytes(),
                     ln.tobytes(), np.asarray(parts, "<u4").tobytes(), bytes(arena)])
