"""Test-side loader for the oracle (oracle/_build/liboracle.so + oracle/mr_oracle.py).

TEST INFRASTRUCTURE: the oracle is the checker, never the thing measured.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from ctypes import POINTER, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
PKG_DIR = os.path.join(ROOT, "distributed-systems-implemented_amd")
for p in (ORACLE_DIR, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

import mr_oracle  # noqa: E402  (pure-Python restatement)

APP_WC, APP_GREP = 1, 2
_lib = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        p = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
        if not os.path.exists(p):
            build_oracle()
        L = ctypes.CDLL(p)
        L.oracle_is_letter.argtypes = [c_uint32]
        L.oracle_is_letter.restype = c_int
        L.oracle_ihash.argtypes = [c_void_p, c_size_t]
        L.oracle_ihash.restype = c_uint32
        L.oracle_fnv1a32.argtypes = [c_void_p, c_size_t]
        L.oracle_fnv1a32.restype = c_uint32
        L.oracle_wc_words.argtypes = [c_void_p, c_size_t, POINTER(c_uint64), POINTER(c_uint32), c_size_t]
        L.oracle_wc_words.restype = c_size_t
        L.oracle_mrsequential.argtypes = [c_int, c_void_p, c_size_t, POINTER(c_void_p), POINTER(c_size_t), c_size_t,
                                          POINTER(c_void_p), POINTER(c_size_t)]
        L.oracle_mr_partitioned.argtypes = [c_int, c_void_p, c_size_t, POINTER(c_void_p), POINTER(c_size_t), c_size_t,
                                            c_uint32, POINTER(c_void_p), POINTER(c_size_t), POINTER(c_uint64)]
        L.oracle_count_mt.argtypes = [c_int, c_void_p, c_size_t, c_void_p, c_size_t, c_int, c_uint32,
                                      POINTER(c_void_p), POINTER(c_size_t), POINTER(c_uint64)]
        L.oracle_count_mt.restype = c_int
        L.oracle_merge_parts.argtypes = [c_int, c_uint32, POINTER(c_void_p), POINTER(c_uint64), c_uint32,
                                         POINTER(c_void_p), POINTER(c_size_t), POINTER(c_uint64)]
        L.oracle_merge_parts.restype = c_int
        L.oracle_free.argtypes = [c_void_p]
        L.oracle_free.restype = None
        _lib = L
    return _lib


def _ptr(b):
    """pointer to bytes or a numpy uint8 array (no copy for numpy)."""
    if isinstance(b, bytes):
        return ctypes.cast(ctypes.c_char_p(b), c_void_p)
    return c_void_p(b.ctypes.data)


def _files(files):
    n = len(files)
    ptrs = (c_void_p * n)(*[_ptr(f) for f in files])
    sizes = (c_size_t * n)(*[len(f) for f in files])
    return ptrs, sizes, files


def _app(app):
    if app == "wc":
        return APP_WC, b""
    assert app.startswith("grep:")
    return APP_GREP, app[5:].encode("utf-8", "surrogateescape")


def c_mrsequential(app: str, files) -> bytes:
    L = lib()
    a, pat = _app(app)
    ptrs, sizes, _keep = _files(files)
    out, n = c_void_p(), c_size_t()
    L.oracle_mrsequential(a, _ptr(pat) if pat else None, len(pat), ptrs, sizes, len(files), ctypes.byref(out),
                          ctypes.byref(n))
    r = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return r


def c_partitioned(app: str, files, nreduce: int) -> list[bytes]:
    L = lib()
    a, pat = _app(app)
    ptrs, sizes, _keep = _files(files)
    out, n = c_void_p(), c_size_t()
    offs = (c_uint64 * (nreduce + 1))()
    L.oracle_mr_partitioned(a, _ptr(pat) if pat else None, len(pat), ptrs, sizes, len(files), nreduce,
                            ctypes.byref(out), ctypes.byref(n), offs)
    r = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return [r[offs[i]:offs[i + 1]] for i in range(nreduce)]


def c_count_mt(app: str, split, nreduce: int, threads: int = 8) -> list[bytes]:
    """The whole job over ONE split (bytes or a numpy uint8 array, no copy), counted
    by `threads` threads (oracle/mrcount.c): mr-out-r for r < nreduce."""
    L = lib()
    a, pat = _app(app)
    out, n = c_void_p(), c_size_t()
    offs = (c_uint64 * (nreduce + 1))()
    rc = L.oracle_count_mt(a, _ptr(pat) if pat else None, len(pat), _ptr(split), len(split), threads, nreduce,
                           ctypes.byref(out), ctypes.byref(n), offs)
    if rc != 0:
        raise MemoryError("oracle_count_mt failed")
    r = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return [r[offs[i]:offs[i + 1]] for i in range(nreduce)]


def c_merge_parts(app: str, outs: list[list[bytes]]) -> list[bytes]:
    """Reduce over the union of several splits' partitioned outputs (each a list of
    R sorted mr-out-r texts): wc counts of equal keys summed, grep lines deduplicated."""
    L = lib()
    a, _ = _app(app)
    R = len(outs[0]) if outs else 0
    joined = [b"".join(o) for o in outs]
    offs = (c_uint64 * (len(outs) * (R + 1)))()
    for i, o in enumerate(outs):
        acc = 0
        for r in range(R):
            offs[i * (R + 1) + r] = acc
            acc += len(o[r])
        offs[i * (R + 1) + R] = acc
    ptrs = (c_void_p * max(1, len(outs)))(*[_ptr(j) for j in joined])
    out, n = c_void_p(), c_size_t()
    roffs = (c_uint64 * (R + 1))()
    rc = L.oracle_merge_parts(a, len(outs), ptrs, offs, R, ctypes.byref(out), ctypes.byref(n), roffs)
    if rc != 0:
        raise ValueError("oracle_merge_parts: malformed input")
    r = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return [r[roffs[i]:roffs[i + 1]] for i in range(R)]


def c_ihash(key: bytes) -> int:
    return int(lib().oracle_ihash(_ptr(key), len(key)))
