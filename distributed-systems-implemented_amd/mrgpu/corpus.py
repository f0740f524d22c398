"""Synthetic corpora (ctypes over build/libmrcorpus.so, csrc/corpus.c).

The reference's pg-*.txt inputs are not bundled, so every
BASELINE config runs on deterministic synthetic text; see csrc/corpus.c for the
generator's properties.  Config presets follow SURVEY.md §8d.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_size_t, c_uint64, c_void_p

import numpy as np

from .lib import BUILD_DIR, MrgError

KIND_ASCII = 0
KIND_UTF8 = 1
MODE_WC = 0
MODE_GREP = 1


class Params(ctypes.Structure):
    _fields_ = [
        ("mode", c_int),
        ("invalid_rate", c_double),
        ("pattern", c_char_p),
        ("match_rate", c_double),
        ("dup_rate", c_double),
        ("line_min", c_int),
        ("line_max", c_int),
        ("vocab_lo", c_uint64),
        ("vocab_hi", c_uint64),
    ]


_lib = None


def _load():
    global _lib
    if _lib is None:
        p = os.path.join(BUILD_DIR, "libmrcorpus.so")
        if not os.path.exists(p):
            raise MrgError(f"{p} not built")
        L = ctypes.CDLL(p)
        L.mrc_vocab_new.argtypes = [c_int, c_double, c_uint64, c_uint64]
        L.mrc_vocab_new.restype = c_void_p
        L.mrc_vocab_free.argtypes = [c_void_p]
        L.mrc_vocab_free.restype = None
        L.mrc_word.argtypes = [c_void_p, c_uint64, c_char_p]
        L.mrc_word.restype = c_int
        L.mrc_fill.argtypes = [c_void_p, c_uint64, c_void_p, c_size_t, POINTER(Params)]
        L.mrc_fill.restype = c_size_t
        L.mrc_fill_files.argtypes = [c_void_p, POINTER(c_uint64), POINTER(c_void_p), POINTER(c_size_t), c_size_t,
                                     POINTER(Params), c_int]
        L.mrc_fill_files.restype = c_int
        _lib = L
    return _lib


class Vocab:
    """Zipf(s) vocabulary of V distinct words (ASCII mixed-case or mixed-script UTF-8)."""

    def __init__(self, kind: int = KIND_ASCII, s: float = 1.07, V: int = 10**6, seed: int = 2):
        self.L = _load()
        self.kind, self.s, self.V, self.seed = kind, s, V, seed
        self.h = self.L.mrc_vocab_new(kind, s, V, seed)
        if not self.h:
            raise MrgError("mrc_vocab_new failed")

    def word(self, k: int) -> bytes:
        b = ctypes.create_string_buffer(64)
        n = self.L.mrc_word(self.h, k, b)
        return b.raw[:n]

    def close(self):
        if self.h:
            self.L.mrc_vocab_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fill_files(self, sizes, seeds, params: Params | None = None, threads: int | None = None,
                   out: np.ndarray | None = None) -> list[np.ndarray]:
        """Generate len(sizes) files in parallel; returns views into one contiguous uint8 array."""
        total = int(sum(sizes))
        buf = out if out is not None else np.empty(total, dtype=np.uint8)
        assert buf.nbytes >= total
        views, ptrs, off = [], [], 0
        for s in sizes:
            v = buf[off:off + s]
            views.append(v)
            ptrs.append(buf.ctypes.data + off)
            off += s
        n = len(sizes)
        c_seeds = (c_uint64 * n)(*[int(x) for x in seeds])
        c_ptrs = (c_void_p * n)(*ptrs)
        c_sizes = (c_size_t * n)(*[int(x) for x in sizes])
        if threads is None:
            threads = min(16, os.cpu_count() or 1)
        self.L.mrc_fill_files(self.h, c_seeds, c_ptrs, c_sizes, n, ctypes.byref(params) if params else None, threads)
        return views


def wc_params(invalid_rate: float = 0.0, vocab_lo: int = 0, vocab_hi: int = 0) -> Params:
    return Params(MODE_WC, invalid_rate, None, 0.0, 0.0, 0, 0, vocab_lo, vocab_hi)


def grep_params(pattern: bytes = b"distributed", match_rate: float = 0.005, dup_rate: float = 0.2,
                line_min: int = 40, line_max: int = 120) -> Params:
    return Params(MODE_GREP, 0.0, pattern, match_rate, dup_rate, line_min, line_max, 0, 0)


# SURVEY.md §8d presets: (kind, s, V, vocab seed, file size, n files, params factory)
CONFIGS = {
    "C1": dict(kind=KIND_ASCII, s=1.07, V=20000, seed=1, file_sizes=[100_000, 180_000, 250_000, 320_000,
                                                                      400_000, 470_000, 530_000, 600_000],
               params=lambda: wc_params(), app="wc", nreduce=10),
    "C2": dict(kind=KIND_ASCII, s=1.07, V=10**6, seed=2, file_sizes=[250_000_000] * 40,
               params=lambda: wc_params(), app="wc", nreduce=10),
    "C3": dict(kind=KIND_UTF8, s=1.07, V=10**6, seed=3, file_sizes=[250_000_000] * 40,
               params=lambda: grep_params(), app="grep", pattern=b"distributed", nreduce=10),
}
