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


C1_SIZES_ = [100_000, 180_000, 250_000, 320_000, 400_000, 470_000, 530_000, 600_000]

# SURVEY.md §8d presets: (kind, s, V, vocab seed, file size, n files, params factory)
CONFIGS = {
    # C1 is English-like prose from c1_files() (Gutenberg substitute), not the Zipf generator
    "C1": dict(generator="c1_files", seed=1, file_sizes=C1_SIZES_, app="wc", nreduce=10),
    "C2": dict(kind=KIND_ASCII, s=1.07, V=10**6, seed=2, file_sizes=[250_000_000] * 40,
               params=lambda: wc_params(), app="wc", nreduce=10),
    "C3": dict(kind=KIND_UTF8, s=1.07, V=10**6, seed=3, file_sizes=[250_000_000] * 40,
               params=lambda: grep_params(), app="grep", pattern=b"distributed", nreduce=10),
}


# ---------------------------------------------------------------- C1 substitute corpus
# the reference runs mrsequential + wc on the Gutenberg texts
# pg-*.txt (main/test-mr.sh:30), which it does not bundle (.gitignore:36).  The
# substitute: 8 files of 0.1-0.6 MB of English-like ASCII prose, seed 1 —
# Gutenberg-style header, chapter headings with roman and arabic numerals,
# paragraphs wrapped at ~70 columns with CRLF line ends, sentences with commas,
# quotes, apostrophes, hyphens, digits and dates.  Pure function of the seed
# (tests/golden/c1_manifest.json pins every file's SHA-256).
_C1_WORDS = (
    "the of and to a in that he was it his i with as had for you not be her on at by which this she all they "
    "have from my but or were him so one there would me their said we been what if when more no out up into "
    "an man could them do time some very upon then little about now only than like over any before such "
    "other great made well down two may should these first see must much day good our your after old know "
    "us shall never way long through came how mr its most where himself without come again those can life "
    "own think house thought hand head room nothing eyes went yet under young every night mind while face "
    "place last work away door something still against heart many same take father mother moment found "
    "left began voice people world things let even done light side round being thing home looked tell "
    "once whole both felt night years better part say might quite just morning another each whom country "
    "lady letter water town street river window friend answer captain question king book family evening "
    "don't can't won't it's I'm she's we'll they'd o'clock well-known half-past to-morrow good-bye"
).split()
_C1_NAMES = ("Elizabeth Darcy Bennet Holmes Watson Pip Estella Jane Rochester Ahab Ishmael Alice Hatter Jekyll Hyde "
             "Dorian Basil Emma Knightley Catherine Heathcliff Marianne Elinor Oliver Fagin Sherlock Moriarty").split()
_ROMAN = ["I", "II", "III", "IV", "V", "VI", "VII", "VIII", "IX", "X", "XI", "XII", "XIII", "XIV", "XV", "XVI",
          "XVII", "XVIII", "XIX", "XX", "XXI", "XXII", "XXIII", "XXIV", "XXV"]
C1_SIZES = C1_SIZES_


def _c1_file(rnd, size: int, idx: int) -> bytes:
    import math
    words = _C1_WORDS
    w = [1.0 / math.pow(k + 1, 1.0) for k in range(len(words))]
    tot = sum(w)
    cum, acc = [], 0.0
    for x in w:
        acc += x / tot
        cum.append(acc)

    def word():
        u = rnd.random()
        if u < 0.04:
            return rnd.choice(_C1_NAMES)
        if u < 0.05:
            return str(rnd.randint(1, 1900))
        v = rnd.random()
        lo, hi = 0, len(cum) - 1
        while lo < hi:
            mid = (lo + hi) // 2
            if cum[mid] < v:
                lo = mid + 1
            else:
                hi = mid
        return words[lo]

    def sentence():
        n = rnd.randint(4, 24)
        ws = [word() for _ in range(n)]
        ws[0] = ws[0][:1].upper() + ws[0][1:]
        for k in range(1, n - 1):
            if rnd.random() < 0.08:
                ws[k] += rnd.choice([",", ",", ";", ":", " --"])
        s = " ".join(ws) + rnd.choice([".", ".", ".", "!", "?"])
        if rnd.random() < 0.15:
            s = '"' + s + '"'
        return s

    def wrap(par: str) -> str:
        lines, cur = [], ""
        for tok in par.split(" "):
            if cur and len(cur) + 1 + len(tok) > 70:
                lines.append(cur)
                cur = tok
            else:
                cur = tok if not cur else cur + " " + tok
        if cur:
            lines.append(cur)
        return "\r\n".join(lines)

    out = [f"The Project Gutenberg-style EBook #{1000 + idx} (synthetic substitute text, seed 1)\r\n\r\n"
           f"Title: A Tale of {rnd.choice(_C1_NAMES)} and {rnd.choice(_C1_NAMES)}\r\n"
           f"Release Date: {rnd.choice(['May', 'June', 'August'])} {rnd.randint(1, 28)}, {rnd.randint(1994, 2012)}"
           f" [EBook #{1000 + idx}]\r\n\r\n*** START OF THIS SYNTHETIC EBOOK ***\r\n\r\n"]
    n, chap = len(out[0]), 0
    while n < size:
        if rnd.random() < 0.03 or chap == 0:
            chap += 1
            t = f"\r\n\r\nCHAPTER {_ROMAN[(chap - 1) % len(_ROMAN)]}. ({chap})\r\n\r\n"
        else:
            t = wrap(" ".join(sentence() for _ in range(rnd.randint(2, 8)))) + "\r\n\r\n"
        out.append(t)
        n += len(t)
    data = "".join(out).encode("ascii")[:size - 2] + b"\r\n"
    return data


def c1_files(seed: int = 1) -> list[bytes]:
    """The C1 substitute corpus: 8 files, C1_SIZES bytes each, ending in CRLF."""
    import random
    rnd = random.Random(seed)
    return [_c1_file(rnd, sz, i) for i, sz in enumerate(C1_SIZES)]
