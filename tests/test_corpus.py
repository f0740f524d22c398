"""CPU tests: the synthetic corpus generator (csrc/corpus.c) has the properties
the configs rely on."""
from __future__ import annotations

import hashlib
import unicodedata

import numpy as np

from mrgpu import corpus as C


def test_deterministic_and_file_independent():
    v = C.Vocab(C.KIND_ASCII, 1.07, 10000, 5)
    a = v.fill_files([100_000, 50_000], [1, 2], C.wc_params())
    b = v.fill_files([50_000], [2], C.wc_params())
    assert bytes(a[1]) == bytes(b[0])
    c = C.Vocab(C.KIND_ASCII, 1.07, 10000, 5).fill_files([100_000], [1], C.wc_params())
    assert bytes(a[0]) == bytes(c[0])
    assert all(bytes(f)[-1:] == b"\n" for f in a)


def test_ascii_corpus_is_ascii_and_zipfy():
    v = C.Vocab(C.KIND_ASCII, 1.07, 100000, 2)
    f = bytes(v.fill_files([2_000_000], [7], C.wc_params())[0])
    assert max(f) < 0x80
    words = f.replace(b"\n", b" ").split()
    assert len(words) > 250_000


def test_vocab_words_distinct_and_letters():
    for kind in (C.KIND_ASCII, C.KIND_UTF8):
        v = C.Vocab(kind, 1.07, 300000, 3)
        ws = [v.word(k) for k in list(range(20000)) + list(range(290000, 300000))]
        assert len(set(ws)) == len(ws)
        for w in ws[:3000]:
            s = w.decode("utf-8")
            assert s and all(unicodedata.category(ch).startswith("L") for ch in s), w


def test_utf8_separators_are_not_letters():
    for cp in (0x00A0, 0x2014, 0x3001, 0x1F600, 0x0301, 0x0660):
        assert not unicodedata.category(chr(cp)).startswith("L")


def test_grep_corpus_valid_utf8_with_matches():
    v = C.Vocab(C.KIND_UTF8, 1.07, 20000, 3)
    f = bytes(v.fill_files([500_000], [9], C.grep_params(match_rate=0.01))[0])
    f.decode("utf-8")  # valid UTF-8 only (SURVEY.md §8c grep caveat)
    lines = f.split(b"\n")
    hits = [l for l in lines if b"distributed" in l]
    assert 0.003 * len(lines) < len(hits) < 0.03 * len(lines)
    assert len(set(hits)) < len(hits)  # some duplicate lines


def test_c1_presets():
    """C1 is the English-like substitute (tests/test_c1.py pins its bytes)."""
    cfg = C.CONFIGS["C1"]
    assert cfg["generator"] == "c1_files" and cfg["file_sizes"] == C.C1_SIZES and cfg["nreduce"] == 10
