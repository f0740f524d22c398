"""CPU tests: pin the oracle before trusting it.

* published FNV-1a-32 KATs (hash/fnv) for both restatements;
* the C oracle reproduces every golden fixture made by the Python restatement;
* the Python restatement reproduces its own committed fixtures (regression);
* Go's UTF-8 decode rule: the Go-faithful decoder, the local rune-start rule and
  CPython's UTF-8 codec agree on which bytes are letters (SURVEY.md §8c pin 3).
"""
from __future__ import annotations

import base64
import json
import os
import random

import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
M = O.mr_oracle


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def dec(s):
    return base64.b64decode(s)


def test_fnv_published_kats():
    kat = _load("fnv_kat.json")
    for k, v in kat["published"].items():
        assert M.fnv1a32(k.encode()) == v
        assert O.lib().oracle_fnv1a32(O._ptr(k.encode()), len(k)) == v
    for k, v in kat["ihash"].items():
        b = dec(k)
        assert M.ihash(b) == v == O.c_ihash(b)
    # worker.go:36 masks the sign bit
    assert M.ihash(b"foobar") == 0xBF9CF968 & 0x7FFFFFFF == 1067252072


@pytest.mark.parametrize("name", sorted(_load("wc_cases.json")))
def test_c_oracle_wc_golden(name):
    case = _load("wc_cases.json")[name]
    files = [dec(f) for f in case["files"]]
    for R, outs in case["out"].items():
        want = [dec(x) for x in outs]
        assert O.c_partitioned("wc", files, int(R)) == want
    assert O.c_mrsequential("wc", files) == dec(case["out"]["1"][0])


@pytest.mark.parametrize("name", sorted(_load("grep_cases.json")))
def test_c_oracle_grep_golden(name):
    case = _load("grep_cases.json")[name]
    files = [dec(f) for f in case["files"]]
    app = "grep:" + dec(case["pattern"]).decode("utf-8", "surrogateescape")
    for R, outs in case["out"].items():
        assert O.c_partitioned(app, files, int(R)) == [dec(x) for x in outs]


def test_python_oracle_regression():
    case = _load("wc_cases.json")["utf8_mix"]
    files = [dec(f) for f in case["files"]]
    assert M.mr_partitioned("wc", files, 10) == [dec(x) for x in case["out"]["10"]]


def _letter_bytes_go(b: bytes) -> list[bool]:
    out = [False] * len(b)
    i = 0
    while i < len(b):
        cp, w = M.decode_rune(b, i)
        let = M.is_letter(cp)
        for k in range(w):
            out[i + k] = let
        i += w
    return out


def _letter_bytes_local(b: bytes) -> list[bool]:
    """Local rule: byte q starts a rune unless a valid sequence longer than k starts at q-k."""
    n = len(b)

    def vl(q):
        if q < 0 or q >= n:
            return 0
        cp, w = M.decode_rune(b, q)
        return w if not (cp == 0xFFFD and w == 1 and b[q:q + 3] != b"\xef\xbf\xbd") else 0

    out = [False] * n
    for q in range(n):
        start = not any(vl(q - k) > k for k in (1, 2, 3))
        if start:
            cp, w = M.decode_rune(b, q)
            let = M.is_letter(cp)
            for k in range(w):
                out[q + k] = let
    return out


def _letter_bytes_codec(b: bytes) -> list[bool]:
    """CPython's UTF-8 codec with 'surrogateescape' gives per-byte attribution."""
    out = []
    for ch in b.decode("utf-8", "surrogateescape"):
        cp = ord(ch)
        if 0xDC80 <= cp <= 0xDCFF:  # an undecodable byte
            out.append(False)
        else:
            out.extend([ch.isalpha()] * len(ch.encode("utf-8")))
    return out


def test_utf8_decode_rules_agree():
    rnd = random.Random(1234)
    alphabet = [b"a", b"Z", b" ", b"\xc3", b"\xa9", b"\xe2", b"\x82", b"\xac", b"\xf0", b"\x9f", b"\x98", b"\x80",
                b"\xed", b"\xa0", b"\xbf", b"\xf4", b"\x90", b"\xc0", b"\xff", b"\xce", b"\xbb", b"\xe4", b"\xb8",
                b"\xad", b"\x8f"]
    for _ in range(3000):
        s = b"".join(rnd.choice(alphabet) for _ in range(rnd.randrange(1, 24)))
        g = _letter_bytes_go(s)
        assert g == _letter_bytes_local(s), s
        assert g == _letter_bytes_codec(s), s
        words_go = M.wc_map(s)
        # maximal runs of letter bytes == FieldsFunc words
        runs, cur = [], bytearray()
        for i, let in enumerate(g):
            if let:
                cur.append(s[i])
            elif cur:
                runs.append(bytes(cur))
                cur = bytearray()
        if cur:
            runs.append(bytes(cur))
        assert runs == words_go


def test_c_decoder_matches_python():
    rnd = random.Random(99)
    data = bytes(rnd.randrange(256) for _ in range(200000))
    assert O.c_mrsequential("wc", [data]) == M.mrsequential("wc", [data])


# encoding/json string encoding of mr-X-Y lines (worker.go:84-86), Go 1.16-1.21
JSON_KAT = [
    (b"the", b'"the"'),
    (b"<a&b>", b'"\\u003ca\\u0026b\\u003e"'),
    (b'a"b\\c', b'"a\\"b\\\\c"'),
    (b"\n\r\t\x08\x0c\x01\x1f", b'"\\n\\r\\t\\u0008\\u000c\\u0001\\u001f"'),
    (b"\x7f/", b'"\x7f/"'),
    (b"\xff", b'"\\ufffd"'),
    (b"\xe2\x80", b'"\\ufffd\\ufffd"'),               # truncated sequence: RuneError per byte
    ("\u2028\u2029".encode(), b'"\\u2028\\u2029"'),
    ("é中\U0001F600".encode(), '"é中\U0001F600"'.encode()),
    (b"\xed\xa0\x80", b'"\\ufffd\\ufffd\\ufffd"'),     # surrogate encoding is invalid UTF-8
]


@pytest.mark.parametrize("raw,want", JSON_KAT)
def test_go_json_string_kat(raw, want):
    import mr_oracle as M
    assert M.go_json_string(raw) == want


def test_go_json_lines_roundtrip_valid_utf8():
    """For valid UTF-8 keys the encoding is lossless: json.loads gives the key back."""
    import json

    import mr_oracle as M
    for key in [b"hello", "na\u00efve \u2028 \u2029 <tag> & \"q\" \\ \t".encode(), "\U0001F600x".encode()]:
        line = M.go_json_kv_line(key, b"1")
        d = json.loads(line)
        assert d["Key"].encode() == key and d["Value"] == "1"
