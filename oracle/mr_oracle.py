"""CPU restatement of the reference MapReduce hot path — TEST INFRASTRUCTURE ONLY.

This module is the *oracle*: a pure-Python restatement of the Go reference's
word-count / grep Map, the ``ihash`` partitioner and the sort/group/Reduce loop.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker.  The product path
(``distributed-systems-implemented_amd``) never imports anything under
``oracle/``.

Parity status: the reference is pure Go and no Go toolchain exists in this
image, and the reference ships no fixtures/golden vectors.  So
this oracle is *parity unpinned* against reference-run outputs.  It is pinned
instead to (1) the published FNV-1a-32 known-answer vectors, (2) the Unicode
13.0.0 UCD (Go 1.16–1.20's table version) through ``unicodedata``, and (3) an
explicit restatement of Go's ``utf8.DecodeRuneInString`` acceptance ranges.

Reference functions restated (file:line under /root/reference):
  * ``wc_map``      -> MapReduce/mrapps/wc.go:21-34  (strings.FieldsFunc + !unicode.IsLetter)
  * ``wc_reduce``   -> MapReduce/mrapps/wc.go:41-44  (strconv.Itoa(len(values)))
  * ``grep_map``    -> MapReduce/mrapps/dgrep.go:18-36 (strings.Split on "\n", literal match)
  * ``grep_reduce`` -> MapReduce/mrapps/dgrep.go:44-46 (returns key)
  * ``ihash``       -> MapReduce/mr/worker.go:33-37  (FNV-1a 32 & 0x7fffffff)
  * ``mrsequential``-> MapReduce/main/mrsequential.go:38-86 (map all, sort, group, reduce)
  * ``mr_partitioned`` -> MapReduce/mr/worker.go:72-78 + 123-146 (ihash % nReduce buckets,
    per-partition sort/group/reduce into mr-out-r)

Pure-Python loops: use on small inputs only (the C oracle in ``mroracle.c`` is
the fast restatement for larger parity cases).
"""
from __future__ import annotations

import unicodedata

UNICODE_VERSION = unicodedata.unidata_version  # "13.0.0" in this image
RUNE_ERROR = 0xFFFD

# FNV-1a 32 constants (hash/fnv: offset32, prime32)
FNV_OFFSET32 = 2166136261
FNV_PRIME32 = 16777619


def decode_rune(b: bytes, i: int) -> tuple[int, int]:
    """Go ``utf8.DecodeRuneInString`` at offset i: returns (rune, width).

    Invalid / truncated / overlong / surrogate encodings return (0xFFFD, 1),
    exactly as Go's ``for i, r := range s`` does (used by strings.FieldsFunc,
    wc.go:26).  Acceptance ranges follow Go's unicode/utf8 first/accept tables.
    """
    n = len(b)
    c0 = b[i]
    if c0 < 0x80:
        return c0, 1
    if c0 < 0xC2 or c0 > 0xF4:
        return RUNE_ERROR, 1
    if c0 < 0xE0:
        need, lo, hi, cp = 1, 0x80, 0xBF, c0 & 0x1F
    elif c0 < 0xF0:
        need, cp = 2, c0 & 0x0F
        lo, hi = (0xA0, 0xBF) if c0 == 0xE0 else ((0x80, 0x9F) if c0 == 0xED else (0x80, 0xBF))
    else:
        need, cp = 3, c0 & 0x07
        lo, hi = (0x90, 0xBF) if c0 == 0xF0 else ((0x80, 0x8F) if c0 == 0xF4 else (0x80, 0xBF))
    if i + need >= n:
        # needs bytes i+1 .. i+need; truncated at end of input -> (RuneError, 1)
        return RUNE_ERROR, 1
    c1 = b[i + 1]
    if c1 < lo or c1 > hi:
        return RUNE_ERROR, 1
    cp = (cp << 6) | (c1 & 0x3F)
    for k in range(2, need + 1):
        ck = b[i + k]
        if ck < 0x80 or ck > 0xBF:
            return RUNE_ERROR, 1
        cp = (cp << 6) | (ck & 0x3F)
    return cp, need + 1


def is_letter(cp: int) -> bool:
    """Go ``unicode.IsLetter`` = general category in {Lu, Ll, Lt, Lm, Lo}.

    Python's ``str.isalpha`` is defined on exactly those categories
    (unicodedata 13.0.0 here).  U+FFFD (category So) is not a letter.
    """
    if cp < 0x80:
        return (0x41 <= cp <= 0x5A) or (0x61 <= cp <= 0x7A)
    return chr(cp).isalpha()


def wc_map(contents: bytes) -> list[bytes]:
    """wc.go:21-34: ``strings.FieldsFunc(contents, !unicode.IsLetter)``.

    Returns the words (maximal runs of letter runes) in input order; each is a
    byte slice of ``contents`` (Go substrings alias the input).
    """
    out: list[bytes] = []
    n = len(contents)
    i = 0
    start = -1
    while i < n:
        cp, w = decode_rune(contents, i)
        if is_letter(cp):
            if start < 0:
                start = i
        elif start >= 0:
            out.append(contents[start:i])
            start = -1
        i += w
    if start >= 0:
        out.append(contents[start:n])
    return out


def wc_reduce(key: bytes, values: list[bytes]) -> bytes:
    """wc.go:41-44: ``strconv.Itoa(len(values))``."""
    return str(len(values)).encode()


def grep_map(contents: bytes, pattern: bytes) -> list[bytes]:
    """dgrep.go:18-36 with a fixed *literal* pattern.

    ``strings.Split(contents, "\\n")`` keeps ``\\r`` and yields a final "" after a
    trailing newline; a line is emitted (once per line) when the literal occurs
    in it.  For a valid-UTF-8 literal, Go's regexp match equals a byte-substring
    test; the empty pattern matches every line.
    dgrep.go:20-23: when ``regexp.Compile`` fails grepMap returns nil — for a
    quoted literal that is exactly an invalid-UTF-8 pattern (regexp/syntax
    rejects it with ErrInvalidUTF8).
    """
    if not valid_utf8(pattern):
        return []
    return [line for line in contents.split(b"\n") if pattern in line]


def valid_utf8(b: bytes) -> bool:
    """Go's utf8.Valid: every rune decodes with width > 1 or is ASCII (decode_rune)."""
    i = 0
    while i < len(b):
        cp, w = decode_rune(b, i)
        if cp == 0xFFFD and w == 1 and b[i] >= 0x80:
            return False
        i += w
    return True


def grep_reduce(key: bytes, values: list[bytes]) -> bytes:
    """dgrep.go:44-46: returns the key."""
    return key


def fnv1a32(key: bytes) -> int:
    h = FNV_OFFSET32
    for c in key:
        h ^= c
        h = (h * FNV_PRIME32) & 0xFFFFFFFF
    return h


def ihash(key: bytes) -> int:
    """worker.go:33-37: ``int(fnv.New32a().Sum32() & 0x7fffffff)``."""
    return fnv1a32(key) & 0x7FFFFFFF


def _map_reduce_fns(app: str):
    if app == "wc":
        return (lambda name, data: wc_map(data)), wc_reduce
    if app.startswith("grep:"):
        pat = app[len("grep:"):].encode("utf-8", "surrogateescape")
        return (lambda name, data: grep_map(data, pat)), grep_reduce
    raise ValueError(f"unknown app {app!r}")


def _group_reduce(keys: list[bytes], reducef) -> bytes:
    """mrsequential.go:59-84 / worker.go:123-146: sort (bytewise), group, reduce, print.

    Each value is implied by the app ("1" for wc, "" for grep); only its count
    matters for wc.Reduce and it is ignored by grepReduce, so ``values`` is a
    list of the right length.
    """
    keys = sorted(keys)  # Go string '<' == unsigned bytewise lexicographic
    out = []
    i = 0
    n = len(keys)
    while i < n:
        j = i + 1
        while j < n and keys[j] == keys[i]:
            j += 1
        values = [b""] * (j - i)
        out.append(keys[i] + b" " + reducef(keys[i], values) + b"\n")
        i = j
    return b"".join(out)


def mrsequential(app: str, files: list[bytes]) -> bytes:
    """mrsequential.go:25-87 -> the bytes of mr-out-0."""
    mapf, reducef = _map_reduce_fns(app)
    inter: list[bytes] = []
    for k, data in enumerate(files):
        inter.extend(mapf(f"file{k}", data))
    return _group_reduce(inter, reducef)


def mr_partitioned(app: str, files: list[bytes], nreduce: int) -> list[bytes]:
    """Map tasks (worker.go:55-97) + reduce tasks (worker.go:99-161): mr-out-r for r<nreduce.

    Every partition produces its file, possibly empty (worker.go:126-148 always runs).
    """
    mapf, reducef = _map_reduce_fns(app)
    buckets: list[list[bytes]] = [[] for _ in range(nreduce)]
    for k, data in enumerate(files):
        for key in mapf(f"file{k}", data):
            buckets[ihash(key) % nreduce].append(key)
    return [_group_reduce(b, reducef) for b in buckets]


# ---------------------------------------------------------------- intermediate files
def go_json_string(s: bytes) -> bytes:
    """encoding/json ``encodeState.string(s, escapeHTML=true)`` (json.Encoder's
    default), Go 1.16-1.21: the encoding of a KeyValue string in mr-X-Y
    (worker.go:84-86).  '"' and '\\' get a backslash, \\n \\r \\t their short
    forms, other bytes < 0x20 and '<' '>' '&' become \\u00XX; a byte that
    decodes to RuneError of width 1 becomes \\ufffd; U+2028 / U+2029 become
    \\u2028 / \\u2029; everything else is copied.  (Go 1.22 added \\b and \\f.)"""
    out = bytearray(b'"')
    i, n = 0, len(s)
    while i < n:
        b = s[i]
        if b < 0x80:
            if b >= 0x20 and b not in b'"\\<>&':
                out.append(b)
            elif b in b'"\\':
                out += b"\\" + bytes([b])
            elif b == 0x0A:
                out += b"\\n"
            elif b == 0x0D:
                out += b"\\r"
            elif b == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + b"%02x" % b
            i += 1
            continue
        cp, w = decode_rune(s, i)
        if cp == RUNE_ERROR and w == 1:
            out += b"\\ufffd"
        elif cp in (0x2028, 0x2029):
            out += b"\\u%04x" % cp
        else:
            out += s[i:i + w]
        i += w
    out += b'"'
    return bytes(out)


def go_json_kv_line(key: bytes, value: bytes) -> bytes:
    """One ``json.NewEncoder(f).Encode(&kv)`` line (worker.go:84-86)."""
    return b'{"Key":' + go_json_string(key) + b',"Value":' + go_json_string(value) + b"}\n"


def intermediate_json_lines(app: str, files: list[bytes], nreduce: int, r: int) -> list[bytes]:
    """The lines a reference map worker writes to mr-X-r for these inputs
    (worker.go:69-92): one per emitted KeyValue of bucket r, in emission order."""
    mapf, _ = _map_reduce_fns(app)
    value = b"1" if app == "wc" else b""
    return [go_json_kv_line(key, value)
            for k, data in enumerate(files) for key in mapf(f"file{k}", data)
            if ihash(key) % nreduce == r]
