"""GPU parity: the HIP path (through the C ABI) vs the oracle, bit-exact.

Gate: for every r, mr-out-r from the GPU equals the oracle's
partition-r output byte for byte (the stricter per-partition check); with
nreduce = 1 that is mrsequential's mr-out-0.  Also the reference's own check
(test-mr.sh:52-53): sorted concatenation of mr-out-* equals sorted mr-out-0.
"""
from __future__ import annotations

import numpy as np
import pytest

import _oracle as O
import cases
from mrgpu import ALL_PARTS, MRG_APP_GREP, MRG_APP_WC
from mrgpu import corpus as C

pytestmark = pytest.mark.gpu


def gpu_partitioned(ctx, app: str, files: list[bytes], nreduce: int) -> list[bytes]:
    """Map each file as its own split (worker.go map task), merge, reduce all partitions."""
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    pat = b"" if app == "wc" else app[5:].encode("utf-8", "surrogateescape")
    parts = None
    for f in files:
        p = ctx.map(a, f, pattern=pat, nreduce=nreduce)
        if parts is None:
            parts = p
        else:
            ctx.merge(parts, p)
            p.free()
    out = ctx.reduce_all(parts)
    parts.free()
    return out


def check(ctx, app, files, nreduces=(1, 10, 64)):
    for R in nreduces:
        got = gpu_partitioned(ctx, app, files, R)
        want = O.c_partitioned(app, files, R)
        assert len(got) == R
        for r in range(R):
            if got[r] != want[r]:
                gl, wl = got[r].split(b"\n"), want[r].split(b"\n")
                diff = next((i for i in range(min(len(gl), len(wl))) if gl[i] != wl[i]), None)
                raise AssertionError(f"app={app} R={R} r={r}: {len(got[r])} vs {len(want[r])} bytes; first diff "
                                     f"line {diff}: got {gl[diff] if diff is not None else None!r} "
                                     f"want {wl[diff] if diff is not None else None!r}")
    # mrsequential gate (R = 1) and test-mr.sh's "sort | grep ." equivalence
    seq = O.c_mrsequential(app, files)
    allp = gpu_partitioned(ctx, app, files, 10)
    lines = sorted(l for part in allp for l in part.split(b"\n") if l)
    assert lines == sorted(l for l in seq.split(b"\n") if l)


@pytest.mark.parametrize("name", sorted(cases.edge_cases()))
def test_wc_edge_cases(wctx, name):
    check(wctx, "wc", cases.edge_cases()[name])


@pytest.fixture(scope="module")
def ctx_grep_bins():
    """grep reduce by the bins for a device output too (option grep_bins = 3;
    by default the bins serve mrg_run_job's output into pinned host memory and
    mrg_reduce_all keeps the radix path)."""
    from mrgpu import Context
    c = Context(0)
    c.set_option("grep_bins", 3)
    yield c
    c.close()


@pytest.mark.parametrize("name", sorted(cases.grep_edge_cases()))
def test_grep_edge_cases(ctx, name):
    files, pat = cases.grep_edge_cases()[name]
    check(ctx, "grep:" + pat.decode("utf-8", "surrogateescape"), files, nreduces=(1, 10))


@pytest.mark.parametrize("name", sorted(cases.grep_edge_cases()))
def test_grep_edge_cases_bins(ctx_grep_bins, name):
    files, pat = cases.grep_edge_cases()[name]
    check(ctx_grep_bins, "grep:" + pat.decode("utf-8", "surrogateescape"), files, nreduces=(1, 10))


@pytest.mark.parametrize("name", ["basic", "tied_lines", "chunk_seams", "long_lines_many_hits", "shared_prefix_70"])
def test_grep_run_job_host_output(ctx, name):
    """mrg_run_job's default path (lines into pinned host memory: the bins fused
    with the output) against the oracle."""
    files, pat = cases.grep_edge_cases()[name]
    for R in (1, 10):
        got = ctx.run_job(MRG_APP_GREP, b"\n".join(files), pattern=pat, nreduce=R)
        want = O.c_partitioned("grep:" + pat.decode("utf-8", "surrogateescape"), [b"\n".join(files)], R)
        assert got == want, f"{name} R={R}"


@pytest.mark.parametrize("pat", [b"a.b", b"x+y", b"(q)", b"[z]", b"^s", b"e$", b"w*", b"u?", b"{2}", b"p|q", "ά\\d".encode()])
def test_grep_regexp_metachars(ctx, pat):
    """dgrep.go:20 compiles the pattern as a regexp and this path matches literals:
    a valid-UTF-8 pattern holding a metacharacter is refused (MRG_EINVAL) instead
    of silently matching differently; with option grep_literal = 1 (the caller
    asked for regexp.QuoteMeta semantics) it is matched as a literal, exactly as
    the oracle's literal grep.  Invalid UTF-8 keeps dgrep.go:20-23's no lines."""
    from mrgpu.lib import MrgError
    files = [b"a.b ab axb\nx+y xy\n(q) q\n[z] z\n^s s\ne$ e\nw* w\nu? u\n{2} 2\np|q pq\n" + "ά\\d ά5\n".encode()]
    with pytest.raises(MrgError, match="metacharacter"):
        ctx.map(MRG_APP_GREP, files[0], pattern=pat, nreduce=10)
    ctx.set_option("grep_literal", 1)
    try:
        check(ctx, "grep:" + pat.decode(), files, nreduces=(1, 10))
        got = gpu_partitioned(ctx, "grep:" + pat.decode(), files, 1)
        assert got[0].count(b"\n") == 1  # exactly the line holding the literal
    finally:
        ctx.set_option("grep_literal", 0)
    # invalid UTF-8 with a metacharacter: regexp.Compile fails -> no lines, no error
    assert gpu_partitioned(ctx, "grep:" + (b"\xff" + pat).decode("utf-8", "surrogateescape"), files, 10) == [b""] * 10


@pytest.mark.parametrize("kind,V,seed,inv", [(C.KIND_ASCII, 5000, 1, 0.0), (C.KIND_ASCII, 200000, 2, 0.0),
                                             (C.KIND_UTF8, 20000, 3, 0.0), (C.KIND_UTF8, 20000, 4, 0.001)])
def test_wc_synthetic(wctx, kind, V, seed, inv):
    files = cases.synthetic(kind, V, [1_000_003, 2_500_000, 777_777], seed, inv)
    check(wctx, "wc", files, nreduces=(1, 10, 64))
    if wctx.stats()["dict_keys"]:
        assert wctx.stats()["dict_hits"] > 0


@pytest.mark.parametrize("lean", [0, -1])
def test_wc_lean_after_ascii(wctx, lean):
    """A split after an all-ASCII one maps with the lean variant (long words all
    through the start-offset list, UTF-8 by the per-lane lead loop): exact on
    mixed-script text with long words, on the window-end and invalid UTF-8
    cases, and on ASCII again; lean -1 keeps the full variant."""
    wctx.set_option("map_lean", lean)
    ascii = cases.synthetic(C.KIND_ASCII, 20000, [1_000_000], 31)
    mixed = cases.synthetic(C.KIND_UTF8, 20000, [1_500_000], 32, 0.0005) + [cases.long_words(500_000, 3)]
    edge = cases.edge_cases()
    try:
        for f in [ascii[0], mixed[0], ascii[0], mixed[1], ascii[0]] + edge["utf8_slot_tail"] + [ascii[0]] + \
                edge["invalid_utf8"]:
            assert gpu_partitioned(wctx, "wc", [f], 10) == O.c_partitioned("wc", [f], 10)
    finally:
        wctx.set_option("map_lean", 0)


@pytest.mark.parametrize("list_cap,lrec", [(0, 0), (300, 0), (0, 8), (300, -1)])
def test_wc_long_words_many(wctx, list_cap, lrec):
    """Mixed-script text with many words over 16 bytes, and splits made only of
    17-70-byte words: words of 17-32 bytes ending inside the map window leave as
    32-byte key records (lrec 0; lrec 8: 8-record regions that overflow, are
    regrown from the busiest map wave's count and re-run; -1: records off), the
    rest go to the map waves' reserved ranges of the long-word list with their
    closing holes (list overflow + re-run: a 300-entry list), and both long-word
    kernels' LDS pre-aggregation of hot long words."""
    files = cases.synthetic(C.KIND_UTF8, 20000, [2_000_000, 1_000_001], 21, 0.0005) + \
        [cases.long_words(3_000_000, 1), cases.long_words(70_000, 2)]
    wctx.set_option("list_cap", list_cap)
    if lrec > 0:
        wctx.set_option("lrec_cap", lrec)
    if lrec < 0:
        wctx.set_option("long_records", -1)
    try:
        check(wctx, "wc", files, nreduces=(1, 10))
    finally:
        wctx.set_option("list_cap", 0)
        wctx.set_option("lrec_cap", 0)
        wctx.set_option("long_records", 0)


def test_wc_long_records_fewer_than_ranges(wctx):
    """Splits with fewer 17-32-byte records than wc_lrec_kernel has ranges (512)
    after a split with millions of them on the same context: the empty ranges'
    partial counts must not be the previous split's (mrcoord's small files
    caught that)."""
    files = [cases.long_words(3_000_000, 1), cases.long_words(2_000, 5)] + \
        cases.synthetic(C.KIND_UTF8, 20000, [1_000, 90_000, 7], 61, 0.001) + [cases.long_words(40, 6)]
    for f in files:
        assert gpu_partitioned(wctx, "wc", [f], 10) == O.c_partitioned("wc", [f], 10)
    check(wctx, "wc", files, nreduces=(10,))


@pytest.mark.parametrize("sort_hits,emit", [(0, 1), (1, 1), (0, 0)])
def test_grep_synthetic(ctx, sort_hits, emit):
    """grep over synthetic lines; the hits resolved in the map kernel's order
    (default) or sorted by position first (option grep_sort_hits = 1); the
    records written by the LongTable insert as it claims a line (default) or by
    a collect pass over the table afterwards (option grep_emit = 0); the edge
    cases (lines across chunks, long lines, no final newline) for the
    non-default paths too."""
    ctx.set_option("grep_sort_hits", sort_hits)
    ctx.set_option("grep_emit", emit)
    try:
        files = cases.synthetic_grep(50000, [3_000_000, 1_000_001], 5)
        check(ctx, "grep:distributed", files, nreduces=(1, 10))
        if sort_hits or not emit:
            for name, (gf, pat) in sorted(cases.grep_edge_cases().items()):
                check(ctx, "grep:" + pat.decode("utf-8", "surrogateescape"), gf, nreduces=(4,))
    finally:
        ctx.set_option("grep_sort_hits", 0)
        ctx.set_option("grep_emit", 1)


def test_grep_list_overflow_rerun(ctx):
    """A hit list far smaller than the split's hits (option list_cap): the line
    resolution, which reads the hit count on the device, runs over a truncated
    list; the counter read after it (or, once an earlier split has set the
    speculative sizes, the one after the insert) sees the overflow, and the map
    repeats with a larger list.  Then a split with far more line bytes than the
    previous one (the speculative record arena overflows and the insert runs
    again with the exact size) — exact output every time."""
    files = cases.synthetic_grep(50000, [2_000_000], 8, match_rate=0.05)
    small = cases.synthetic_grep(5000, [20_000], 9, match_rate=0.02)
    big = cases.synthetic_grep(50000, [6_000_000], 10, match_rate=0.6)
    ctx.set_option("list_cap", 500)
    try:
        check(ctx, "grep:distributed", files, nreduces=(10,))
        assert gpu_partitioned(ctx, "grep:distributed", small, 10) == O.c_partitioned("grep:distributed", small, 10)
        ctx.set_option("list_cap", 500)  # (the sizes of `small` are now the speculative ones)
        assert gpu_partitioned(ctx, "grep:distributed", files, 10) == O.c_partitioned("grep:distributed", files, 10)
        assert gpu_partitioned(ctx, "grep:distributed", small, 10) == O.c_partitioned("grep:distributed", small, 10)
        assert gpu_partitioned(ctx, "grep:distributed", big, 10) == O.c_partitioned("grep:distributed", big, 10)
    finally:
        ctx.set_option("list_cap", 0)


def test_wc_lds_overflow_and_table_growth(ctx):
    """Force the HBM paths: tiny HBM table (growth + re-run) and a corpus whose
    distinct keys overflow every workgroup's LDS table."""
    files = cases.synthetic(C.KIND_ASCII, 2_000_000, [8_000_000], 9)
    ctx.set_option("short_table_log2", 10)
    try:
        check(ctx, "wc", files, nreduces=(10,))
        st = ctx.stats()
        assert st["lds_overflow"] > 0
    finally:
        ctx.set_option("short_table_log2", 0)


DEFAULT_SPILL_BUCKETS = 256  # mrgpu_internal.h kSpillBucketsLo


@pytest.mark.parametrize("nb", [0, 512, 2048])
def test_wc_spill_region_full(wctx, nb):
    """Tiny spill streams: they overflow and the rest of their keys take the HBM-table path
    (those buckets then merge through the HBM table instead of emitting directly), in
    the default (256 buckets), the 512-bucket and the high-cardinality (2048-bucket,
    12-wave) layouts."""
    files = cases.synthetic(C.KIND_ASCII, 1_000_000, [6_000_000], 15)
    wctx.set_option("spill_stream_keys", 8 if nb == 0 else 2)  # (2048 buckets: ~0.5 records per stream)
    wctx.set_option("spill_buckets", nb)
    try:
        check(wctx, "wc", files, nreduces=(10,))
        assert wctx.stats()["spill_ovf"] > 0
        assert wctx.stats()["spill_buckets"] == (nb or DEFAULT_SPILL_BUCKETS)
    finally:
        wctx.set_option("spill_stream_keys", 0)
        wctx.set_option("spill_buckets", 0)


def test_wc_record_buffer_growth(wctx):
    """A record buffer far too small for the distinct keys: the map grows it and re-runs."""
    files = cases.synthetic(C.KIND_ASCII, 200_000, [3_000_000], 17)
    wctx.set_option("rec_cap", 64)
    try:
        check(wctx, "wc", files, nreduces=(10,))
    finally:
        wctx.set_option("rec_cap", 0)


@pytest.mark.parametrize("rounds,big", [(0, 0), (1, 0), (2, 0), (0, 2), (0, -1), (3, -1)])
def test_wc_bucket_aggregator_overflow(ctx, rounds, big):
    """More distinct spilled keys per bucket than the aggregator's LDS table holds:
    misses carried through further aggregation rounds (default), counted in the
    HBM table right away (1 round), or after one carried round (2)."""
    voc = C.Vocab(C.KIND_ASCII, 1.07, 3_000_000, 16)  # every word of a 3M vocabulary at least once
    files = [bytes(voc.fill_files([26_000_000], [16], C.wc_params(vocab_lo=0, vocab_hi=3_000_000))[0])]
    ctx.set_option("agg_rounds", rounds)
    ctx.set_option("agg_carry_min", -1)  # carry every miss (default: < 64 per bucket settle in HBM)
    # big = 0: 1024-thread tables in every round; -1: 512-thread tables in every
    # round; 2: 512-thread round 0, 1024-thread later rounds (the 512-bucket default)
    ctx.set_option("agg_big0", -1 if big != 0 else 1)
    ctx.set_option("agg_big_later", -1 if big < 0 else 0)
    try:
        check(ctx, "wc", files, nreduces=(10,))
        st = ctx.stats()
        assert st["agg_miss"] > 0
        assert st["agg_rounds"] == (rounds if rounds else st["agg_rounds"])
        if rounds == 0:
            assert st["agg_rounds"] > 1
        ctx.set_option("agg_carry_min", 4096)  # buckets with < 4096 misses settle them in HBM
        check(ctx, "wc", files, nreduces=(10,))
    finally:
        ctx.set_option("agg_rounds", 0)
        ctx.set_option("agg_carry_min", 0)
        ctx.set_option("agg_big0", 0)
        ctx.set_option("agg_big_later", 0)


@pytest.mark.parametrize("rounds,stage", [(0, -1), (1, -1), (0, 1), (1, 1)])
def test_wc_high_cardinality_buckets(ctx, rounds, stage):
    """2048 spill buckets (high-cardinality layout: 12-wave map workgroups, 4x
    the aggregator workgroups; stage 1: the 1088-key mini dictionary, 16-wave
    workgroups write-combining the 8-byte streams in LDS), forced and chosen by the feedback
    rule: exact on a 3M-word vocabulary, in rounds or with every miss counted in HBM."""
    voc = C.Vocab(C.KIND_ASCII, 1.07, 3_000_000, 16)
    files = [bytes(voc.fill_files([26_000_000], [16], C.wc_params(vocab_lo=0, vocab_hi=3_000_000))[0])]
    ctx.set_option("agg_rounds", rounds)
    ctx.set_option("hi_stage", stage)
    ctx.set_option("spill_buckets", 2048)
    try:
        check(ctx, "wc", files, nreduces=(10,))
        assert ctx.stats()["spill_buckets"] == 2048
        ctx.set_option("spill_buckets", 0)
        ctx.set_option("spill_hi_keys", 1_000_000)  # the feedback rule: this split has ~2.4M spilled keys
        gpu_partitioned(ctx, "wc", files, 10)  # decides the next split's bucket count
        got = gpu_partitioned(ctx, "wc", files, 10)
        assert got == O.c_partitioned("wc", files, 10)
        assert ctx.stats()["spill_buckets"] == 2048  # chosen from the previous split
        ctx.set_option("spill_hi_keys", 1 << 40)
        gpu_partitioned(ctx, "wc", files, 10)
        gpu_partitioned(ctx, "wc", files, 10)
        assert ctx.stats()["spill_buckets"] == DEFAULT_SPILL_BUCKETS
    finally:
        ctx.set_option("agg_rounds", 0)
        ctx.set_option("spill_buckets", 0)
        ctx.set_option("spill_hi_keys", 0)
        ctx.set_option("hi_stage", 0)


@pytest.mark.parametrize("case", ["tiny_streams", "host_pieces", "utf8_long"])
def test_wc_staged_spill(ctx_dict, case):
    """The write-combined 2048-bucket map (hi_stage): every 8-byte spill record
    goes through a stream's 4-record LDS group or straight to memory, and the
    groups are flushed after each workgroup round and at the end.  Tiny streams
    (groups reaching past a stream's capacity, the rest through the HBM table),
    host input mapped piece by piece (resumed launches: cursors and groups carry
    over), and mixed-script text with long words; all exact, with the dictionary
    option on (the staged kernel's mini dictionary: 1024 short + 64 mid keys, built
    from the same sample; its hits are counted)."""
    c = ctx_dict
    c.set_option("spill_buckets", 2048)
    c.set_option("hi_stage", 1)
    try:
        if case == "tiny_streams":
            files = cases.synthetic(C.KIND_ASCII, 1_000_000, [6_000_000], 15)
            c.set_option("spill_stream_keys", 6)
            check(c, "wc", files, nreduces=(10,))
            assert c.stats()["spill_ovf"] > 0
        elif case == "host_pieces":
            files = cases.synthetic(C.KIND_ASCII, 500_000, [9_000_001, 8_000_000, 7_000_003], 73)
            joined = b"\n".join(files)
            c.set_option("ingest_piece", 1 << 20)
            c.set_option("ingest_min", 1 << 20)
            assert c.run_job(MRG_APP_WC, joined, nreduce=10) == O.c_partitioned("wc", files, 10)
            assert c.stats()["staged_bytes"] == len(joined)
        else:
            files = cases.synthetic(C.KIND_UTF8, 300_000, [5_000_000, 3_000_001], 74, 0.0005) + \
                [cases.long_words(2_000_000, 3)]
            check(c, "wc", files, nreduces=(1, 10))
            gpu_partitioned(c, "wc", files[:1], 10)  # (the long-word file alone has no dictionary hits)
        assert c.stats()["spill_buckets"] == 2048 and c.stats()["dict_hits"] > 0
        # the next split of the context: the kept mini image is re-checked on its sample
        check(c, "wc", files[:1], nreduces=(10,))
    finally:
        for k in ("spill_buckets", "hi_stage", "spill_stream_keys", "ingest_piece", "ingest_min"):
            c.set_option(k, 0)


@pytest.mark.parametrize("digit_bits,fold,grep_k1,compact,own",
                         [(8, 0, 0, 0, 1), (8, -1, 0, -1, 1), (10, 0, 0, 0, 0), (10, -1, -1, -1, 0), (8, 0, -1, 0, 1),
                          (10, -1, 0, 0, 1)])
def test_reduce_sort_variants(ctx, digit_bits, fold, grep_k1, compact, own):
    """The reduce's sort variants give the same bytes: the hand-written radix
    passes with 8-bit (default) or 10-bit digits (own_sort=0 is kept as an
    alias: the same passes since rocPRIM left),
    the partition folded into the first key pass (default) or sorted on its own,
    grep lines radix-sorted on 16 key bytes (default) or 8 (more tied runs), tied
    runs merge-sorted on compact key copies (default) or on the records.
    The corpus has 8-byte keys differing only in their last byte's low bits (ties
    of the folded key), 9-16-byte keys sharing 8-byte prefixes, long keys and UTF-8."""
    base = [b"abcdefg" + bytes([c]) for c in range(ord("a"), ord("z") + 1)]
    base += [b"abcdefgh" + bytes([c]) * k for c in range(ord("a"), ord("p")) for k in (1, 3, 8, 20)]
    words = b" ".join(base * 3) + b"\n"
    files = [words] + cases.synthetic(C.KIND_UTF8, 30000, [2_000_000, 700_001], 41, 0.001)
    ctx.set_option("sort_digit_bits", digit_bits)
    ctx.set_option("sort_fold_part", fold)
    ctx.set_option("grep_sort_k1", grep_k1)
    ctx.set_option("sort_compact_ties", compact)
    ctx.set_option("own_sort", own)
    try:
        check(ctx, "wc", files, nreduces=(1, 10, 64))
        check(ctx, "wc", [words, words[::-1]], nreduces=(1, 10, 300))  # ASCII only: the packed sort key
        check(ctx, "grep:distributed", cases.synthetic_grep(20000, [1_500_000], 42), nreduces=(1, 10))
    finally:
        ctx.set_option("sort_digit_bits", 0)
        ctx.set_option("sort_fold_part", 0)
        ctx.set_option("grep_sort_k1", 0)
        ctx.set_option("sort_compact_ties", 0)
        ctx.set_option("own_sort", 1)


@pytest.mark.parametrize("tie_rank", [1, 0])
def test_grep_tied_runs(ctx, tie_rank):
    """grep lines tied on their first 16 bytes, ordered per run by rank (default:
    waves for runs <= 64 keys, a workgroup's bitonic sort for 65-2048, the merge
    sort beyond) or all merge-sorted (tie_rank=0): one prefix shared by 3000
    distinct lines (R=1: a run over 2048; R=10: ~300 per partition), 40 prefixes
    x 50 lines, pairs; suffixes that differ only past byte 64, NUL bytes, UTF-8,
    lines that are prefixes of each other."""
    rnd = np.random.default_rng(11)
    lines = set()
    big = b"distributed sys "  # 16 bytes
    while len(lines) < 3000:
        tail = bytes(rnd.integers(32, 127, size=int(rnd.integers(0, 90))).astype(np.uint8))
        lines.add(big + tail)
    for k in range(40):
        pre = b"distributed %03d " % k + b"x" * 0  # 16 bytes
        for _ in range(50):
            lines.add(pre + bytes(rnd.integers(40, 44, size=int(rnd.integers(0, 6))).astype(np.uint8)))
    far = b"distributed far " + b"y" * 48  # equal through byte 63
    for _ in range(300):
        lines.add(far + bytes(rnd.integers(0, 3, size=int(rnd.integers(0, 40))).astype(np.uint8)).replace(b"\n", b""))
    for k in range(500):
        lines.add(b"distributed pair%05d" % k)
        lines.add(b"distributed pair%05d\xc3\xa9" % k)
    ls = sorted(lines)
    rnd.shuffle(ls)
    text = b"\n".join(ls) + b"\n"
    ctx.set_option("tie_rank", tie_rank)
    try:
        check(ctx, "grep:distributed", [text, text[: len(text) // 2] + b"\n"], nreduces=(1, 10))
    finally:
        ctx.set_option("tie_rank", 1)


@pytest.mark.parametrize("tie_rank", [1, 0])
def test_grep_log_prefix_runs(ctx, tie_rank):
    """Log-like grep input: 150 000 matching lines behind one 24-byte timestamp
    prefix (one tied run of 150 000 at nReduce=1: listed as 4096-key pieces and
    merge-sorted), plus 20 000 behind another and runs just over and under the
    2048-key mid-run limit; and wc over 3 000 distinct 40-letter words sharing
    their first 32 letters (a tied run far over 64 keys after the 16-byte key
    pass: its members past the first 65 marked by the 64-wide window kernel)."""
    rnd = np.random.default_rng(23)
    lines = []
    for pre, k in ((b"2026-10-17T08:00:00 INFO distributed", 150_000), (b"2026-10-17T08:00:01 WARN distributed", 20_000),
                   (b"2026-10-17T08:00:02 INFO distributed", 2049), (b"2026-10-17T08:00:03 INFO distributed", 2048)):
        ids = rnd.permutation(k * 4)[:k]
        lines += [pre + b" req=%07d" % i for i in ids]
    rnd.shuffle(lines)
    text = b"\n".join(lines) + b"\n"
    ctx.set_option("tie_rank", tie_rank)
    try:
        check(ctx, "grep:distributed", [text], nreduces=(1, 7))
    finally:
        ctx.set_option("tie_rank", 1)
    base = b"q" * 32
    words = sorted({base + bytes(rnd.integers(97, 123, size=8).astype(np.uint8)) for _ in range(3000)})
    rnd.shuffle(words)
    check(ctx, "wc", [b" ".join(words * 2) + b"\n"], nreduces=(1,))


@pytest.mark.parametrize("own", [1, 0])
@pytest.mark.parametrize("kind,bits", [("u32", 32), ("u32", 4), ("u32", 20), ("u64", 64), ("u64", 60), ("u64", 12),
                                       ("u64keys", 34), ("u64keys", 64)])
def test_radix_sort_hook(ctx, own, kind, bits):
    """The reduce's radix sort (mrg_sort_pairs) against numpy's stable argsort:
    sizes around the 4096-key tile (0, 1, 4095, 4096, 4097), 1e5 keys, and 3e6
    (733 tiles: more than can be resident at once, so the look-back waits on
    tiles started later); uniform keys, keys from 5 values (ties: stability),
    all keys equal, high bits set past `bits` (ignored by the sort); 8-bit
    radix digits (default) and 10-bit ones (option sort_digit_bits = 10)."""
    rng = np.random.default_rng(bits * 7 + own)
    dt = np.uint32 if kind == "u32" else np.uint64
    width = 32 if kind == "u32" else 64
    mask = (1 << bits) - 1 if bits < width else (1 << width) - 1
    ctx.set_option("own_sort", own)
    try:
      for digit_bits in (0, 10):
        ctx.set_option("sort_digit_bits", digit_bits)
        for n in (0, 1, 4095, 4096, 4097, 100_000, 3_000_000):
            for dist in ("uniform", "few", "equal"):
                if n >= 3_000_000 and dist != "uniform":
                    continue
                if dist == "uniform":
                    keys = rng.integers(0, 1 << width, size=n, dtype=np.uint64 if width == 64 else np.int64).astype(dt)
                elif dist == "few":
                    keys = rng.choice(np.array([0, 3, mask, mask >> 1, 1 << (bits - 1)], dtype=np.uint64),
                                      size=n).astype(dt)
                else:
                    keys = np.full(n, mask & 0x5A5A5A5A5A5A5A5A, dtype=dt)
                masked = keys & dt(mask)
                order = np.argsort(masked, kind="stable")
                if kind == "u64keys":
                    ko, _ = ctx.sort_pairs(keys, None, bits)
                    assert np.array_equal(ko, keys[order]), (n, dist)
                else:
                    vals = np.arange(n, dtype=np.uint32)
                    ko, vo = ctx.sort_pairs(keys, vals, bits)
                    assert np.array_equal(vo, order.astype(np.uint32)), (n, dist)
                    assert np.array_equal(ko, keys[order]), (n, dist)
    finally:
        ctx.set_option("own_sort", 1)
        ctx.set_option("sort_digit_bits", 0)


@pytest.mark.parametrize("bins,prefix32", [(1, 1), (0, 1), (0, 0)])
def test_reduce_bucketed_sort(ctx, bins, prefix32):
    """The wc reduce's key pass variants: the hand-written sample sort (option
    sort_bins=1), rocPRIM on the key's top 32 bits (the default: ties of the
    first ~4 characters ordered by full comparison) and rocPRIM on the whole
    60/64-bit key (sort_prefix32=0): splitters from a sorted sample, a skewed input
    (20 000 distinct words starting with 'q'), > 8192 keys tied on their first 8
    bytes (an overflowing bin: the rocPRIM fallback), ties of the packed / folded key,
    UTF-8 keys (the folded key), 1e5+ distinct keys."""
    rnd = np.random.default_rng(7)
    qwords = [b"q" + bytes(rnd.integers(97, 123, size=int(rnd.integers(1, 12))).astype(np.uint8)) for _ in range(20000)]
    # 10 000 keys tied on their first 8 bytes: one sample-sort bin of > 8192 equal
    # sort keys (the pass falls back to rocPRIM) and a long tied run
    tied = [b"abcdefgh" + bytes(rnd.integers(97, 123, size=int(rnd.integers(1, 8))).astype(np.uint8)) for _ in range(10000)]
    skew = b" ".join(qwords + tied) + b"\n"
    files = [skew] + cases.synthetic(C.KIND_ASCII, 300000, [3_000_000], 43) + \
        cases.synthetic(C.KIND_UTF8, 100000, [2_000_000], 44, 0.001)
    ctx.set_option("sort_bins", bins)
    ctx.set_option("sort_prefix32", prefix32)
    try:
        check(ctx, "wc", files, nreduces=(1, 10, 64))
        check(ctx, "wc", [skew], nreduces=(1, 2))
    finally:
        ctx.set_option("sort_bins", 0)
        ctx.set_option("sort_prefix32", 1)


def test_wc_large_vs_oracle(wctx):
    """64 MB C2-style corpus: full bytes vs the C oracle."""
    voc = C.Vocab(C.KIND_ASCII, 1.07, 10**6, 2)
    files = [bytes(f) for f in voc.fill_files([16_000_000] * 4, [2000 + i for i in range(4)], C.wc_params())]
    check(wctx, "wc", files, nreduces=(10,))


def test_run_job_device_resident(ctx):
    """mrg_run_job over an HBM-resident buffer == per-file map + merge + reduce."""
    files = cases.synthetic(C.KIND_ASCII, 100000, [3_000_000, 2_000_000], 12)
    joined = b"\n".join(files)  # '\n' ends every file's last word/line: identical to per-file splits
    d = ctx.device_alloc(len(joined))
    try:
        ctx.h2d(d, joined)
        got = ctx.run_job(MRG_APP_WC, device_ptr=d, nbytes=len(joined), nreduce=10)
    finally:
        ctx.device_free(d)
    assert got == O.c_partitioned("wc", files, 10)


def test_export_import_reduce_task(ctx):
    """worker.go flow: map task X -> intermediate mr-X-r (export) -> reduce task r (import, merge, reduce)."""
    files = cases.synthetic(C.KIND_UTF8, 30000, [700_000, 900_000, 500_000], 13)
    R = 5
    inter = {}
    for x, f in enumerate(files):
        p = ctx.map(MRG_APP_WC, f, nreduce=R)
        for r in range(R):
            inter[(x, r)] = ctx.export(p, r)
        p.free()
    want = O.c_partitioned("wc", files, R)
    for r in range(R):
        acc = None
        for x in range(len(files)):
            q = ctx.import_(inter[(x, r)])
            if acc is None:
                acc = q
            else:
                ctx.merge(acc, q)
                q.free()
        assert ctx.reduce(acc, r) == want[r]
        acc.free()


def test_exchange_single_rank(ctx):
    """mrg_exchange with one rank (no communicator) keeps every key."""
    files = cases.synthetic(C.KIND_ASCII, 5000, [400_000], 14)
    p = ctx.map(MRG_APP_WC, files[0], nreduce=4)
    q = ctx.exchange(p)
    assert ctx.reduce_all(q) == O.c_partitioned("wc", files, 4)


def test_exchange_rccl_one_rank():
    """mrg_comm_init + mrg_exchange / mrg_run_job with a 1-rank RCCL communicator
    (RCCL refuses two ranks on one GPU; the P > 1 pack / unpack path is covered
    by test_exchange_group_multi_rank)."""
    from mrgpu import Context
    files = cases.synthetic(C.KIND_UTF8, 20000, [600_000], 17, 0.001)
    with Context(0) as c2:
        c2.comm_init(Context.unique_id(), 1, 0)
        p = c2.map(MRG_APP_WC, files[0], nreduce=6)
        q = c2.exchange(p)
        assert c2.reduce_all(q) == O.c_partitioned("wc", files, 6)
        assert c2.run_job(MRG_APP_WC, files[0], nreduce=6) == O.c_partitioned("wc", files, 6)


@pytest.mark.parametrize("app,R", [("wc", 6), ("wc", 64), ("grep:distributed", 10), ("wc-hi", 64)])
def test_exchange_rccl_collectives_one_rank(app, R):
    """The RCCL collectives of mrg_exchange themselves (ncclAllToAll of the
    P x 2 counts, then one group of two ncclAllToAllv: records and long-key
    bytes) on a one-rank communicator (option exch_force_rccl): every key comes
    back through RCCL, unpacked and re-aggregated, exact against the oracle.
    Long UTF-8 keys put bytes in the arena stream too."""
    from mrgpu import Context
    name, pat = (app.split(":") + [None])[:2]
    hi = name == "wc-hi"  # C5's shape: the staged 2048-bucket map, ~10^6 distinct keys
    if hi:
        name, app = "wc", "wc"
        voc = C.Vocab(C.KIND_ASCII, 0.8, 2_000_000, 31)
        files = [bytes(voc.fill_files([12_000_000], [31], C.wc_params(vocab_lo=0, vocab_hi=2_000_000))[0])]
    else:
        files = cases.synthetic(C.KIND_UTF8, 20000, [700_000], 29, 0.001)
    if pat:  # matching lines, some tied on their first bytes
        lines = files[0].split(b"\n")
        for i in range(0, len(lines), 37):
            lines[i] += b" distributed"
        files = [b"\n".join(lines)]
    want = O.c_partitioned(app, files, R)
    assert sum(len(w) for w in want) > 0
    with Context(0) as c2:
        c2.comm_init(Context.unique_id(), 1, 0)
        c2.set_option("exch_force_rccl", 1)
        if hi:
            c2.set_option("spill_buckets", 2048)
            c2.set_option("hi_stage", 1)
        kind = MRG_APP_WC if name == "wc" else MRG_APP_GREP
        p = c2.map(kind, files[0], nreduce=R, **({"pattern": pat.encode()} if pat else {}))
        if hi:
            assert c2.stats()["spill_buckets"] == 2048
        q = c2.exchange(p)
        st = c2.stats()
        assert st["rccl_nranks"] == 1 and st["rccl_rank"] == 0
        assert st["exchange_a2a_ms"] > 0 and st["shuffle_recv_records"] > 0
        assert c2.reduce_all(q) == want
        p.free()
        q.free()


@pytest.mark.parametrize("P,app,R", [(2, "wc", 10), (3, "wc", 64), (4, "grep:distributed", 10), (8, "wc", 64)])
def test_exchange_group_multi_rank(P, app, R):
    """The P > 1 shuffle (owner counts, pack per owner, all-to-all, unpack with the
    sources' arena displacements, exact re-aggregation on the owner) with P
    contexts on one device (mrg_exchange_group: peer copies where mrg_exchange
    uses RCCL; everything else is the same code).  Rank i maps its own splits;
    partition r comes from owner r % P and must equal the oracle's mr-out-r over
    all ranks' inputs.  Long words (> 16 B, arena bytes) and UTF-8 included."""
    from mrgpu import Context
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    pat = b"" if app == "wc" else app[5:].encode("utf-8", "surrogateescape")
    files = []
    for i in range(P):
        if app == "wc":
            f = cases.synthetic(C.KIND_UTF8, 20000, [200_000 + 37_000 * i], 40 + i, 0.001)[0]
            f = f + b" " + b"longword" * (3 + i) + b" " + b"Z" * (17 + i) + b"\n"
        else:
            voc = C.Vocab(C.KIND_UTF8, 1.07, 20000, 50 + i)
            f = bytes(voc.fill_files([150_000], [60 + i], C.grep_params(match_rate=0.03))[0])
        files.append(f)
    want = O.c_partitioned(app, files, R)
    ctxs = [Context(0) for _ in range(P)]
    try:
        local = [ctxs[i].map(a, files[i], pattern=pat, nreduce=R) for i in range(P)]
        owned = Context.exchange_group(ctxs, local)
        for i in range(P):
            out = ctxs[i].reduce_all(owned[i])
            for r in range(R):
                assert out[r] == (want[r] if r % P == i else b""), f"rank {i} partition {r}"
        for q in local + owned:
            q.free()
    finally:
        for c in ctxs:
            c.close()


def test_export_matches_host_codec(ctx):
    """mrg_parts_export bytes decode (mrgpu.intermediate) to the oracle's word counts."""
    import collections
    from mrgpu import intermediate as I
    files = cases.synthetic(C.KIND_UTF8, 20000, [300_000], 18, 0.001)
    p = ctx.map(MRG_APP_WC, files[0], nreduce=7)
    d = I.decode(ctx.export(p))
    want = collections.Counter(O.mr_oracle.wc_map(files[0]))
    assert dict(zip(d["keys"], (int(c) for c in d["count"]))) == dict(want)
    assert all(int(pp) == O.c_ihash(k) % 7 for k, pp in zip(d["keys"], d["kpart"]))


@pytest.fixture(scope="module")
def ctx_sorted_hits():
    """grep with option grep_sort_hits = 1 (hits sorted by position before the
    line resolution: the round-4 path)."""
    from mrgpu import Context
    c = Context(0)
    c.set_option("grep_sort_hits", 1)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_grep_radix():
    """grep reduce by the radix passes + tie ranking + line writer (option
    grep_bins = 0; the default is the bucketed sort fused with the output)."""
    from mrgpu import Context
    c = Context(0)
    c.set_option("grep_bins", 0)
    yield c
    c.close()


@pytest.mark.parametrize("name", ["basic", "tied_lines", "long_lines_many_hits", "chunk_seams", "overlapping",
                                  "prefix5_utf8"])
def test_grep_edge_cases_radix_reduce(ctx_grep_radix, name):
    files, pat = cases.grep_edge_cases()[name]
    check(ctx_grep_radix, "grep:" + pat.decode("utf-8", "surrogateescape"), files, nreduces=(1, 10))


@pytest.mark.parametrize("mode", [3, 2])
def test_grep_bins_many_lines(mode):
    """The bucketed grep reduce over ~3 x 10^5 distinct matching lines (hundreds of
    bins, partitions R = 1 / 10 / 64 / 1000, some empty), tied 16-byte prefixes,
    lines of 1-3000 bytes, against the oracle; mode 3: the sorting workgroups
    write the lines (the default for host output); mode 2: bins sorted, then
    the line writer."""
    import random
    from mrgpu import Context
    rnd = random.Random(5)
    lines = []
    for i in range(300_000):  # > 262 144 distinct lines: 8192 splitter samples (the register-blocked sort)
        k = rnd.random()
        if k < 0.3:    # shared 24-byte prefix: ties past the entries' first 24 bytes
            lines.append(b"distributed systems are h" + str(rnd.randrange(10**6)).encode())
        elif k < 0.35:  # long lines
            lines.append(b"x" * rnd.randrange(100, 3000) + b"distributed" + str(i).encode())
        else:
            lines.append(bytes(rnd.choice(b"abcdefgh ") for _ in range(rnd.randrange(0, 40))) + b"distributed"
                         + bytes(rnd.choice(b"xyz") for _ in range(rnd.randrange(0, 8))))
    data = b"\n".join(lines) + b"\n"
    with Context(0) as c:
        c.set_option("grep_bins", mode)
        check(c, "grep:distributed", [data], nreduces=(1, 10, 64, 1000))
        # a Zipf-frequent first word: > 4096 lines share their first 8 bytes
        # (one bin per 128-bit key prefix, not per 8-byte one)
        many = b"".join(b"fzlsGaIu distributed %07d\n" % rnd.randrange(10**7) for _ in range(20000))
        check(c, "grep:distributed", [many], nreduces=(1, 10))


@pytest.mark.parametrize("bins", [1, -1])
def test_grep_bins_host_output_many_lines(bins):
    """mrg_run_job's default grep output, lines written into pinned host memory
    by the workgroups that sort the bins, over ~10^5 distinct matching lines
    (~400 bins), with the previous reduce's splitters reused (1) or sampled
    afresh (-1): tied prefixes, long lines, R = 1 / 10 / 64, and a split whose
    one tied prefix overflows the bins (the radix path redoes it), then the
    first split again."""
    import random
    from mrgpu import Context
    rnd = random.Random(11)
    lines = []
    for i in range(100_000):
        k = rnd.random()
        if k < 0.3:
            lines.append(b"distributed systems are h" + str(rnd.randrange(10**6)).encode())
        elif k < 0.33:
            lines.append(b"y" * rnd.randrange(100, 2000) + b"distributed" + str(i).encode())
        else:
            lines.append(bytes(rnd.choice(b"abcdefgh ") for _ in range(rnd.randrange(0, 40))) + b"distributed"
                         + bytes(rnd.choice(b"xyz") for _ in range(rnd.randrange(0, 8))))
    data = b"\n".join(lines) + b"\n"
    many = b"".join(b"distributed tied prefix, one bin %07d\n" % rnd.randrange(10**7) for _ in range(9000))
    with Context(0) as c:
        c.set_option("grep_bins", bins)
        try:
            for d in (data, many, data):
                for R in (1, 10, 64):
                    assert c.run_job(MRG_APP_GREP, d, pattern=b"distributed", nreduce=R) == \
                        O.c_partitioned("grep:distributed", [d], R), (bins, R, len(d))
        finally:
            c.set_option("grep_bins", 1)


def test_grep_bins_splitter_reuse():
    """A context reuses its last grep reduce's splitters for a reduce of similar
    size: a split whose lines sort nothing like the previous one's (every line
    beyond the old splitters: one bin far past the LDS sort) is still exact (the
    bin is flagged and the radix path redoes the reduce), and the context then
    samples afresh."""
    import random
    from mrgpu import Context
    rnd = random.Random(9)

    def corpus(first: bytes):
        return b"".join(first + bytes(rnd.choice(b"abcdefghij") for _ in range(rnd.randrange(5, 30)))
                        + b" distributed " + str(i).encode() + b"\n" for i in range(60_000))
    a, z = corpus(b"a"), corpus(b"zz")
    with Context(0) as c:
        for R in (1, 7):
            for data in (a, z, z, a):
                got = c.run_job(MRG_APP_GREP, data, pattern=b"distributed", nreduce=R)
                assert got == O.c_partitioned("grep:distributed", [data], R)


@pytest.mark.parametrize("path", ["default", "sorted"])
def test_grep_record_counts_one_per_line(ctx, ctx_sorted_hits, path):
    """The map's grep records count every matching line occurrence exactly once
    (dgrep.go:30-33 emits one KeyValue per line; mr-X-r holds that many JSON
    lines): lines crossing chunk seams with hits on both sides, lines over
    three chunks, > 4 KiB lines with hits in many chunks, every grep edge case.
    The counts come from mrg_parts_export (mrgpu.intermediate)."""
    import collections

    import mr_oracle as M
    from mrgpu import intermediate as I
    c = ctx if path == "default" else ctx_sorted_hits
    todo = [("seam_lines", [cases.grep_seam_lines()], b"distributed"),
            ("seam_lines_e", [cases.grep_seam_lines(b"e")], b"e")]
    todo += [(k, f, p) for k, (f, p) in cases.grep_edge_cases().items()]
    for name, files, pat in todo:
        for f in files:
            parts = c.map(MRG_APP_GREP, f, pattern=pat, nreduce=5)
            d = I.decode(c.export(parts))
            parts.free()
            got = collections.Counter()
            for k, n in zip(d["keys"], d["count"]):
                got[k] += int(n)
            want = collections.Counter(M.grep_map(f, pat))
            assert got == want, f"{name}: {sum(got.values())} records vs {sum(want.values())} matching lines"


def test_export_json_grep_seam_lines(ctx):
    """mr-X-r JSON lines of grep on the default path for seam-crossing lines
    with hits on both sides: one line per matching line occurrence
    (worker.go:80-92), as the reference map worker writes them."""
    import mr_oracle as M
    files = [cases.grep_seam_lines()]
    R = 4
    p = ctx.map(MRG_APP_GREP, files[0], pattern=b"distributed", nreduce=R)
    for r in range(R):
        got = ctx.export_json(p, r)
        assert sorted(got.splitlines(keepends=True)) == sorted(
            M.intermediate_json_lines("grep:distributed", files, R, r)), f"partition {r}"
    p.free()


JSON_GREP_LINES = (b'plain distributed line\n'
                   b'quote " and backslash \\ distributed <b>&amp;</b>\n'
                   b'ctrl \x01\x08\x0c\t\r distributed\n'
                   + "unicode distributed \u00e9\u4e2d\U0001F600 \u2028 \u2029 x\n".encode()
                   + b'invalid \xff\xe2\x80 distributed\n'
                   + b'distributed\n' * 3 + b'short distributed\n' * 2)


@pytest.mark.parametrize("app", ["wc", "grep:distributed"])
def test_export_json_matches_reference_format(ctx, app):
    """mrg_parts_export_json: the lines mr/worker.go:80-92 writes to mr-X-r (one per
    occurrence, Go's json.Encoder escaping), as a multiset, for every partition."""
    import mr_oracle as M
    if app == "wc":
        files = cases.synthetic(C.KIND_UTF8, 3000, [60_000], 31, 0.002)
        files.append(b"Zzzzzzzzzzzzzzzzzzzzzz " * 3 + b"\n")
    else:
        files = [JSON_GREP_LINES * 3]
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    pat = b"" if app == "wc" else app[5:].encode("utf-8", "surrogateescape")
    R = 7
    p = ctx.map(a, b"\n".join(files), pattern=pat, nreduce=R)
    allj = []
    for r in range(R):
        got = ctx.export_json(p, r)
        want = M.intermediate_json_lines(app, files, R, r)
        assert sorted(got.splitlines(keepends=True)) == sorted(want), f"partition {r}"
        allj.append(got)
    assert sorted(ctx.export_json(p).splitlines(keepends=True)) == sorted(
        l for r in range(R) for l in M.intermediate_json_lines(app, files, R, r))
    p.free()


@pytest.mark.parametrize("app", ["wc", "grep:distributed"])
def test_import_json_reference_intermediates(ctx, app):
    """mrg_parts_import_json over mr-X-Y files as reference map workers write them
    (oracle encoder), then the GPU reduce: mr-out-r equals the reference's reduce
    of the decoded keys (worker.go:100-146; invalid UTF-8 in a grep line comes back
    as U+FFFD, the reference's own JSON round trip)."""
    import json

    import mr_oracle as M
    if app == "wc":
        files = cases.synthetic(C.KIND_UTF8, 3000, [50_000, 30_000], 32, 0.002)
    else:
        files = [JSON_GREP_LINES * 2, JSON_GREP_LINES]
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    R = 5
    _, reducef = M._map_reduce_fns(app)
    for r in range(R):
        data = b"".join(l for f in files for l in M.intermediate_json_lines(app, [f], R, r)[::-1])  # any line order
        parts = ctx.import_json(a, R, data)
        keys = [json.loads(l)["Key"].encode("utf-8") for l in data.splitlines()]
        want = M._group_reduce([k for k in keys if M.ihash(k) % R == r], reducef)
        assert ctx.reduce(parts, r) == want, f"partition {r}"
        parts.free()
    empty = ctx.import_json(a, R, b"")
    assert ctx.reduce(empty, 0) == b""
    empty.free()
    with pytest.raises(Exception):
        ctx.import_json(a, R, b'{"Key":"x"}\n')


def test_import_rejects_malformed(ctx):
    """mrg_parts_import checks every record before it reaches the device
    (a corrupt intermediate must be MRG_EFORMAT, never an
    out-of-bounds read or a record in the wrong partition)."""
    import struct

    from mrgpu import MrgError
    from mrgpu import intermediate as I
    R = 8
    keys = [b"alpha", b"b" * 16, b"long" * 9, b"q"]
    parts = [O.c_ihash(k) % R for k in keys]
    good = I.encode(MRG_APP_WC, R, keys, [3, 1, 2, 5], parts)
    q = ctx.import_(good)
    assert ctx.reduce_all(q)[parts[0]].count(b"alpha 3\n") == 1
    q.free()
    n = len(keys)
    off_k0, off_cnt, off_koff = I.HDR.size, I.HDR.size + 16 * n, I.HDR.size + 24 * n
    off_len, off_part = I.HDR.size + 32 * n, I.HDR.size + 36 * n

    def put(buf, off, fmt, v):
        b = bytearray(buf)
        struct.pack_into(fmt, b, off, v)
        return bytes(b)

    bad = {
        "partition >= nreduce": put(good, off_part, "<I", R),
        "partition != ihash % R": put(good, off_part, "<I", (parts[0] + 1) % R),
        "inline key > 16 bytes": put(good, off_len + 4, "<I", 17),
        "arena key past the arena": put(good, off_koff + 8 * 2, "<Q", 10**6),
        "arena length past the arena": put(good, off_len + 8, "<I", 10**6),
        "prefix word differs": put(good, off_k0 + 8 * 2, "<Q", 0x4141414141414141),
        "zero count": put(good, off_cnt, "<Q", 0),
        "bytes past inline length": put(good, off_len, "<I", 2),
        "truncated": good[:-3],
        "size lies": put(good, 16, "<Q", 2**62),
    }
    for why, data in bad.items():
        with pytest.raises(MrgError, match="import"):
            ctx.import_(data)
        assert why


# ---------------------------------------------------------------- full-scale splits
GIB = 1 << 30
TILED_TOTAL = 4_500_000_000  # > 2^32: byte offsets past 4 GiB, every 1 GiB descriptor base


def _seam_tiles(app: str) -> list[tuple[bytes, int]]:
    """(tile, cut): tile = '\\n' + ... + '\\n'; the 1 GiB boundary falls at byte
    `cut` of the tile, inside a word (wc) or a pattern occurrence (grep)."""
    if app == "wc":
        words = [(b"Xylophonequartzseam", 7), (b"abcdefghijklmnop", 8), (b"seamword", 3), ("ééé".encode(), 3),
                 (b"qz", 1)]
        return [(b"\nleft " + w + b" right\n", 6 + k) for w, k in words]
    return [(b"\nzz distributed seam line\n", 6), (b"\nno match here\ndistributed\n", 15),
            (b"\n" + "é distributed é".encode() + b"\n", 1), (b"\nx distributed y\n", 4),
            (b"\ndistributedness\n", 1)]


def _tiled_device(base: bytes, app: str):
    """base repeated until TILED_TOTAL bytes, with a seam tile placed across every
    1 GiB boundary (and 2^32) and '\\n' padding before it.  Returns the device
    tensor, the number of base tiles and the seam tiles used."""
    import torch
    L = len(base)
    assert base.endswith(b"\n")
    seams = _seam_tiles(app)
    buf = torch.empty(TILED_TOTAL, dtype=torch.uint8, device="cuda:0")
    dbase = torch.frombuffer(bytearray(base), dtype=torch.uint8).to("cuda:0")
    bounds = [j * GIB for j in range(1, TILED_TOTAL // GIB + 1)]
    cur, nb, used = 0, 0, []
    for j, b in enumerate(bounds):
        tile, cut = seams[j % len(seams)]
        start = b - cut
        while cur + L <= start:
            buf[cur:cur + L].copy_(dbase)
            cur += L
            nb += 1
        buf[cur:start].fill_(10)
        buf[start:start + len(tile)].copy_(torch.frombuffer(bytearray(tile), dtype=torch.uint8).to("cuda:0"))
        used.append(tile)
        cur = start + len(tile)
    while cur + L <= TILED_TOTAL:
        buf[cur:cur + L].copy_(dbase)
        cur += L
        nb += 1
    buf[cur:].fill_(10)
    torch.cuda.synchronize()
    return buf, nb, used


def _wc_counts(parts: list[bytes]) -> list[dict]:
    out = []
    for p in parts:
        d = {}
        for line in p.split(b"\n")[:-1]:
            k, c = line.rsplit(b" ", 1)
            d[k] = int(c)
        out.append(d)
    return out


def test_wc_split_past_4gib_vs_oracle(ctx):
    """One 4.5 GB split (SURVEY.md §8c gate at scale): an oracle-checked 32 MB
    corpus tiled ~140 times, plus crafted words straddling every 1 GiB boundary
    and 2^32 (long, 16-byte, short and UTF-8 words).  Expected mr-out-r = the
    base's counts x tiles + the seam tiles' counts, exactly."""
    voc = C.Vocab(C.KIND_ASCII, 1.07, 10**6, 2)
    base = bytes(voc.fill_files([32_000_000], [4242], C.wc_params())[0])
    R = 10
    buf, nb, seams = _tiled_device(base, "wc")
    try:
        got = ctx.run_job(MRG_APP_WC, device_ptr=buf.data_ptr(), nbytes=TILED_TOTAL, nreduce=R)
    finally:
        del buf
    want = _wc_counts(O.c_partitioned("wc", [base], R))
    for r, d in enumerate(_wc_counts(O.c_partitioned("wc", seams, R))):
        for k in want[r]:
            want[r][k] *= nb
        for k, c in d.items():
            want[r][k] = want[r].get(k, 0) + c
    for r in range(R):
        exp = b"".join(k + b" " + str(want[r][k]).encode() + b"\n" for k in sorted(want[r]))
        assert got[r] == exp, f"partition {r}: {len(got[r])} vs {len(exp)} bytes"
    assert b"Xylophonequartzseam 1\n" in got[O.c_ihash(b"Xylophonequartzseam") % R]


def test_grep_split_past_4gib_vs_oracle(ctx):
    """grep over the same kind of 4.5 GB tiled split: occurrences and lines
    straddling every 1 GiB boundary; duplicates of the base's lines collapse, so
    mr-out-r = the oracle's output over [base] + seam tiles."""
    voc = C.Vocab(C.KIND_UTF8, 1.07, 10**5, 3)
    base = bytes(voc.fill_files([32_000_000], [4343], C.grep_params(b"distributed", match_rate=0.01))[0])
    R = 10
    buf, nb, seams = _tiled_device(base, "grep")
    try:
        got = ctx.run_job(MRG_APP_GREP, pattern=b"distributed", device_ptr=buf.data_ptr(), nbytes=TILED_TOTAL,
                          nreduce=R)
    finally:
        del buf
    assert nb > 100
    assert got == O.c_partitioned("grep:distributed", [base] + seams, R)


def _merge_partitioned_wc(outs: list[list[bytes]], R: int) -> list[bytes]:
    """Σ of several oracle wc outputs (same R) -> the oracle output of the union."""
    merged = [dict() for _ in range(R)]
    for out in outs:
        for r, d in enumerate(_wc_counts(out)):
            m = merged[r]
            for k, c in d.items():
                m[k] = m.get(k, 0) + c
    return [b"".join(k + b" " + str(m[k]).encode() + b"\n" for k in sorted(m)) for m in merged]


def _group_job(files: list[bytes], R: int) -> list[list[bytes]]:
    """Rank i maps files[i] on its own context, the P-context shuffle, then every
    owner reduces; returns each rank's mr-out-r list."""
    from mrgpu import Context
    P = len(files)
    ctxs = [Context(0) for _ in range(P)]
    try:
        local = [ctxs[i].map(MRG_APP_WC, files[i], nreduce=R) for i in range(P)]
        owned = Context.exchange_group(ctxs, local)
        outs = [ctxs[i].reduce_all(owned[i]) for i in range(P)]
        st = [c.stats() for c in ctxs]
        for q in local + owned:
            q.free()
        assert all(s["shuffle_send_bytes"] > 0 for s in st)
        return outs
    finally:
        for c in ctxs:
            c.close()


def test_exchange_group_c4_shape():
    """C4's shape (8 ranks, nReduce = 64, C2 generator, 64 MB per rank, seed 4+g):
    owner r % 8 of every partition equals the oracle over all ranks' inputs."""
    from concurrent.futures import ThreadPoolExecutor
    P, R = 8, 64
    voc = C.Vocab(C.KIND_ASCII, 1.07, 10**6, 4)
    files = [bytes(f) for f in voc.fill_files([64_000_000] * P, [4 + g for g in range(P)], C.wc_params())]
    with ThreadPoolExecutor(P) as ex:  # the C oracle releases the GIL
        per = list(ex.map(lambda f: O.c_partitioned("wc", [f], R), files))
    want = _merge_partitioned_wc(per, R)
    outs = _group_job(files, R)
    for i in range(P):
        for r in range(R):
            assert outs[i][r] == (want[r] if r % P == i else b""), f"rank {i} partition {r}"


def test_exchange_group_c5_shape():
    """C5's shape (high cardinality): 4 ranks, each emitting its 3 M-word share of
    a Zipf(0.8, 1.2e7) vocabulary once up front plus sampled words (>= 3 M
    distinct keys per rank), nReduce = 64 — multi-round aggregation on every rank
    and millions of records through the shuffle."""
    P, R, V = 4, 64, 12_000_000
    voc = C.Vocab(C.KIND_ASCII, 0.8, V, 5)
    files = [bytes(voc.fill_files([32_000_000], [5 + g], C.wc_params(vocab_lo=3_000_000 * g,
                                                                      vocab_hi=3_000_000 * (g + 1)))[0])
             for g in range(P)]
    want = O.c_partitioned("wc", files, R)
    outs = _group_job(files, R)
    for i in range(P):
        for r in range(R):
            assert outs[i][r] == (want[r] if r % P == i else b""), f"rank {i} partition {r}"


def test_exchange_group_c5_p8_full_keys():
    """C5's owner side at C5's key counts: 8 ranks, nReduce = 64,
    each rank's split holds EVERY word of the Zipf(0.8, 1e7) vocabulary once (100
    files, each emitting its 1e5-word share up front, as bench.py's C5 corpus) plus
    sampled words, so every rank maps >= 1e7 distinct keys and each owner unpacks
    and re-aggregates ~8 x 1.25e6 records.  Owner r % 8 of every partition must
    equal the oracle's merge of all ranks' outputs (worker.go:123-146); the other
    partitions must be empty."""
    from concurrent.futures import ThreadPoolExecutor
    from mrgpu import Context
    P, R, V, NF = 8, 64, 10**7, 100
    voc = C.Vocab(C.KIND_ASCII, 0.8, V, 5)
    SZ = 1_500_000  # > a file's 1e5-word vocabulary share
    files = []
    for g in range(P):
        buf = np.empty(NF * SZ, dtype=np.uint8)

        def one(i, g=g, buf=buf):  # (the C generator releases the GIL)
            voc.fill_files([SZ], [5 + 1000 * g + i], C.wc_params(vocab_lo=V * i // NF, vocab_hi=V * (i + 1) // NF),
                           threads=1, out=buf[i * SZ:(i + 1) * SZ])
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(one, range(NF)))
        files.append(buf.tobytes())
    with ThreadPoolExecutor(4) as ex:  # the C oracle releases the GIL
        per = list(ex.map(lambda f: O.c_count_mt("wc", f, R, 4), files))
    want = O.c_merge_parts("wc", per)
    del per
    ctxs = [Context(0) for _ in range(P)]
    try:
        local = [ctxs[i].map(MRG_APP_WC, files[i], nreduce=R) for i in range(P)]
        keys = [c.stats()["distinct_keys"] for c in ctxs]
        assert min(keys) >= V, keys
        owned = Context.exchange_group(ctxs, local)
        for i in range(P):
            out = ctxs[i].reduce_all(owned[i])
            for r in range(R):
                assert out[r] == (want[r] if r % P == i else b""), f"rank {i} partition {r}"
        for q in local + owned:
            q.free()
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("app", ["wc", "grep:distributed", "wc-2048"])
def test_host_input_streamed_in_pieces(ctx, app):
    """Host input copied piece by piece on a second stream while the map runs
    over the resident pieces: 1 MiB-ish pieces over a
    ~24 MB split (dictionary on, words / lines across every piece seam) equal the
    oracle, as does the same split as device input."""
    nb = 2048 if app == "wc-2048" else 0
    app = app.split("-")[0]
    if app == "wc":
        files = cases.synthetic(C.KIND_UTF8, 50000, [9_000_001, 8_000_000, 7_000_003], 71, 0.001)
    else:
        files = cases.synthetic_grep(50000, [9_000_001, 8_000_000, 7_000_003], 72, match_rate=0.02)
    joined = b"\n".join(files)
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    pat = b"" if app == "wc" else b"distributed"
    want = O.c_partitioned(app, files, 10)
    ctx.set_option("ingest_piece", 1 << 20)
    ctx.set_option("ingest_min", 1 << 20)
    ctx.set_option("dict_min_bytes", 1)
    ctx.set_option("spill_buckets", nb)
    try:
        assert ctx.run_job(a, joined, pattern=pat, nreduce=10) == want
        assert ctx.stats()["staged_bytes"] == len(joined)
    finally:
        ctx.set_option("spill_buckets", 0)
        ctx.set_option("ingest_piece", 0)
        ctx.set_option("ingest_min", 0)
        ctx.set_option("dict_min_bytes", 0)


@pytest.mark.parametrize("direct", [0, -1, 1])
def test_run_job_output_to_host(ctx, direct):
    """mrg_run_job's output lines written straight into pinned host memory by
    the formatting kernel (option out_direct, default), through a device buffer
    and a copy (-1), or directly for wc only (1): the same bytes as the oracle
    on wc edge cases (long words, an empty output) and grep edge cases."""
    ctx.set_option("out_direct", direct)
    try:
        edge = cases.edge_cases()
        for name in ("empty", "big_word", "utf8_mix", "mixed_lengths", "long_shared_prefix"):
            for f in edge.get(name, []):
                assert ctx.run_job(MRG_APP_WC, f, nreduce=10) == O.c_partitioned("wc", [f], 10), name
        for name, (gf, pat) in sorted(cases.grep_edge_cases().items()):
            for f in gf:
                want = O.c_partitioned("grep:" + pat.decode("utf-8", "surrogateescape"), [f], 4)
                assert ctx.run_job(MRG_APP_GREP, f, pattern=pat, nreduce=4) == want, name
    finally:
        ctx.set_option("out_direct", 0)


@pytest.mark.parametrize("app", ["wc", "wc-copied", "grep:distributed"])
def test_run_job_async_pipelined(ctx, app):
    """mrg_run_job_async / mrg_job_wait: jobs queued two deep (the second job's
    map overlaps the first's output transfer), outputs returned in order and
    byte-equal to the oracle; a third queued job is refused; a synchronous job
    after async ones waits for their transfers.  wc outputs are written straight
    into the pinned buffer, or (wc-copied: option async_direct_max -1, as C5's
    110 MB outputs are) formatted in device memory and copied on the output stream."""
    from mrgpu.lib import MrgError
    if app == "wc-copied":
        ctx.set_option("async_direct_max", -1)
        try:
            return test_run_job_async_pipelined(ctx, "wc")
        finally:
            ctx.set_option("async_direct_max", 0)
    a = MRG_APP_WC if app == "wc" else MRG_APP_GREP
    pat = b"" if app == "wc" else b"distributed"
    if app == "wc":
        jobs = [cases.synthetic(C.KIND_UTF8, 20000, [700_000, 300_001], 70 + k, 0.0005) for k in range(3)]
    else:
        jobs = [cases.synthetic_grep(20000, [800_000, 250_000], 80 + k) for k in range(3)]
    joined = [b"\n".join(f) for f in jobs]
    want = [O.c_partitioned(app, f, 10) for f in jobs]
    ctx.run_job_async(a, joined[0], pattern=pat, nreduce=10)
    ctx.run_job_async(a, joined[1], pattern=pat, nreduce=10)
    with pytest.raises(MrgError, match="two jobs in flight"):
        ctx.run_job_async(a, joined[2], pattern=pat, nreduce=10)  # (refused: not queued)
    assert ctx.job_wait() == want[0]
    ctx.run_job_async(a, joined[2], pattern=pat, nreduce=10)
    assert ctx.job_wait() == want[1]
    # a synchronous job in between: the queued transfer finishes first, both exact
    assert ctx.run_job(a, joined[0], pattern=pat, nreduce=10) == want[0]
    assert ctx.job_wait() == want[2]
    with pytest.raises(MrgError, match="no job queued"):
        ctx.job_wait()
