"""Shared parity inputs: edge cases the reference's semantics hinge on
 plus seeded synthetic corpora."""
from __future__ import annotations

import random

from mrgpu import corpus as C

W16 = b"abcdefghijklmnop"  # exactly 16 letters (the inline-key limit)



def utf8_slot_tail(rune):
    """Words of 16 ASCII letters starting at the last owned byte of chunks 0..3 (992
    bytes each), followed by `rune` (a letter, or U+00D7, a non-letter), so the rune
    straddles the end of the chunk's 1 KiB window."""
    r = rune.encode()
    out = bytearray()
    for c in range(4):
        start = 992 * c + 991 - (len(r) - 2 if len(r) > 2 else 0)
        out += b"ab " * ((start - len(out)) // 3)
        out += b" " * (start - len(out))
        out += b"q" * 16 + r + b"z " + b"tail words "
    return bytes(out)

def edge_cases() -> dict[str, list[bytes]]:
    """name -> list of files (each file = one map split)."""
    big_word = b"Z" * 5000
    rnd = random.Random(11)
    noisy = bytes(rnd.randrange(256) for _ in range(20000))
    utf8_mix = ("Ωμέγα, Привет мир! 中文字符 𐐷𐐸 ĳ ǅ ʰ ª º µ ß ÿ  x—y、z 😀 é "
                "٠١ Ⅻ ⅻ ⓐ 〆 ー ｱ").encode() * 30
    chunk_cross = (b"x" * 2040 + b" " + b"abcdefghijklmnopqrstuvwxyz " * 3 + b"k" * 2100 + b" end") * 3
    return {
        "empty": [b""],
        "one_word": [b"hello"],
        "no_trailing_sep": [b"alpha beta gamma"],
        "only_separators": [b" \n\t,.;:!?0123456789 " * 50],
        "w16_w17": [W16 + b" " + W16 + b"q " + W16[:-1] + b"\n" + W16 + b"qr"],
        "case_sensitive": [b"The the THE tHe the The\nthe"],
        "big_word": [big_word + b" " + big_word + b"\n" + b"small"],
        "all_letters": [b"q" * 70000],
        "chunk_cross": [chunk_cross],
        "random_bytes": [noisy],
        "utf8_mix": [utf8_mix],
        "invalid_utf8": [b"ab\xffcd\xc0\xafef\xe2\x82gh\xed\xa0\x80ij\xf4\x90\x80\x80kl\xc3mn\x80op\xce\xbb\xce"],
        "truncated_at_eof": [b"word \xe2\x82", b"x\xf0\x9f\x98"],
        # a word starting in the last owned lane of a 992-byte wc chunk whose 17th
        # byte begins a multi-byte letter ending past the 1 KiB window (slot byte 1024
        # = input byte chunk start + 1008): only the input bytes after the window tell
        # that the word is longer than 16 bytes
        "utf8_slot_tail": [utf8_slot_tail(rune) for rune in ("\u00e9", "\u4e2d", "\U00010400", "\u00d7")],
        "multi_file": [b"one two three\n", b"two three\n", b"three"],
        "apostrophes": [b"don't can't won't it's O'Neil rock'n'roll"],
        # splits whose last bytes are a word, for every n % 4 (the map streams the
        # split with range-checked 16-byte loads and patches its last n % 4 bytes)
        "tail_bytes": [b"a", b"ab", b"abc", b"abcd", b"abcde", b"xy z", b"q r st", b"  uvw"],
        # words of 1..20 letters at every offset around the 992-byte wc chunk seams
        # (and the 944/976/960-byte ones of earlier layouts / grep), 16-byte lanes and the
        # 1 KiB windows, split lengths of every residue mod 4
        "mixed_lengths": [mixed_words(n, seed) for seed, n in
                          enumerate([12345, 7777, 2002, 945, 944, 943, 1889, 5000, 977, 976, 975, 1953, 2929, 961,
                                     993, 992, 991, 1985, 2977])],
        # > 64 distinct keys with one 8-byte prefix: the reduce's long tied run (sort
        # falls back to the k1 pass), plus prefix-of-another-key orderings
        "shared_prefix": [b" ".join(b"abcdefgh" + bytes([97 + i % 26, 97 + i // 26 % 26]) * (1 + i % 3)
                                    for i in range(600)) + b" abcdefgh abcdefg abcdefghi"],
        # > 64 distinct keys longer than 16 bytes sharing their first 16: a long tied
        # run even after the k1 pass (the reduce merge-sorts it by full comparison)
        "long_shared_prefix": [b"\n".join(b"abcdefghijklmnopq" + bytes([97 + (i * 7) % 26, 97 + (i * 11) % 26]) * (i % 4)
                                           for i in range(700)) + b" abcdefghijklmnop abcdefghijklmnopq"],
    }


def long_words(n: int, seed: int) -> bytes:
    """About n bytes of words of 17-70 bytes (ASCII, Greek, Deseret letters) drawn
    from a 300-word vocabulary with a skewed law (hot long words repeat across
    chunks and workgroups), separated by 1-2 ASCII / U+3001 separators: chunks
    holding only words over 16 bytes (the long-word list and kernel)."""
    rnd = random.Random(3000 + seed)
    alph = ["abcdefghijklmnopqrstuvwxyz", "αβγδεζηθικλμνξοπρστυφχψω", "".join(chr(0x10400 + i) for i in range(40))]
    vocab = []
    for k in range(300):
        a = alph[k % 3]
        ln = rnd.randint(17, 70) // len(a[0].encode()) + 1
        vocab.append("".join(rnd.choice(a) for _ in range(ln)).encode())
    out = bytearray()
    while len(out) < n:
        out += vocab[min(int(rnd.paretovariate(0.7)) - 1, 299)]
        out += rnd.choice([b" ", b"\n", b", ", "\u3001".encode()])
    return bytes(out)


def mixed_words(n: int, seed: int) -> bytes:
    """Deterministic text of exactly n bytes ending in a letter: words of 1-20
    letters (some longer than the 16-byte inline key) and 1-3 byte separators."""
    rnd = random.Random(1000 + seed)
    out = bytearray()
    while len(out) < n:
        out += bytes(rnd.choice(b"abcdefghijklmnopqrstuvwxyzABC") for _ in range(rnd.randint(1, 20)))
        out += bytes(rnd.choice(b" \n,.;0") for _ in range(rnd.randint(1, 3)))
    out = out[:n]
    out[-1] = ord("z")
    return bytes(out)


def _seams(pat: bytes, nseams: int) -> bytes:
    """Occurrences of pat starting 1..12 bytes before every 960-byte seam (so each
    one crosses a seam), a "di" decoy before each, lines of 'q' in between."""
    b = bytearray(b"q" * (960 * (nseams + 1)))
    for i in range(1, nseams + 1):
        at = 960 * i - 1 - (i % 12)
        b[at - 4:at - 1] = b"di\n"
        b[at:at + len(pat)] = pat
        b[at + len(pat)] = 0x0A
    return bytes(b)


def grep_seam_lines(pat: bytes = b"distributed") -> bytes:
    """Matching lines that cross 960-byte map-chunk seams with occurrences on
    both sides (each chunk keeps its own first hit of the line), lines spanning
    three or more chunks with a hit in every chunk, the same seam-crossing line
    several times, lines over 4 KiB (the workgroup resolution path) with hits
    in many chunks or only far apart, and an occurrence ending exactly at a
    seam.  Every line occurrence must count once (dgrep.go:30-33)."""
    rnd = random.Random(77)
    out = bytearray()

    def pad_to(off):  # filler lines up to input offset off
        while len(out) < off:
            k = min(off - len(out), rnd.randint(1, 50))
            out.extend(b"x" * (k - 1) + b"\n" if k > 1 else b"\n")

    for i in range(1, 60):
        seam = 960 * (3 * i)
        pad_to(seam - 200 + (i % 7))
        kind = i % 6
        if kind == 0:    # hits just before and just after the seam
            line = b"a" * (190 - (i % 7) - len(pat)) + pat + b"b" * 5 + pat + b"c" * 20
        elif kind == 1:  # hit before the seam, hit straddling it
            line = b"a" * 20 + pat + b"a" * (176 - (i % 7) - 2 * len(pat)) + pat + b"z" * 30
        elif kind == 2:  # a line over three chunks, a hit in each
            line = pat + b"m" * 900 + pat + b"m" * 950 + pat + b"m" * 10
        elif kind == 3:  # hit only after the seam (the line starts in the chunk before)
            line = b"w" * 250 + pat + b"w" * 3
        elif kind == 4:  # occurrence ending exactly at the seam, another after it
            line = b"q" * (200 - (i % 7) - len(pat)) + pat + pat + b"r"
        else:            # an occurrence straddling the seam only
            line = b"s" * (200 - (i % 7) - 4) + pat + b"t" * 9
        out.extend(line + b"\n")
        if i % 5 == 0:  # the same line again at another seam offset
            pad_to(960 * (3 * i + 1) - 100)
            out.extend(line + b"\n")
    # > 4 KiB lines: hits in many chunks; hits far apart (first near the start)
    out.extend(b"y" * 37 + b"".join(pat + b"h" * 600 for _ in range(20)) + b"\n")
    out.extend(pat + b"k" * 9000 + pat + b"k" * 7000 + pat + b"\n")
    out.extend(b"k" * 6000 + pat + b"\n")
    out.extend(b"y" * 37 + b"".join(pat + b"h" * 600 for _ in range(20)) + b"\n")  # a repeat
    return bytes(out)


def grep_edge_cases() -> dict[str, tuple[list[bytes], bytes]]:
    return {
        "basic": ([b"a distributed system\nnothing here\ndistributed\n\ndistributed distributed x\n"], b"distributed"),
        "cr_kept": ([b"line distributed\r\nother\r\n"], b"distributed"),
        "dup_lines": ([b"x distributed\nx distributed\ny\nx distributed"], b"distributed"),
        "utf8_pattern": (["καλημέρα κόσμε\nγεια σου κόσμε\nhello\n".encode()], "κόσμε".encode()),
        "no_trailing_nl": ([b"abc\ndistributedness"], b"distributed"),
        "pattern_at_edges": ([b"distributed" * 300 + b"\n" + b"q" * 3000 + b"distributed"], b"distributed"),
        "long_pattern": ([(b"x" * 100 + b"\n") * 10 + b"y" * 70 + b"\n" + b"zz" + b"y" * 70 + b"zz\n"], b"y" * 70),
        "empty_pattern": ([b"a\nb\n\nc"], b""),
        "newline_pattern": ([b"a\nb\n"], b"a\nb"),
        "multi_file": ([b"distributed one\n", b"distributed two\ndistributed one\n"], b"distributed"),
        "long_lines": ([(b"w" * 5000 + b" distributed " + b"v" * 3000 + b"\n") * 3], b"distributed"),
        # > 64 distinct matching lines with one 16-byte prefix, in scrambled order,
        # and lines that are prefixes of others: the reduce's long tied run
        # the pattern ending exactly at the split's end, for every n % 4 (the
        # grep map streams 16-byte range-checked loads and patches the last dword)
        "tail_n_mod4": ([b"x\n" + b"y" * k + b" distributed" for k in range(4)], b"distributed"),
        # occurrences straddling every 960-byte chunk seam (own bytes + look-ahead),
        # a 2-byte-prefix decoy before each, and a 65-byte pattern across seams
        "chunk_seams": ([_seams(b"distributed", 40)], b"distributed"),
        "pattern_65_seams": ([b"".join(b"r" * (960 * i - 30) + b"z" * 65 + b"\n" for i in range(1, 12))], b"z" * 65),
        "tied_lines": ([b"".join(b"the distributed system " + str((i * 7919) % 1000).encode() * (1 + i % 3) + b"\n"
                                 for i in range(1000)) + b"the distributed system \nthe distributed system\n"],
                       b"distributed"),
        # strings.Split yields a final "" after a trailing '\n'; the empty pattern
        # matches it, so mr-out holds " \n" 
        "empty_pattern_trailing_nl": ([b"a\nb\n", b"\n", b"x\n\ny\n"], b""),
        # a frequent one-byte pattern in lines longer than a lane's scan window
        # (4 KiB), the same long line twice (bytewise table compare), overlapping
        # occurrences, and hits right after a newline
        "long_lines_many_hits": ([_long_line(21000, 1) + b"\nshort e line\n" + _long_line(21000, 1) + b"\n"
                                  + _long_line(9000, 2) + b"\neee\ne\n" + _long_line(5000, 3)], b"e"),
        "overlapping": ([b"aaaaaa\nxaax\naaa\naa\na\n"], b"aa"),
        # the grep map's 4-byte prefix filter: a 4-byte pattern at every offset
        # mod 16 (across dwords, lanes and chunk seams) with 3-byte decoys,
        # overlapping occurrences, lines shorter than the pattern, the pattern
        # at the split's end; a 5-byte UTF-8 pattern with its first 4 bytes as
        # decoys
        "prefix4_offsets": ([b"".join(b"x" * k + b"dis dist\n" for k in range(40)) + _seams(b"dist", 30) + b"aaaa",
                             b"aaaaaaa\naaa\nxaaaax\naaaa"], b"dist"),
        "prefix4_overlap": ([b"aaaaaaa\naaa\nxaaaax\n" * 70 + b"aaaa"], b"aaaa"),
        "prefix5_utf8": (["".join("y" * k + "aκ aκc\n" for k in range(33)).encode() + _seams("aκc".encode(), 12)],
                         "aκc".encode()),
        # > 64 distinct matching lines sharing a 70-byte prefix that differ later,
        # strict prefixes of one another, NUL bytes past byte 64 (the reduce's
        # arena-compare fallback past the 64 bytes its sort words cover)
        "shared_prefix_70": ([_shared_prefix_lines()], b"distributed"),
        # dgrep.go:20-23: regexp.Compile fails on invalid UTF-8, grepMap returns nil
        "invalid_utf8_pattern": ([b"ab\xffcd\n\xff\nxx\n"], b"\xff"),
        "truncated_utf8_pattern": (["κόσμε\n".encode(), b"\xce\n"], b"\xce"),
    }


def _long_line(n: int, seed: int) -> bytes:
    """n bytes of one line (no '\n'): letters with frequent 'e' and spaces."""
    rnd = random.Random(500 + seed)
    return bytes(rnd.choice(b"abcdeeee ") for _ in range(n))


def _shared_prefix_lines() -> bytes:
    prefix = b"distributed " + b"p" * 58  # 70 bytes
    lines = [prefix, prefix + b"a", prefix + b"ab", prefix + b"a\x00", prefix + b"\x00"]
    for i in range(120):
        tail = bytes([97 + (i * 7) % 26, 97 + (i * 13) % 26]) * (1 + i % 3)
        if i % 5 == 0:
            lines.append(prefix[:66] + b"\x00" + prefix[67:] + tail)
        else:
            lines.append(prefix + tail)
    lines = lines * 2  # duplicates collapse in Reduce
    random.Random(9).shuffle(lines)
    return b"\n".join(lines) + b"\n"


def synthetic(kind: int, V: int, sizes: list[int], seed: int, invalid_rate: float = 0.0) -> list[bytes]:
    voc = C.Vocab(kind, 1.07, V, seed)
    files = voc.fill_files(sizes, [seed * 1000 + i for i in range(len(sizes))], C.wc_params(invalid_rate))
    return [bytes(f) for f in files]


def synthetic_grep(V: int, sizes: list[int], seed: int, match_rate: float = 0.02) -> list[bytes]:
    voc = C.Vocab(C.KIND_UTF8, 1.07, V, seed)
    files = voc.fill_files(sizes, [seed * 1000 + i for i in range(len(sizes))], C.grep_params(match_rate=match_rate))
    return [bytes(f) for f in files]
