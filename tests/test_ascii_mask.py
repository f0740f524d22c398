"""The map kernel's ASCII letter mask (mrgpu_device.h ascii_mask16) gathers
per-byte letter flags with byte dot products (v_dot4_u32_u8); this restates it
in numpy and checks it against the plain per-byte predicate ([A-Za-z], the ASCII
half of unicode.IsLetter, MapReduce/mrapps/wc.go:23) on random and exhaustive
inputs.  CPU only: it pins the arithmetic, the GPU parity tests pin the kernel."""
import numpy as np

W_LO = np.array([1, 2, 4, 8], dtype=np.uint32)
W_HI = np.array([16, 32, 64, 128], dtype=np.uint32)


def flags4(x):
    """0x80 in each letter byte (the SWAR test: (y + 0x1F) & ~(y + 0x05) & 0x80, y = x | 0x20)."""
    y = (x | np.uint32(0x20202020)).astype(np.uint64)
    a = (y + 0x1F1F1F1F) & 0xFFFFFFFF
    b = (y + 0x05050505) & 0xFFFFFFFF
    return (a & ~b & 0x80808080).astype(np.uint32)


def dot4(a, w, acc):
    by = a.view(np.uint8).reshape(-1, 4).astype(np.uint32)
    return (by * w).sum(axis=1).astype(np.uint32) + acc


def mask16(d):  # d: (n, 4) uint32 little-endian dwords of 16 bytes
    lo = dot4(flags4(d[:, 1]), W_HI, dot4(flags4(d[:, 0]), W_LO, 0))
    hi = dot4(flags4(d[:, 3]), W_HI, dot4(flags4(d[:, 2]), W_LO, 0))
    return (lo | (hi << 8)) >> 7


def reference(d):
    by = d.view(np.uint8).reshape(-1, 16)
    letter = ((by | 0x20).astype(np.int32) - 0x61 >= 0) & ((by | 0x20).astype(np.int32) - 0x61 < 26)
    return (letter.astype(np.uint32) << np.arange(16, dtype=np.uint32)).sum(axis=1).astype(np.uint32)


def test_mask16_random():
    rng = np.random.default_rng(7)
    d = (rng.integers(0, 1 << 32, size=(200_000, 4), dtype=np.uint64) & 0x7F7F7F7F).astype(np.uint32)
    assert np.array_equal(mask16(d), reference(d))


def test_mask16_every_byte_value_in_every_position():
    base = np.full((128 * 16, 4), 0x20202020, dtype=np.uint32)  # spaces
    by = base.view(np.uint8).reshape(-1, 16)
    for pos in range(16):
        by[pos * 128:(pos + 1) * 128, pos] = np.arange(128, dtype=np.uint8)
    assert np.array_equal(mask16(base), reference(base))
