"""CPU tests: the C-ABI library loads and exports every symbol include/mrgpu.h
declares (no compute calls: there is no GPU in the build container)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from mrgpu import lib as mlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mrgpu.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mrg_[a-z0-9_]+)\s*\(", txt)))


def test_header_lists_expected_entry_points():
    syms = declared_symbols()
    assert set(syms) == set(mlib.EXPORTED)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(mlib.LIB_PATH):
        pytest.skip("libmrgpu.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", mlib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mrg_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    L = mlib.load_library()
    for s in declared_symbols():
        assert hasattr(L, s)


def test_library_is_gfx950_code_object():
    if not os.path.exists(mlib.LIB_PATH):
        pytest.skip("not built")
    data = open(mlib.LIB_PATH, "rb").read()  # the embedded offload bundle names its target
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_host_ihash_matches_oracle():
    import _oracle as O
    for k in [b"", b"a", b"foobar", b"distributed", "κόσμε".encode()]:
        assert mlib.ihash(k) == O.c_ihash(k) == O.mr_oracle.ihash(k)


def test_no_gpu_open_fails_loudly():
    """Without a GPU the product must refuse to run (no CPU fallback)."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(mlib.MrgError):
        mlib.Context(0)
