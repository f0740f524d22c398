"""mrgpu — MI355X-native MapReduce hot path (wc / grep) behind the C ABI of include/mrgpu.h.

Package layout (the hyphenated directory `distributed-systems-implemented_amd/`
holds this package; add that directory to sys.path to import it):
  csrc/          HIP kernels for gfx950 + the C ABI (build/libmrgpu.so)
  mrgpu/lib.py   ctypes binding of the C ABI
  mrgpu/mr.py    host mirror of the reference interface (KeyValue, ihash, map/reduce tasks,
                 mrsequential) over the C ABI
  mrgpu/corpus.py synthetic corpora (build/libmrcorpus.so)
"""
from .lib import (ALL_PARTS, MRG_APP_GREP, MRG_APP_WC, Context, MrgError, Parts, device_count, ihash,  # noqa: F401
                  load_library)
