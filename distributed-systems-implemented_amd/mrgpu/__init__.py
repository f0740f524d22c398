"""mrgpu — MI355X-native MapReduce hot path (wc / grep) behind the C ABI of include/mrgpu.h.

Package layout (the hyphenated directory `distributed-systems-implemented_amd/`
holds this package; add that directory to sys.path to import it):
  csrc/          HIP kernels for gfx950 + the C ABI (build/libmrgpu.so)
  csrc/mrhost.cpp  C++ hosts over the C ABI (build/mrseq_gpu = main/mrsequential.go,
                 build/mrjob_gpu = worker map / reduce tasks, build/mrcoord_gpu =
                 mr/coordinator.go + one worker process per GPU)
  mrgpu/lib.py   ctypes binding of the C ABI
  mrgpu/intermediate.py  host codec of the MRGI intermediate format (mrg_parts_export)
  mrgpu/dist.py  multi-rank plumbing (ownership r % P, out-of-band RCCL id, max-over-ranks)
  mrgpu/corpus.py synthetic corpora (build/libmrcorpus.so)
"""
from .lib import (ALL_PARTS, MRG_APP_GREP, MRG_APP_WC, Context, MrgError, Parts, device_count, ihash,  # noqa: F401
                  load_library)
