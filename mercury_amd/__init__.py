"""mercury_amd -- MI355X-native packet fingerprint/classify path for
cisco/mercury's libmerc API.

The compute path is libmercury_amd.so (hand-written gfx950 HIP kernels behind
the C-ABI in include/mfp.h).  This package is a thin ctypes host binding used
by tests and bench.py; it never falls back to a CPU implementation.
"""
from .api import (FP_TYPE_NAMES, MSG_NAMES, RECORD_DTYPE, DESC_DTYPE, Context, MercuryAmdError,  # noqa: F401
                  fingerprints, library_path, load_library, parse_filter)

__all__ = ["Context", "MercuryAmdError", "fingerprints", "load_library", "library_path", "RECORD_DTYPE",
           "DESC_DTYPE", "FP_TYPE_NAMES", "MSG_NAMES", "parse_filter"]
