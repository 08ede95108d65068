"""mercury_amd -- MI355X-native packet fingerprint/classify path for
cisco/mercury's libmerc API.

The compute path is libmercury_amd.so (hand-written gfx950 HIP kernels behind
the C-ABI in include/mfp.h).  This package is a thin ctypes host binding used
by tests and bench.py; it never falls back to a CPU implementation.
"""
from .api import (write_json, ANALYSIS_DTYPE, FP_TYPE_NAMES, MSG_NAMES, NO_PROCESS, RECORD_DTYPE, DESC_DTYPE,  # noqa: F401
                  STATUS_NAMES, Context, MercuryAmdError, fingerprints, library_path, load_library,
                  normalize_server_name, lpm_query, parse_filter, resource_stats, PcapReader, tpacket3_block, Prevalence,
                  SIGHTING_DTYPE, PacketProcessor, pcap_file_header)

__all__ = ["Context", "write_json", "MercuryAmdError", "fingerprints", "load_library", "library_path", "RECORD_DTYPE",
           "DESC_DTYPE", "FP_TYPE_NAMES", "MSG_NAMES", "parse_filter", "ANALYSIS_DTYPE", "NO_PROCESS",
           "STATUS_NAMES", "normalize_server_name", "lpm_query", "resource_stats", "PcapReader", "tpacket3_block", "Prevalence",
           "SIGHTING_DTYPE", "PacketProcessor", "pcap_file_header"]
