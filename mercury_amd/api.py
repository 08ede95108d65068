"""ctypes binding of libmercury_amd.so (include/mfp.h)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

DESC_DTYPE = np.dtype([("offset", "<u8"), ("caplen", "<u4"), ("linktype", "<u2"), ("flags", "<u2")])
RECORD_DTYPE = np.dtype([("fp_offset", "<u8"), ("fp_len", "<u4"), ("fp_type", "u1"), ("msg", "u1"),
                         ("flags", "u1"), ("xflags", "u1"), ("sni_off", "<u2"), ("sni_len", "<u2"),
                         ("ua_off", "<u2"), ("ua_len", "<u2"), ("src_port", "<u2"), ("dst_port", "<u2"),
                         ("net", "<u4")])
ANALYSIS_DTYPE = np.dtype([("score", "<f8"), ("malware_prob", "<f8"), ("process", "<u4"), ("attr", "<u2"),
                           ("status", "u1"), ("flags", "u1"), ("proc_slot", "<u4"), ("reserved", "<u4")])
SIGHTING_DTYPE = np.dtype([("hash", "<u8"), ("first", "<u8"), ("last", "<u8"), ("count", "<u4"),
                           ("first_seen", "<u4")])
assert DESC_DTYPE.itemsize == 16 and RECORD_DTYPE.itemsize == 32 and ANALYSIS_DTYPE.itemsize == 32
assert SIGHTING_DTYPE.itemsize == 32
NO_PROCESS = 0xFFFFFFFF
# attribute tags (include/mfp.h): the archive's own tags take bits 10..15 and
# their probabilities come in MFP_ATTR_DB_TAGS doubles per packet
ATTR_DB_FIRST = 10
ATTR_DB_TAGS = 6
AN_VALID, AN_MALWARE, AN_CLASSIFY_MALWARE = 1, 2, 4
STATUS_NAMES = ["no_info_available", "labeled", "randomized", "unlabeled", "unanalyzed"]

# fingerprint::get_type_name (src/libmerc/fingerprint.h:159-192)
FP_TYPE_NAMES = ["unknown", "tls", "tls_server", "http", "http_server", "ssh", "ssh_kex", "tcp", "dhcp",
                 "smtp_server", "dtls", "dtls_server", "quic", "tcp_server", "openvpn", "tofsee", "stun",
                 "ssh_init", "ssh_server", "ssh_kex_server", "ssh_init_server"]
MSG_NAMES = ["none", "tls.client_hello", "tls.server_hello", "tls.certificate", "ssh.init", "ssh.kex",
             "http.request", "http.response", "tcp.syn", "tcp.syn_ack", "dtls.client_hello",
             "dtls.server_hello", "dtls.hello_verify_request", "quic.initial", "stun", "openvpn_tcp",
             "other"]   # MFP_MSG_OTHER: a selected protocol outside the path (no record)

# mfp_tcp_seg (include/mfp.h): reassembly inputs per packet
SEG_DTYPE = np.dtype([("seq", "<u4"), ("more", "<u4"), ("pay_off", "<u4"), ("pay_len", "<u2"), ("kind", "u1"),
                      ("reserved", "u1")])
SEG_DATA, SEG_SUPPLEMENTARY, SEG_SSH = 1, 2, 4
# mfp_process_batch_reassembly props bits: reassembled, then reassembly_flag_val
# (reassembly.hpp:73-91) and reassembly_overlap_flags (reassembly.hpp:93-105)
REASM_FLAGS = ["missing_segment", "timeout", "out_of_order", "out_of_buffer", "max_segments_exceed",
               "segment_overlaps", "truncated"]
REASM_OVERLAPS = ["back_partial_overlap", "back_subset_overlap", "front_partial_overlap", "front_superset_overlap"]

MODE_WRITE_JSON = 0
MODE_ANALYSIS = 1


class MercuryAmdError(RuntimeError):
    pass


def library_path():
    # MFP_LIB: an alternative build of the same library (profiling variants)
    return os.environ.get("MFP_LIB") or os.path.join(_HERE, "libmercury_amd.so")


_lib = None


def load_library():
    """Load the HIP extension; raises (loudly) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise MercuryAmdError(f"{path} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.mfp_init.restype = vp
    lib.mfp_init.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    lib.mfp_init_ex.restype = vp
    lib.mfp_init_ex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
    lib.mfp_resource_stats_ex.restype = ctypes.c_int
    lib.mfp_resource_stats_ex.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    lib.mfp_finalize.argtypes = [vp]
    lib.mfp_process_batch_device.restype = ctypes.c_int
    lib.mfp_process_batch_device.argtypes = [vp, vp, vp, sz, vp, vp, sz, vp, vp]
    lib.mfp_process_batch_host.restype = ctypes.c_longlong
    lib.mfp_process_batch_host.argtypes = [vp, vp, sz, vp, sz, vp, vp, sz]
    lib.mfp_fp_arena_bound.restype = sz
    lib.mfp_fp_arena_bound.argtypes = [sz, sz]
    lib.mfp_last_error.restype = ctypes.c_char_p
    lib.mfp_reference_version.restype = ctypes.c_uint32
    lib.mfp_analysis_enabled.restype = ctypes.c_int
    lib.mfp_analysis_enabled.argtypes = [vp]
    lib.mfp_analyze_batch_device.restype = ctypes.c_int
    lib.mfp_analyze_batch_device.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    lib.mfp_analyze_batch_device_pipelined.restype = ctypes.c_int
    lib.mfp_analyze_batch_device_pipelined.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    lib.mfp_analysis_flush.restype = ctypes.c_int
    lib.mfp_analysis_flush.argtypes = [vp]
    lib.mfp_analyze_batch_device_deferred_pipelined.restype = ctypes.c_int
    lib.mfp_analyze_batch_device_deferred_pipelined.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    lib.mfp_analysis_defer_newest.restype = ctypes.c_int
    lib.mfp_analysis_defer_newest.argtypes = [vp]
    lib.mfp_process_batch_host_seg.restype = ctypes.c_longlong
    lib.mfp_process_batch_host_seg.argtypes = [vp, vp, sz, vp, sz, vp, vp, sz, vp]
    lib.mfp_reassembler_create.restype = vp
    lib.mfp_reassembler_destroy.argtypes = [vp]
    lib.mfp_reassembler_flows.restype = ctypes.c_uint64
    lib.mfp_reassembler_flows.argtypes = [vp]
    lib.mfp_reassembler_frames.restype = vp
    lib.mfp_reassembler_frames.argtypes = [vp, ctypes.POINTER(sz)]
    lib.mfp_reassembly_enabled.restype = ctypes.c_int
    lib.mfp_reassembly_enabled.argtypes = [vp]
    lib.mfp_process_batch_reassembly_analysis.restype = ctypes.c_longlong
    lib.mfp_process_batch_reassembly_analysis.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, vp, sz, vp, vp, vp, vp]
    lib.mfp_write_json_batch_reassembly_analysis.restype = ctypes.c_longlong
    lib.mfp_write_json_batch_reassembly_analysis.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, vp, sz, vp, vp,
                                                             ctypes.c_int]
    lib.mfp_write_json_batch_reassembly.restype = ctypes.c_longlong
    lib.mfp_write_json_batch_reassembly.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, sz, vp, vp, ctypes.c_int]
    lib.mfp_process_batch_reassembly_context.restype = ctypes.c_longlong
    lib.mfp_process_batch_reassembly_context.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, vp, sz, vp, vp, vp, vp, vp]
    lib.mfp_process_batch_reassembly.restype = ctypes.c_longlong
    lib.mfp_process_batch_reassembly.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp, vp, sz, vp, vp]
    lib.mfp_process_batch_host_ex.restype = ctypes.c_longlong
    lib.mfp_process_batch_host_ex.argtypes = [vp, vp, sz, vp, sz, vp, vp, sz, vp, vp]
    lib.mfp_analysis_device_bytes.restype = ctypes.c_uint64
    lib.mfp_analysis_device_bytes.argtypes = [vp]
    lib.mfp_attribute_count.restype = ctypes.c_int
    lib.mfp_attribute_count.argtypes = [vp]
    lib.mfp_resource_version.restype = ctypes.c_char_p
    lib.mfp_resource_version.argtypes = [vp]
    lib.mfp_analysis_report_os.restype = ctypes.c_int
    lib.mfp_analysis_report_os.argtypes = [vp, ctypes.c_int]
    lib.mfp_process_os_info.restype = ctypes.c_int
    lib.mfp_process_os_info.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.POINTER(ctypes.c_uint64)]
    lib.mfp_process_name.restype = ctypes.c_char_p
    lib.mfp_process_name.argtypes = [vp, ctypes.c_uint32]
    lib.mfp_attribute_name.restype = ctypes.c_char_p
    lib.mfp_attribute_name.argtypes = [vp, ctypes.c_uint32]
    lib.mfp_analysis_counters.restype = ctypes.c_int
    lib.mfp_analysis_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), sz]
    lib.mfp_analysis_stats.restype = ctypes.c_int
    lib.mfp_analysis_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    lib.mfp_resource_stats.restype = ctypes.c_int
    lib.mfp_resource_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    lib.mfp_lpm_query.restype = ctypes.c_longlong
    lib.mfp_lpm_query.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, vp, sz]
    lib.mfp_normalize_server_name.restype = ctypes.c_int
    lib.mfp_normalize_server_name.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz]
    lib.mfp_parse_filter.restype = ctypes.c_int
    lib.mfp_parse_filter.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    lib.mfp_parse_filter_ex.restype = ctypes.c_int
    lib.mfp_parse_filter_ex.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
    lib.mfp_process_pipelined.restype = ctypes.c_longlong
    lib.mfp_process_pipelined.argtypes = [vp, vp, sz, vp, sz, vp, vp, sz, vp, vp, sz]
    lib.mfp_profile_enable.restype = ctypes.c_int
    lib.mfp_profile_enable.argtypes = [vp, ctypes.c_int]
    lib.mfp_profile_read.restype = ctypes.c_int
    lib.mfp_profile_read.argtypes = [vp, ctypes.c_uint32, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_double)]
    lib.mfp_pcap_open.restype = vp
    lib.mfp_pcap_open.argtypes = [ctypes.c_char_p]
    lib.mfp_pcap_linktype.restype = ctypes.c_int
    lib.mfp_pcap_linktype.argtypes = [vp]
    lib.mfp_pcap_read_batch.restype = ctypes.c_longlong
    lib.mfp_pcap_read_batch.argtypes = [vp, vp, sz, vp, sz, vp, ctypes.POINTER(ctypes.c_size_t)]
    lib.mfp_pcap_close.argtypes = [vp]
    lib.mfp_tpacket3_block.restype = ctypes.c_longlong
    lib.mfp_tpacket3_block.argtypes = [vp, vp, sz, vp, sz, vp]
    lib.mfp_write_json_batch.restype = ctypes.c_longlong
    lib.mfp_write_json_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp, sz, vp, ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.c_int]
    lib.mfp_write_json_batch_analysis.restype = ctypes.c_longlong
    lib.mfp_write_json_batch_analysis.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, sz, vp,
                                                  ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    u64 = ctypes.c_uint64
    lib.mfp_prevalence_create.restype = vp
    lib.mfp_prevalence_create.argtypes = [ctypes.c_uint32]
    lib.mfp_prevalence_destroy.argtypes = [vp]
    lib.mfp_prevalence_size.restype = u64
    lib.mfp_prevalence_size.argtypes = [vp]
    lib.mfp_prevalence_contains.restype = ctypes.c_int
    lib.mfp_prevalence_contains.argtypes = [vp, u64]
    lib.mfp_prevalence_keys.restype = ctypes.c_longlong
    lib.mfp_prevalence_keys.argtypes = [vp, vp, sz]
    lib.mfp_prevalence_distinct_exact.restype = ctypes.c_int
    lib.mfp_prevalence_distinct_exact.argtypes = [vp, vp, sz]
    lib.mfp_prevalence_resolve_distinct.restype = ctypes.c_int
    lib.mfp_prevalence_resolve_distinct.argtypes = [vp, vp, sz]
    lib.mfp_prevalence_resolve_sequence.restype = ctypes.c_int
    lib.mfp_prevalence_resolve_sequence.argtypes = [vp, vp, sz, vp]
    lib.mfp_prevalence_capacity.restype = ctypes.c_uint32
    lib.mfp_prevalence_capacity.argtypes = [vp]
    lib.mfp_prevalence_summary.restype = ctypes.c_longlong
    lib.mfp_prevalence_summary.argtypes = [vp, vp, sz, vp]
    lib.mfp_prevalence_resolve_shard.restype = ctypes.c_int
    lib.mfp_prevalence_resolve_shard.argtypes = [vp, vp, sz, vp, sz, vp]
    lib.mfp_prevalence_advance.restype = ctypes.c_int
    lib.mfp_prevalence_advance.argtypes = [vp, vp, sz]
    lib.mfp_analysis_prevalence.restype = vp
    lib.mfp_analysis_prevalence.argtypes = [vp]
    lib.mfp_analysis_set_prevalence.restype = ctypes.c_int
    lib.mfp_analysis_set_prevalence.argtypes = [vp, vp]
    lib.mfp_analysis_defer.restype = ctypes.c_int
    lib.mfp_analysis_defer.argtypes = [vp, ctypes.c_int]
    lib.mfp_analysis_distinct.restype = ctypes.c_longlong
    lib.mfp_analysis_distinct.argtypes = [vp, vp, sz]
    lib.mfp_analysis_sequence.restype = ctypes.c_longlong
    lib.mfp_analysis_sequence.argtypes = [vp, vp, sz]
    lib.mfp_analysis_resolve.restype = ctypes.c_int
    lib.mfp_analysis_resolve.argtypes = [vp, vp, sz]
    lib.mfp_analysis_last.restype = ctypes.c_longlong
    lib.mfp_analysis_last.argtypes = [vp, vp, sz]
    lib.mfp_analysis_resolve_sequence.restype = ctypes.c_int
    lib.mfp_analysis_resolve_sequence.argtypes = [vp, vp, sz]
    # batch packet processors (include/mfp_pkt_proc.h)
    lib.mfp_pkt_proc_create.restype = vp
    lib.mfp_pkt_proc_create.argtypes = [vp, ctypes.c_int, ctypes.POINTER(PktProcOpts), SINK_FN, vp]
    lib.mfp_pkt_proc_apply.restype = ctypes.c_int
    lib.mfp_pkt_proc_apply.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint16, vp]
    for f in ("mfp_pkt_proc_flush", "mfp_pkt_proc_drain", "mfp_pkt_proc_finalize"):
        getattr(lib, f).restype = ctypes.c_int
        getattr(lib, f).argtypes = [vp]
    lib.mfp_pkt_proc_destroy.argtypes = [vp]
    lib.mfp_pkt_proc_stats.restype = ctypes.c_int
    lib.mfp_pkt_proc_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), sz]
    lib.mfp_pcap_file_header.restype = sz
    lib.mfp_pcap_file_header.argtypes = [vp]
    lib.mfp_reassembler_dumped.restype = vp
    lib.mfp_reassembler_dumped.argtypes = [vp, ctypes.POINTER(sz)]
    _lib = lib
    return lib


class PktProcOpts(ctypes.Structure):
    """mfp_pkt_proc_opts (include/mfp_pkt_proc.h)."""
    _fields_ = [("batch_pkts", ctypes.c_size_t), ("arena_bytes", ctypes.c_size_t), ("flush_us", ctypes.c_uint32),
                ("json_threads", ctypes.c_int), ("chunk", ctypes.c_size_t)]


SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
PKT_PROC_JSON, PKT_PROC_FILTER_PCAP = 0, 1
PKT_PROC_STATS = ["packets", "batches", "records", "bytes", "device_ns", "writer_ns", "skipped"]


def pcap_file_header():
    """The 24-byte header of a `mercury -w` output file (mfp_pcap_file_header)."""
    lib = load_library()
    b = ctypes.create_string_buffer(24)
    assert lib.mfp_pcap_file_header(b) == 24
    return b.raw


class PacketProcessor:
    """A batch packet processor (include/mfp_pkt_proc.h) over a context made
    with MODE_WRITE_JSON: kind PKT_PROC_JSON (pkt_proc_json_writer_llq's
    output) or PKT_PROC_FILTER_PCAP (`mercury -w`).  apply() takes one
    packet, as pkt_proc::apply does; the output collects in `self.out`."""

    def __init__(self, ctx, kind=PKT_PROC_JSON, batch_pkts=0, arena_bytes=0, flush_us=0, json_threads=0, chunk=0):
        self.lib = ctx.lib
        self.out = bytearray()
        self.calls = 0

        def sink(_user, data, n):
            self.out += ctypes.string_at(data, n)
            self.calls += 1
            return 0
        self._sink = SINK_FN(sink)          # kept alive as long as the processor
        opts = PktProcOpts(batch_pkts, arena_bytes, flush_us, json_threads, chunk)
        self.h = self.lib.mfp_pkt_proc_create(ctx.h, kind, ctypes.byref(opts), self._sink, None)
        if not self.h:
            raise MercuryAmdError("mfp_pkt_proc_create failed: " + _err(self.lib))

    def _check(self, r, what):
        if r:
            raise MercuryAmdError(f"{what} failed ({r}): " + _err(self.lib))

    def apply(self, packet, ts_sec=0, ts_nsec=0, linktype=1, length=None):
        b = bytes(packet)
        n = len(b)
        self._check(self.lib.mfp_pkt_proc_apply(self.h, ts_sec, ts_nsec, n, n if length is None else length,
                                                linktype, b), "mfp_pkt_proc_apply")

    def flush(self):
        self._check(self.lib.mfp_pkt_proc_flush(self.h), "mfp_pkt_proc_flush")

    def drain(self):
        self._check(self.lib.mfp_pkt_proc_drain(self.h), "mfp_pkt_proc_drain")

    def finalize(self):
        self._check(self.lib.mfp_pkt_proc_finalize(self.h), "mfp_pkt_proc_finalize")

    def stats(self):
        v = (ctypes.c_uint64 * len(PKT_PROC_STATS))()
        self._check(self.lib.mfp_pkt_proc_stats(self.h, v, len(PKT_PROC_STATS)), "mfp_pkt_proc_stats")
        return dict(zip(PKT_PROC_STATS, list(v)))

    def close(self):
        if self.h:
            self.lib.mfp_pkt_proc_destroy(self.h)
            self.h = None


def _err(lib):
    return lib.mfp_last_error().decode("utf-8", "replace")


class Context:
    """One device context (the analogue of libmerc's mercury_context plus a
    processor).  `config` uses the reference's packet_filter_cfg syntax."""

    def __init__(self, config="tls,dtls,ssh,http,tcp,tcp.syn_ack", device=0, mode=MODE_WRITE_JSON, enc_key=None):
        """enc_key: the 16-byte key of an encrypted resource archive (libmerc_config.enc_key)."""
        self.lib = load_library()
        key = None if enc_key is None else ctypes.create_string_buffer(bytes(enc_key), 16)
        self.h = self.lib.mfp_init_ex(config.encode() if config is not None else None, device, mode, key)
        if not self.h:
            raise MercuryAmdError("mfp_init failed: " + _err(self.lib))

    def close(self):
        if getattr(self, "reasm", None):
            self.lib.mfp_reassembler_destroy(self.reasm)
            self.reasm = None
        if self.h:
            self.lib.mfp_finalize(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fp_arena_bound(self, desc):
        return int(self.lib.mfp_fp_arena_bound(len(desc), int(desc["caplen"].astype(np.uint64).sum())))

    def process_host(self, arena, desc):
        """arena: uint8 numpy array, desc: DESC_DTYPE array -> (records, fp_arena bytes)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        cap = self.fp_arena_bound(desc)
        fp = np.zeros(cap, dtype=np.uint8)
        used = self.lib.mfp_process_batch_host(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                               rec.ctypes.data, fp.ctypes.data, cap)
        if used < 0:
            raise MercuryAmdError("mfp_process_batch_host failed: " + _err(self.lib))
        return rec, fp[:used].tobytes()

    def process_host_segments(self, arena, desc):
        """The device walk with the per-packet reassembly inputs -> (records,
        fp arena bytes, SEG_DTYPE array)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        seg = np.zeros(max(n, 1), dtype=SEG_DTYPE)
        cap = self.fp_arena_bound(desc)
        fp = np.zeros(cap, dtype=np.uint8)
        used = self.lib.mfp_process_batch_host_seg(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                                   rec.ctypes.data, fp.ctypes.data, cap, seg.ctypes.data)
        if used < 0:
            raise MercuryAmdError("mfp_process_batch_host_seg failed: " + _err(self.lib))
        return rec, fp[:used].tobytes(), seg[:n]

    def process_host_reassembly(self, arena, desc, ts_ns=None, analysis=False, merged=True):
        """A host batch in stream order through the context's TCP reassembler
        (config with "reassembly"; state persists across calls) -> (records,
        fp arena bytes, props (uint16, REASM_* bits), arena ++ rebuilt frames,
        desc indexing it).  merged=False: None in place of arena ++ frames (a
        caller that renders no JSON skips the copy)."""
        if not self.lib.mfp_reassembly_enabled(self.h):
            raise MercuryAmdError("the configuration has no \"reassembly\"")
        if not getattr(self, "reasm", None):
            self.reasm = self.lib.mfp_reassembler_create()
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        props = np.zeros(max(n, 1), dtype=np.uint16)
        out_desc = np.zeros(max(n, 1), dtype=DESC_DTYPE)
        ts = None if ts_ns is None else np.ascontiguousarray(ts_ns, dtype=np.uint64)
        cap = self.fp_arena_bound(desc) + int(self.lib.mfp_fp_arena_bound(n, n * 8400))
        fp = np.zeros(cap, dtype=np.uint8)
        an = ap = None
        if analysis:
            an = np.zeros(max(n, 1), dtype=ANALYSIS_DTYPE)
            ap = np.zeros((max(n, 1), ATTR_DB_TAGS), np.float64)
            used = self.lib.mfp_process_batch_reassembly_analysis(
                self.h, self.reasm, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                None if ts is None else ts.ctypes.data, rec.ctypes.data, fp.ctypes.data, cap, props.ctypes.data,
                out_desc.ctypes.data, an.ctypes.data, ap.ctypes.data)
        else:
            used = self.lib.mfp_process_batch_reassembly(self.h, self.reasm, arena.ctypes.data, arena.nbytes,
                                                         desc.ctypes.data, n, None if ts is None else ts.ctypes.data,
                                                         rec.ctypes.data, fp.ctypes.data, cap, props.ctypes.data,
                                                         out_desc.ctypes.data)
        if used < 0:
            raise MercuryAmdError("mfp_process_batch_reassembly failed: " + _err(self.lib))
        joined = None
        if merged:
            flen = ctypes.c_size_t(0)
            ptr = self.lib.mfp_reassembler_frames(self.reasm, ctypes.byref(flen))
            frames = np.ctypeslib.as_array((ctypes.c_uint8 * flen.value).from_address(ptr)) if flen.value else \
                np.zeros(0, np.uint8)
            joined = np.concatenate([arena, frames])
        out = (rec, fp[:used].tobytes(), props[:n], joined, out_desc[:n])
        return out + (an[:n], ap[:n]) if analysis else out

    def analyze_host_reassembly(self, arena, desc, ts_ns=None, analysis=True):
        """The analysis_context path with reassembly (a MODE_ANALYSIS context
        with "reassembly"; mfp_process_batch_reassembly_context) -> (records, fp
        arena bytes, props, arena ++ frames, desc indexing it, analysis records
        or None, attribute probabilities or None, more_pkts_needed (uint8))."""
        if not self.lib.mfp_reassembly_enabled(self.h):
            raise MercuryAmdError("the configuration has no \"reassembly\"")
        if not getattr(self, "reasm", None):
            self.reasm = self.lib.mfp_reassembler_create()
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        props = np.zeros(max(n, 1), dtype=np.uint16)
        out_desc = np.zeros(max(n, 1), dtype=DESC_DTYPE)
        more = np.zeros(max(n, 1), dtype=np.uint8)
        ts = None if ts_ns is None else np.ascontiguousarray(ts_ns, dtype=np.uint64)
        cap = self.fp_arena_bound(desc) + int(self.lib.mfp_fp_arena_bound(n, n * 8400))
        fp = np.zeros(cap, dtype=np.uint8)
        an = ap = None
        if analysis:
            an = np.zeros(max(n, 1), dtype=ANALYSIS_DTYPE)
            ap = np.zeros((max(n, 1), ATTR_DB_TAGS), np.float64)
        used = self.lib.mfp_process_batch_reassembly_context(
            self.h, self.reasm, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
            None if ts is None else ts.ctypes.data, rec.ctypes.data, fp.ctypes.data, cap, props.ctypes.data,
            out_desc.ctypes.data, None if an is None else an.ctypes.data, None if ap is None else ap.ctypes.data,
            more.ctypes.data)
        if used < 0:
            raise MercuryAmdError("mfp_process_batch_reassembly_context failed: " + _err(self.lib))
        flen = ctypes.c_size_t(0)
        ptr = self.lib.mfp_reassembler_frames(self.reasm, ctypes.byref(flen))
        frames = np.ctypeslib.as_array((ctypes.c_uint8 * flen.value).from_address(ptr)).copy() if flen.value else \
            np.zeros(0, np.uint8)
        return (rec, fp[:used].tobytes(), props[:n], np.concatenate([arena, frames]), out_desc[:n],
                None if an is None else an[:n], None if ap is None else ap[:n], more[:n])

    @property
    def analysis_enabled(self):
        return bool(self.lib.mfp_analysis_enabled(self.h))

    def process_host_analysis(self, arena, desc, attr_prob=False):
        """Fingerprint + classify a host batch -> (records, fp arena bytes, analysis
        records), plus the (n, ATTR_DB_TAGS) attribute probabilities when attr_prob."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        an = np.zeros(n, dtype=ANALYSIS_DTYPE)
        ap = np.zeros((max(n, 1), ATTR_DB_TAGS), np.float64) if attr_prob else None
        cap = self.fp_arena_bound(desc)
        fp = np.zeros(cap, dtype=np.uint8)
        used = self.lib.mfp_process_batch_host_ex(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                                  rec.ctypes.data, fp.ctypes.data, cap, an.ctypes.data,
                                                  ap.ctypes.data if ap is not None else None)
        if used < 0:
            raise MercuryAmdError("mfp_process_batch_host_ex failed: " + _err(self.lib))
        if attr_prob:
            return rec, fp[:used].tobytes(), an, ap[:n]
        return rec, fp[:used].tobytes(), an

    def process_pipelined(self, arena, desc, chunk=0, analysis=False, out=None, attr_prob=None):
        """Host batch through the two-stream pipeline (mfp_process_pipelined).
        `out`: optional preallocated (records, fp arena, analysis) host arrays
        (page-locked for full PCIe rate); attr_prob: None, or a float64 array
        of n * ATTR_DB_TAGS for the attribute probabilities.  Returns (records,
        fp arena bytes used, analysis records or None)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        if out is None:
            rec = np.zeros(n, dtype=RECORD_DTYPE)
            fp = np.zeros(self.fp_arena_bound(desc), dtype=np.uint8)
            an = np.zeros(n, dtype=ANALYSIS_DTYPE) if analysis else None
        else:
            rec, fp, an = out
        if attr_prob is not None and attr_prob.size < n * ATTR_DB_TAGS:
            raise ValueError("attr_prob needs n * ATTR_DB_TAGS doubles")
        used = self.lib.mfp_process_pipelined(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                              rec.ctypes.data, fp.ctypes.data, fp.nbytes,
                                              an.ctypes.data if an is not None else None,
                                              attr_prob.ctypes.data if attr_prob is not None else None, chunk)
        if used < 0:
            raise MercuryAmdError("mfp_process_pipelined failed: " + _err(self.lib))
        return rec, int(used), an

    def analyze_device(self, d_arena, d_desc, n, d_rec, d_fp, d_out, stream=0, d_attr_prob=None):
        r = self.lib.mfp_analyze_batch_device(self.h, d_arena, d_desc, n, d_rec, d_fp, d_out, d_attr_prob, stream)
        if r != 0:
            raise MercuryAmdError("mfp_analyze_batch_device failed: " + _err(self.lib))

    def analyze_device_pipelined(self, d_arena, d_desc, n, d_rec, d_fp, d_out, stream=0, d_attr_prob=None):
        """mfp_analyze_batch_device_pipelined: this batch's kernels run while
        the previous batch's sightings are decided; a batch's records are final
        after the next call or analysis_flush()."""
        r = self.lib.mfp_analyze_batch_device_pipelined(self.h, d_arena, d_desc, n, d_rec, d_fp, d_out, d_attr_prob,
                                                         stream)
        if r != 0:
            raise MercuryAmdError("mfp_analyze_batch_device_pipelined failed: " + _err(self.lib))

    def analysis_flush(self):
        if self.lib.mfp_analysis_flush(self.h) != 0:
            raise MercuryAmdError("mfp_analysis_flush failed: " + _err(self.lib))

    def analyze_device_deferred_pipelined(self, d_arena, d_desc, n, d_rec, d_fp, d_out, stream=0, d_attr_prob=None):
        """mfp_analyze_batch_device_deferred_pipelined (a deferred context, the
        shards of one stream): this batch's kernels are launched and the previous
        batch, if undecided, is the one analysis_distinct / analysis_resolve* act
        on -- shard.ordered_prevalence_merge decides it while the device runs
        this one."""
        r = self.lib.mfp_analyze_batch_device_deferred_pipelined(self.h, d_arena, d_desc, n, d_rec, d_fp, d_out,
                                                                  d_attr_prob, stream)
        if r != 0:
            raise MercuryAmdError("mfp_analyze_batch_device_deferred_pipelined failed: " + _err(self.lib))

    def analysis_defer_newest(self):
        """After the last deferred pipelined call: the analysis_* calls act on its batch."""
        if self.lib.mfp_analysis_defer_newest(self.h) != 0:
            raise MercuryAmdError("mfp_analysis_defer_newest failed: " + _err(self.lib))

    def process_name(self, pid):
        if pid == NO_PROCESS:
            return ""
        s = self.lib.mfp_process_name(self.h, int(pid))
        return s.decode() if s else None

    def attribute_name(self, bit):
        s = self.lib.mfp_attribute_name(self.h, int(bit))
        return s.decode() if s else None

    def device_table_bytes(self):
        """Bytes of the classifier's tables in HBM."""
        return int(self.lib.mfp_analysis_device_bytes(self.h))

    def attribute_count(self):
        return int(self.lib.mfp_attribute_count(self.h))

    def resource_version(self):
        s = self.lib.mfp_resource_version(self.h)
        return s.decode() if s is not None else None

    def report_os(self, on=True):
        """libmerc_config.report_os: os_info of the selected process in results."""
        if self.lib.mfp_analysis_report_os(self.h, 1 if on else 0) != 0:
            raise MercuryAmdError(_err(self.lib))

    def os_info(self, proc_slot):
        """[(os name, prevalence)] of a process slot (empty unless report_os)."""
        if proc_slot == NO_PROCESS:
            return []
        nm, pv = ctypes.c_char_p(), ctypes.c_uint64(0)
        cnt = self.lib.mfp_process_os_info(self.h, int(proc_slot), 0, None, None)
        if cnt < 0:
            raise MercuryAmdError(_err(self.lib))
        out = []
        for k in range(cnt):
            self.lib.mfp_process_os_info(self.h, int(proc_slot), k, ctypes.byref(nm), ctypes.byref(pv))
            out.append((nm.value.decode("latin-1"), int(pv.value)))
        return out

    def analysis_stats(self):
        out = (ctypes.c_uint64 * 4)()
        if self.lib.mfp_analysis_stats(self.h, out) != 0:
            raise MercuryAmdError(_err(self.lib))
        return list(out)

    COUNTER_NAMES = ("classified", "pending", "oversize", "deferred", "lane_priors", "lane_updates", "wave_priors",
                     "wave_updates", "work_items", "lane_scored", "feature_slots", "seen_merges")

    def analysis_counters(self):
        """The last analysis batch's device counters (mfp_analysis_counters) as a dict."""
        out = (ctypes.c_uint64 * len(self.COUNTER_NAMES))()
        if self.lib.mfp_analysis_counters(self.h, out, len(self.COUNTER_NAMES)) != 0:
            raise MercuryAmdError(_err(self.lib))
        return dict(zip(self.COUNTER_NAMES, (int(x) for x in out)))

    def profile(self, on=True):
        """Bracket every kernel launch of this context with HIP events (resets the totals)."""
        if self.lib.mfp_profile_enable(self.h, 1 if on else 0) != 0:
            raise MercuryAmdError(_err(self.lib))

    def profile_read(self):
        """{kernel name: (launches, total ms)} since profile(True), in first-launch order."""
        out = {}
        name = ctypes.create_string_buffer(64)
        cnt, ms = ctypes.c_uint64(0), ctypes.c_double(0.0)
        i = 0
        while True:
            r = self.lib.mfp_profile_read(self.h, i, name, 64, ctypes.byref(cnt), ctypes.byref(ms))
            if r == 1:
                return out
            if r != 0:
                raise MercuryAmdError(_err(self.lib))
            out[name.value.decode()] = (int(cnt.value), float(ms.value))
            i += 1

    # ---- the unknown-TLS prevalence LRU (see include/mfp.h) ----
    def prevalence(self):
        return Prevalence(handle=self.lib.mfp_analysis_prevalence(self.h))

    def set_prevalence(self, prev):
        if self.lib.mfp_analysis_set_prevalence(self.h, prev.h if prev is not None else None) != 0:
            raise MercuryAmdError(_err(self.lib))

    def defer(self, on=True):
        if self.lib.mfp_analysis_defer(self.h, 1 if on else 0) != 0:
            raise MercuryAmdError(_err(self.lib))

    def analysis_distinct(self):
        """The last deferred batch's distinct unknown-TLS fingerprints
        (SIGHTING_DTYPE), or None when the batch has too many for its table."""
        n = self.lib.mfp_analysis_distinct(self.h, None, 0)
        if n == -3:
            return None
        if n < 0:
            raise MercuryAmdError(_err(self.lib))
        out = np.zeros(max(n, 1), SIGHTING_DTYPE)
        self.lib.mfp_analysis_distinct(self.h, out.ctypes.data, n)
        return out[:n]

    def analysis_distinct_count(self):
        """How many distinct unknown-TLS fingerprints the last deferred batch
        has (its table's counter; no export), or None when too many for it."""
        n = self.lib.mfp_analysis_distinct(self.h, None, 0)
        if n == -3:
            return None
        if n < 0:
            raise MercuryAmdError(_err(self.lib))
        return int(n)

    def analysis_sequence(self):
        n = self.lib.mfp_analysis_sequence(self.h, None, 0)
        if n < 0:
            raise MercuryAmdError(_err(self.lib))
        out = np.zeros(max(n, 1), np.uint64)
        self.lib.mfp_analysis_sequence(self.h, out.ctypes.data, n)
        return out[:n]

    def analysis_resolve(self, sightings):
        d = np.ascontiguousarray(sightings, SIGHTING_DTYPE)
        if self.lib.mfp_analysis_resolve(self.h, d.ctypes.data, len(d)) != 0:
            raise MercuryAmdError(_err(self.lib))

    def last_analysis(self):
        """The last analysed batch's analysis records as they are on the device now."""
        n = self.lib.mfp_analysis_last(self.h, None, 0)
        if n < 0:
            raise MercuryAmdError(_err(self.lib))
        out = np.zeros(max(n, 1), ANALYSIS_DTYPE)
        self.lib.mfp_analysis_last(self.h, out.ctypes.data, n)
        return out[:n]

    def analysis_resolve_sequence(self, seen):
        b = np.ascontiguousarray(seen, np.uint8)
        if self.lib.mfp_analysis_resolve_sequence(self.h, b.ctypes.data, len(b)) != 0:
            raise MercuryAmdError(_err(self.lib))

    def process_device(self, d_arena, d_desc, n, d_rec, d_fp, fp_cap, d_used, stream=0):
        """All arguments are device pointers (ints, e.g. torch data_ptr())."""
        r = self.lib.mfp_process_batch_device(self.h, d_arena, d_desc, n, d_rec, d_fp, fp_cap, d_used, stream)
        if r != 0:
            raise MercuryAmdError("mfp_process_batch_device failed: " + _err(self.lib))


class Prevalence:
    """The unknown-TLS prevalence LRU (fingerprint_prevalence, analysis.h:362-421):
    mfp_prevalence_* on the host.  `owned=False` wraps a context's own object."""

    def __init__(self, capacity=100000, handle=None):
        self.lib = load_library()
        self.owned = handle is None
        self.h = handle if handle is not None else self.lib.mfp_prevalence_create(capacity)
        if not self.h:
            raise MercuryAmdError(_err(self.lib))

    def close(self):
        if self.h and self.owned:
            self.lib.mfp_prevalence_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.lib.mfp_prevalence_size(self.h))

    def __contains__(self, h):
        return bool(self.lib.mfp_prevalence_contains(self.h, int(h)))

    def keys(self):
        """Hashes from least to most recently used."""
        n = self.lib.mfp_prevalence_keys(self.h, None, 0)
        out = np.zeros(max(n, 1), np.uint64)
        self.lib.mfp_prevalence_keys(self.h, out.ctypes.data, n)
        return out[:n]

    def resolve_sequence(self, hashes):
        """seen[j] = 1 when hashes[j] was in the set at sighting j (unlabeled)."""
        h = np.ascontiguousarray(hashes, np.uint64)
        seen = np.zeros(max(len(h), 1), np.uint8)
        if self.lib.mfp_prevalence_resolve_sequence(self.h, h.ctypes.data, len(h), seen.ctypes.data) != 0:
            raise MercuryAmdError(_err(self.lib))
        return seen[:len(h)]

    @property
    def capacity(self):
        return int(self.lib.mfp_prevalence_capacity(self.h))

    def summary(self, hashes):
        """The distinct hashes of one shard's sightings by last sighting, most
        recent first, at most the capacity (mfp_prevalence_summary)."""
        h = np.ascontiguousarray(hashes, np.uint64)
        out = np.zeros(max(self.capacity, 1), np.uint64)
        k = self.lib.mfp_prevalence_summary(self.h, h.ctypes.data, len(h), out.ctypes.data)
        if k < 0:
            raise MercuryAmdError(_err(self.lib))
        return out[:k]

    def resolve_shard(self, hashes, prior):
        """Decide one shard's sightings from the set the earlier shards'
        summaries (`prior`, the nearest shard's first) leave on top of this
        set; the set itself is not changed."""
        h = np.ascontiguousarray(hashes, np.uint64)
        pr = np.ascontiguousarray(prior, np.uint64)
        seen = np.zeros(max(len(h), 1), np.uint8)
        if self.lib.mfp_prevalence_resolve_shard(self.h, h.ctypes.data, len(h), pr.ctypes.data, len(pr),
                                                 seen.ctypes.data) != 0:
            raise MercuryAmdError(_err(self.lib))
        return seen[:len(h)]

    def advance(self, recent):
        """This set becomes the set after a step of shards (`recent`: every
        shard's summary, the last shard's first)."""
        r = np.ascontiguousarray(recent, np.uint64)
        if self.lib.mfp_prevalence_advance(self.h, r.ctypes.data, len(r)) != 0:
            raise MercuryAmdError(_err(self.lib))

    def distinct_exact(self, sightings):
        d = np.ascontiguousarray(sightings, SIGHTING_DTYPE)
        return self.lib.mfp_prevalence_distinct_exact(self.h, d.ctypes.data, len(d)) == 1

    def resolve_distinct(self, sightings):
        """Decide first_seen of each entry in place; False (nothing applied)
        when the entries could evict."""
        if len(sightings) and not sightings.flags["C_CONTIGUOUS"]:
            raise ValueError("sightings must be contiguous (decided in place)")
        r = self.lib.mfp_prevalence_resolve_distinct(self.h, sightings.ctypes.data, len(sightings))
        if r == -2:
            return False
        if r != 0:
            raise MercuryAmdError(_err(self.lib))
        return True


def resource_stats(path, enc_key=None):
    """Host-only load of a resource archive (enc_key: 16-byte key of an
    encrypted one): {fingerprints, entries, processes, updates, ...}."""
    lib = load_library()
    out = (ctypes.c_uint64 * 8)()
    key = None if enc_key is None else ctypes.create_string_buffer(bytes(enc_key), 16)
    if lib.mfp_resource_stats_ex(path.encode(), key, out) != 0:
        raise MercuryAmdError(_err(lib))
    keys = ["fingerprints", "entries", "processes", "updates", "known_prevalence", "asn_prefixes", "disabled",
            "process_names"]
    return dict(zip(keys, list(out)))


def lpm_query(resources, queries):
    """Host-only: the archive's subnet LC-tries built as the device gets them
    and queried with the device's lookup; queries = [(dst_ip, server_name)].
    Returns [(asn, domain_faking)] (subnet_data::get_asn_info /
    is_domain_faking, addr.cc:172-208, 707-792)."""
    lib = load_library()
    text = "".join(f"{ip}\t{name}\n" for ip, name in queries).encode("latin-1")
    n = len(queries)
    asn = np.zeros(max(n, 1), np.uint32)
    fake = np.zeros(max(n, 1), np.int8)
    got = lib.mfp_lpm_query(resources.encode(), text, asn.ctypes.data, fake.ctypes.data, n)
    if got < 0:
        raise MercuryAmdError(_err(lib))
    return [(int(asn[i]), int(fake[i])) for i in range(got)]


def normalize_server_name(name):
    """server_identifier::get_normalized_domain_name as the device applies it (host)."""
    lib = load_library()
    b = name if isinstance(name, bytes) else name.encode("latin-1")
    buf = ctypes.create_string_buffer(512)
    n = lib.mfp_normalize_server_name(b, len(b), buf, 512)
    if n < 0:
        raise MercuryAmdError("normalize_server_name failed")
    return buf.raw[:n].decode("latin-1")


def parse_filter(cfg):
    """packet_filter_cfg -> (selection bits, tls format); host only."""
    lib = load_library()
    sel, fmt = ctypes.c_uint32(0), ctypes.c_uint32(0)
    if lib.mfp_parse_filter(None if cfg is None else cfg.encode(), ctypes.byref(sel), ctypes.byref(fmt)) < 0:
        raise MercuryAmdError(_err(lib))
    return sel.value, fmt.value


def parse_filter_ex(cfg):
    """packet_filter_cfg -> (selection bits, bits of the selected protocols
    outside the path that are identified first); host only."""
    lib = load_library()
    sel, fmt, other = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
    rc = lib.mfp_parse_filter_ex(None if cfg is None else cfg.encode(), ctypes.byref(sel), ctypes.byref(fmt),
                                 ctypes.byref(other))
    if rc < 0:
        raise MercuryAmdError(_err(lib))
    return sel.value, other.value, (_err(lib) if rc > 0 else "")


def fingerprints(rec, fp_arena):
    """Per-packet fingerprint strings from records + arena bytes."""
    out = []
    for r in rec:
        n = int(r["fp_len"])
        if r["fp_type"] == 0 or n == 0:
            out.append("")
        else:
            o = int(r["fp_offset"])
            out.append(fp_arena[o:o + n].decode("latin-1"))
    return out


class PcapReader:
    """Classic pcap file -> packet batches (arena, descriptors, timestamps):
    mfp_pcap_open / mfp_pcap_read_batch, the reference's pcap_file_open and
    pcap_file_read_packet semantics (src/pcap_file_io.c:106-254, 393-468).
    Host only."""

    def __init__(self, path):
        self.lib = load_library()
        self.h = self.lib.mfp_pcap_open(os.fsencode(path))
        if not self.h:
            raise MercuryAmdError(_err(self.lib))
        self.linktype = self.lib.mfp_pcap_linktype(self.h)

    def read_batch(self, max_pkts=65536, arena_bytes=64 << 20):
        """Up to max_pkts packets: (arena u8 incl. 16 zero bytes of slack,
        desc DESC_DTYPE, ts_ns u64); empty arrays at the end of the file."""
        arena = np.empty(max(arena_bytes, 65536 + 16), np.uint8)
        desc = np.empty(max_pkts, DESC_DTYPE)
        ts = np.empty(max_pkts, np.uint64)
        used = ctypes.c_size_t(0)
        n = self.lib.mfp_pcap_read_batch(self.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, max_pkts,
                                         ts.ctypes.data, ctypes.byref(used))
        if n < 0:
            raise MercuryAmdError("pcap read failed: " + _err(self.lib))
        return arena[:used.value + 16], desc[:n], ts[:n]

    def __iter__(self):
        while True:
            a, d, t = self.read_batch()
            if len(d) == 0:
                return
            yield a, d, t

    def close(self):
        if self.h:
            self.lib.mfp_pcap_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tpacket3_block(block, max_pkts=4096):
    """Descriptors + ns timestamps for the packets of one TPACKET_V3 ring
    block (a uint8 array; it is the arena, zero copy): mfp_tpacket3_block,
    process_all_packets_in_block (src/af_packet_v3.c:174-210)."""
    lib = load_library()
    block = np.ascontiguousarray(block, dtype=np.uint8)
    desc = np.empty(max_pkts, DESC_DTYPE)
    ts = np.empty(max_pkts, np.uint64)
    n = lib.mfp_tpacket3_block(block.ctypes.data, block.ctypes.data, block.nbytes, desc.ctypes.data, max_pkts,
                               ts.ctypes.data)
    if n < 0:
        raise MercuryAmdError(_err(lib))
    return desc[:n], ts[:n]


def write_json(arena, desc, rec, fp_arena, ts_ns=None, threads=1, ctx=None, analysis=None, attr_prob=None,
               props=None):
    """JSON record lines for a fingerprinted batch (mfp_write_json_batch: the
    text of stateful_pkt_proc::write_json, src/libmerc/pkt_proc.cc:1157-1253);
    with ctx + analysis (+ attr_prob), the --analysis "analysis" objects
    (mfp_write_json_batch_analysis); with props (process_host_reassembly's
    output, whose arena/desc go with it) the reassembler's properties
    (mfp_write_json_batch_reassembly).  Returns (list of per-packet lines as
    bytes, b"" when the reference writes nothing; count of records that could
    not be rebuilt). Host only."""
    lib = load_library()
    an = None if analysis is None else np.ascontiguousarray(analysis, dtype=ANALYSIS_DTYPE)
    ap = None if attr_prob is None else np.ascontiguousarray(attr_prob, dtype=np.float64)
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    rec = np.ascontiguousarray(rec, dtype=RECORD_DTYPE)
    fp = np.frombuffer(bytes(fp_arena) + b"\0", dtype=np.uint8)
    n = len(desc)
    ts = None if ts_ns is None else np.ascontiguousarray(ts_ns, dtype=np.uint64)
    ends = np.zeros(max(n, 1), np.uint64)
    skipped = ctypes.c_uint64(0)
    cap = 1 << 16
    while True:
        out = np.empty(cap, np.uint8)
        if props is not None and an is not None:
            pr = np.ascontiguousarray(props, dtype=np.uint16)
            got = lib.mfp_write_json_batch_reassembly_analysis(
                ctx.h, arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data, fp.ctypes.data, pr.ctypes.data,
                an.ctypes.data, None if ap is None else ap.ctypes.data, None if ts is None else ts.ctypes.data,
                out.ctypes.data, cap, ends.ctypes.data, ctypes.byref(skipped), int(threads))
        elif props is not None:
            pr = np.ascontiguousarray(props, dtype=np.uint16)
            got = lib.mfp_write_json_batch_reassembly(arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data,
                                                      fp.ctypes.data, pr.ctypes.data,
                                                      None if ts is None else ts.ctypes.data, out.ctypes.data, cap,
                                                      ends.ctypes.data, ctypes.byref(skipped), int(threads))
        elif an is not None:
            got = lib.mfp_write_json_batch_analysis(ctx.h, arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data,
                                                    fp.ctypes.data, an.ctypes.data,
                                                    None if ap is None else ap.ctypes.data,
                                                    None if ts is None else ts.ctypes.data, out.ctypes.data, cap,
                                                    ends.ctypes.data, ctypes.byref(skipped), int(threads))
        else:
            got = lib.mfp_write_json_batch(arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data, fp.ctypes.data,
                                           None if ts is None else ts.ctypes.data, out.ctypes.data, cap,
                                           ends.ctypes.data, ctypes.byref(skipped), int(threads))
        if got == -2:
            cap *= 4
            continue
        if got < 0:
            raise MercuryAmdError("mfp_write_json_batch failed: " + _err(lib))
        break
    buf = out[:got].tobytes()
    lines, prev = [], 0
    for i in range(n):
        e = int(ends[i])
        lines.append(buf[prev:e])
        prev = e
    return lines, int(skipped.value)
