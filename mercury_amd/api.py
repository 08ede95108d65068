"""ctypes binding of libmercury_amd.so (include/mfp.h)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

DESC_DTYPE = np.dtype([("offset", "<u8"), ("caplen", "<u4"), ("linktype", "<u2"), ("flags", "<u2")])
RECORD_DTYPE = np.dtype([("fp_offset", "<u8"), ("fp_len", "<u4"), ("fp_type", "u1"), ("msg", "u1"),
                         ("flags", "u1"), ("status", "u1"), ("sni_off", "<u2"), ("sni_len", "<u2"),
                         ("ua_off", "<u2"), ("ua_len", "<u2"), ("src_port", "<u2"), ("dst_port", "<u2"),
                         ("reserved", "<u4")])
assert DESC_DTYPE.itemsize == 16 and RECORD_DTYPE.itemsize == 32

# fingerprint::get_type_name (src/libmerc/fingerprint.h:159-192)
FP_TYPE_NAMES = ["unknown", "tls", "tls_server", "http", "http_server", "ssh", "ssh_kex", "tcp", "dhcp",
                 "smtp_server", "dtls", "dtls_server", "quic", "tcp_server", "openvpn", "tofsee", "stun",
                 "ssh_init", "ssh_server", "ssh_kex_server", "ssh_init_server"]
MSG_NAMES = ["none", "tls.client_hello", "tls.server_hello", "tls.certificate", "ssh.init", "ssh.kex",
             "http.request", "http.response", "tcp.syn", "tcp.syn_ack", "dtls.client_hello",
             "dtls.server_hello", "dtls.hello_verify_request"]

MODE_WRITE_JSON = 0
MODE_ANALYSIS = 1


class MercuryAmdError(RuntimeError):
    pass


def library_path():
    return os.path.join(_HERE, "libmercury_amd.so")


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
    lib.mfp_finalize.argtypes = [vp]
    lib.mfp_process_batch_device.restype = ctypes.c_int
    lib.mfp_process_batch_device.argtypes = [vp, vp, vp, sz, vp, vp, sz, vp, vp]
    lib.mfp_process_batch_host.restype = ctypes.c_longlong
    lib.mfp_process_batch_host.argtypes = [vp, vp, sz, vp, sz, vp, vp, sz]
    lib.mfp_fp_arena_bound.restype = sz
    lib.mfp_fp_arena_bound.argtypes = [sz, sz]
    lib.mfp_last_error.restype = ctypes.c_char_p
    lib.mfp_reference_version.restype = ctypes.c_uint32
    lib.mfp_parse_filter.restype = ctypes.c_int
    lib.mfp_parse_filter.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    _lib = lib
    return lib


def _err(lib):
    return lib.mfp_last_error().decode("utf-8", "replace")


class Context:
    """One device context (the analogue of libmerc's mercury_context plus a
    processor).  `config` uses the reference's packet_filter_cfg syntax."""

    def __init__(self, config="tls,dtls,ssh,http,tcp,tcp.syn_ack", device=0, mode=MODE_WRITE_JSON):
        self.lib = load_library()
        self.h = self.lib.mfp_init(config.encode() if config is not None else None, device, mode)
        if not self.h:
            raise MercuryAmdError("mfp_init failed: " + _err(self.lib))

    def close(self):
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

    def process_device(self, d_arena, d_desc, n, d_rec, d_fp, fp_cap, d_used, stream=0):
        """All arguments are device pointers (ints, e.g. torch data_ptr())."""
        r = self.lib.mfp_process_batch_device(self.h, d_arena, d_desc, n, d_rec, d_fp, fp_cap, d_used, stream)
        if r != 0:
            raise MercuryAmdError("mfp_process_batch_device failed: " + _err(self.lib))


def parse_filter(cfg):
    """packet_filter_cfg -> (selection bits, tls format); host only."""
    lib = load_library()
    sel, fmt = ctypes.c_uint32(0), ctypes.c_uint32(0)
    if lib.mfp_parse_filter(None if cfg is None else cfg.encode(), ctypes.byref(sel), ctypes.byref(fmt)) != 0:
        raise MercuryAmdError(_err(lib))
    return sel.value, fmt.value


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
