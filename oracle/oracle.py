"""ctypes binding for the C oracle (oracle/mfp_oracle.c) -- TEST
INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmfp_oracle.so")

SEL = {
    "tls.client_hello": 1 << 0, "tls.server_hello": 1 << 1, "tls.server_certificate": 1 << 2,
    "ssh.client": 1 << 3, "ssh.server": 1 << 4, "http.request": 1 << 5, "http.response": 1 << 6,
    "tcp": 1 << 7, "tcp.syn_ack": 1 << 8, "dtls": 1 << 9,
}
SEL["tls"] = SEL["tls.client_hello"] | SEL["tls.server_hello"] | SEL["tls.server_certificate"]
SEL["ssh"] = SEL["ssh.client"] | SEL["ssh.server"]
SEL["http"] = SEL["http.request"] | SEL["http.response"]
SEL_ALL = SEL["tls"] | SEL["ssh"] | SEL["http"] | SEL["tcp"] | SEL["tcp.syn_ack"] | SEL["dtls"]


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    src = os.path.join(HERE, "mfp_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        cmd = f"gcc -O2 -std=c11 -fPIC -shared -o {LIB} {src} -lpthread"
        if os.system(cmd) != 0:
            raise RuntimeError("oracle build failed: " + cmd)
    return LIB


class Config(ctypes.Structure):
    _fields_ = [("select", ctypes.c_uint32), ("tls_format", ctypes.c_uint32), ("mode", ctypes.c_uint32)]


class Result(ctypes.Structure):
    _fields_ = [("fp_type", ctypes.c_uint32), ("fp_len", ctypes.c_uint32), ("msg", ctypes.c_uint32),
                ("emit", ctypes.c_uint32), ("truncated", ctypes.c_uint32),
                ("sni_off", ctypes.c_int32), ("sni_len", ctypes.c_int32),
                ("ua_off", ctypes.c_int32), ("ua_len", ctypes.c_int32),
                ("ip_vers", ctypes.c_uint8), ("ip_proto", ctypes.c_uint8),
                ("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16),
                ("src_addr", ctypes.c_uint8 * 16), ("dst_addr", ctypes.c_uint8 * 16),
                ("fp", ctypes.c_char * 8193)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        _lib.mfpo_process.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint16,
                                      ctypes.POINTER(Config), ctypes.POINTER(Result)]
        _lib.mfpo_process_batch.restype = ctypes.c_longlong
        _lib.mfpo_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.POINTER(Config)] + [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
        _lib.mfpo_time_batch.restype = ctypes.c_double
        _lib.mfpo_time_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.POINTER(Config), ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_ulonglong)]
    return _lib


def config(select=SEL_ALL, tls_format=0, mode=0):
    return Config(select, tls_format, mode)


def process(pkt, linktype=1, cfg=None):
    cfg = cfg or config()
    r = Result()
    lib().mfpo_process(pkt, len(pkt), linktype, ctypes.byref(cfg), ctypes.byref(r))
    return r


def process_batch(arena, desc, cfg=None):
    """Returns (fp_type u8[n], fp_len u32[n], flags u8[n], list of fp strings)."""
    cfg = cfg or config()
    n = len(desc)
    fp_type = np.zeros(n, np.uint8)
    fp_len = np.zeros(n, np.uint32)
    flags = np.zeros(n, np.uint8)
    fp_off = np.zeros(n, np.uint64)
    cap = int(desc["caplen"].astype(np.int64).sum()) * 3 + 64 * n + 64
    out = np.zeros(cap, np.uint8)
    tot = lib().mfpo_process_batch(arena.ctypes.data, desc.ctypes.data, n, ctypes.byref(cfg),
                                   fp_type.ctypes.data, fp_len.ctypes.data, flags.ctypes.data,
                                   fp_off.ctypes.data, out.ctypes.data, cap)
    if tot < 0:
        raise RuntimeError("oracle fp arena too small")
    raw = out[:tot].tobytes()
    strs = [raw[int(o):int(o) + int(l)].decode("latin-1") for o, l in zip(fp_off, fp_len)]
    return fp_type, fp_len, flags, strs


def time_batch(arena, desc, cfg=None, threads=1, reps=1):
    cfg = cfg or config()
    b = ctypes.c_ulonglong(0)
    t = lib().mfpo_time_batch(arena.ctypes.data, desc.ctypes.data, len(desc), ctypes.byref(cfg),
                              threads, reps, ctypes.byref(b))
    return t, b.value
