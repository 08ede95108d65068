"""Small helpers shared by tests, bench.py and the golden-vector generator:
classic-pcap reading, the packet batch layout (arena + 16-byte descriptors,
see include/mfp.h) and the "MFPB" batch file that oracle/_ref/merc_ref_drv
reads."""
import struct

import numpy as np

DESC_DTYPE = np.dtype([("offset", "<u8"), ("caplen", "<u4"), ("linktype", "<u2"), ("flags", "<u2")])


def read_pcap(path):
    """Return [(linktype, bytes)] for a classic pcap file."""
    with open(path, "rb") as f:
        buf = f.read()
    magic = struct.unpack_from("<I", buf, 0)[0]
    if magic in (0xA1B2C3D4, 0xA1B23C4D):
        e = "<"
    elif magic in (0xD4C3B2A1, 0x4D3CB2A1):
        e = ">"
    else:
        raise ValueError(f"{path}: not a classic pcap")
    lt = struct.unpack_from(e + "I", buf, 20)[0] & 0xFFFF
    out, o = [], 24
    while o + 16 <= len(buf):
        incl = struct.unpack_from(e + "I", buf, o + 8)[0]
        o += 16
        if o + incl > len(buf):
            break
        out.append((lt, buf[o:o + incl]))
        o += incl
    return out


def write_pcap(path, pkts, linktype=1):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, linktype))
        for i, p in enumerate(pkts):
            f.write(struct.pack("<IIII", 1700000000 + i, 0, len(p), len(p)))
            f.write(p)


def make_batch(pkts, align=1):
    """pkts: [(linktype, bytes)] -> (arena uint8 array, desc structured array)."""
    n = len(pkts)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    offs = []
    o = 0
    for lt, p in pkts:
        offs.append(o)
        o += len(p)
        if align > 1:
            o = (o + align - 1) // align * align
    arena = np.zeros(max(o, 1), dtype=np.uint8)
    for i, (lt, p) in enumerate(pkts):
        arena[offs[i]:offs[i] + len(p)] = np.frombuffer(p, dtype=np.uint8)
        desc[i] = (offs[i], len(p), lt, 0)
    return arena, desc


def write_mfpb(path, arena, desc):
    with open(path, "wb") as f:
        f.write(b"MFPB" + b"\0" * 4 + struct.pack("<Q", len(desc)))
        f.write(desc.tobytes())
        f.write(arena.tobytes())
