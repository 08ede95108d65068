"""Host ingest: the pcap reader and the TPACKET_V3 block
walk fill batch arenas + descriptors the way the reference's readers hand
packets to pkt_proc::apply (src/pcap_file_io.c:106-254, 393-468;
src/af_packet_v3.c:174-210).  Host only: these run without a GPU, except the
last test, which pushes a pcap through the device path."""
import os
import struct

import numpy as np
import pytest

import mercury_amd
from tests import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REF_PCAP = "/root/reference/unit_tests/pcaps/top_100_fingerprints.pcap"


def write_pcap(path, pkts, linktype=1, big_endian=False, ts=None, network_field=None, incl=None):
    e = ">" if big_endian else "<"
    with open(path, "wb") as f:
        net = linktype if network_field is None else network_field
        f.write(struct.pack(e + "IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, net))
        for k, p in enumerate(pkts):
            sec, usec = ts[k] if ts else (1000 + k, 10 * k)
            n = len(p) if incl is None else incl[k]
            f.write(struct.pack(e + "IIII", sec, usec, n, n))
            f.write(p)


def packets(n, seed=1):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 1600, n)
    sizes[:3] = [0, 1, 65536]
    return [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]


def read_all(path, max_pkts=7, arena_bytes=1 << 20):
    out, ts = [], []
    with mercury_amd.PcapReader(path) as r:
        lt = r.linktype
        while True:
            a, d, t = r.read_batch(max_pkts=max_pkts, arena_bytes=arena_bytes)
            if len(d) == 0:
                break
            assert a[-16:].tobytes() == bytes(16)          # zero slack after the last packet
            for x in d:
                assert int(x["linktype"]) == lt and int(x["flags"]) == 0
                out.append(a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes())
            ts += [int(v) for v in t]
    return lt, out, ts


@pytest.mark.parametrize("big_endian", [False, True])
def test_pcap_round_trip(tmp_path, big_endian):
    pk = packets(300)
    p = tmp_path / "a.pcap"
    write_pcap(p, pk, big_endian=big_endian, network_field=(1 if not big_endian else 0x00010000))
    lt, got, ts = read_all(p)
    assert lt == 1
    assert got == pk
    assert ts == [(1000 + k) * 10**9 + 10 * k * 1000 for k in range(len(pk))]


def test_pcap_swapped_linktype_quirk(tmp_path):
    """A byte-swapped file's link type is htons() of the 32-bit field
    (pcap_file_io.c:236): Ethernet written big-endian reads as 0 (BSD
    loopback), as in the reference."""
    p = tmp_path / "be.pcap"
    write_pcap(p, packets(5), linktype=1, big_endian=True)
    with mercury_amd.PcapReader(p) as r:
        assert r.linktype == 0


def test_pcap_oversize_record(tmp_path):
    """A record longer than BUFLEN yields its first 65536 bytes; the next
    record is intact (pcap_file_io.c:438-456)."""
    big = bytes(range(256)) * 300          # 76 800 bytes
    pk = [b"\x01\x02", big, b"tail"]
    p = tmp_path / "big.pcap"
    write_pcap(p, pk)
    _, got, _ = read_all(p, max_pkts=2, arena_bytes=200000)
    assert got == [b"\x01\x02", big[:65536], b"tail"]


def test_pcap_arena_boundary(tmp_path):
    """A packet that does not fit the remaining arena starts the next batch."""
    pk = [bytes([k]) * 40000 for k in range(5)]
    p = tmp_path / "b.pcap"
    write_pcap(p, pk)
    with mercury_amd.PcapReader(p) as r:
        sizes = []
        while True:
            a, d, _ = r.read_batch(max_pkts=100, arena_bytes=100000)
            if len(d) == 0:
                break
            sizes.append(len(d))
            assert a.nbytes <= 100000
    assert sizes == [2, 2, 1]


def test_pcap_errors(tmp_path):
    ng = tmp_path / "x.pcapng"
    ng.write_bytes(struct.pack("<I", 0x0A0D0D0A) + bytes(60))
    with pytest.raises(mercury_amd.MercuryAmdError, match="pcap-ng"):
        mercury_amd.PcapReader(ng)
    bad = tmp_path / "lt.pcap"
    write_pcap(bad, [b"x"], linktype=147)
    with pytest.raises(mercury_amd.MercuryAmdError, match="linktype"):
        mercury_amd.PcapReader(bad)
    with pytest.raises(mercury_amd.MercuryAmdError):
        mercury_amd.PcapReader(tmp_path / "missing.pcap")
    # a record cut short: the packets before it are delivered, then an error
    cut = tmp_path / "cut.pcap"
    write_pcap(cut, [b"abcd", b"efgh", b"ij"], incl=[4, 4, 10])
    with mercury_amd.PcapReader(cut) as r:
        a, d, _ = r.read_batch(max_pkts=10)
        assert len(d) == 2
        with pytest.raises(mercury_amd.MercuryAmdError, match="caplen"):
            r.read_batch(max_pkts=10)
    # a partial record header is the end of the file
    part = tmp_path / "part.pcap"
    write_pcap(part, [b"abcd"])
    with open(part, "ab") as f:
        f.write(b"\x00" * 7)
    _, got, _ = read_all(part)
    assert got == [b"abcd"]


@pytest.mark.skipif(not os.path.exists(REF_PCAP), reason="reference tree not present")
def test_pcap_reference_file_matches_golden_packets():
    """The reference's own top_100_fingerprints.pcap read by mfp_pcap equals
    the packets committed in tests/golden/ref_packets.npz (made by
    tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLD, "ref_packets.npz"))
    sel = [i for i, s in enumerate(z["sources"]) if str(s).startswith("top_100_fingerprints.pcap:")]
    lt, got, _ = read_all(REF_PCAP, max_pkts=64)
    assert lt == 1 and len(sel) > 50
    for i in sel:                      # source "<file>:<packet index in the file>"
        k = int(str(z["sources"][i]).rsplit(":", 1)[1])
        o, n = int(z["desc"][i]["offset"]), int(z["desc"][i]["caplen"])
        assert got[k] == z["arena"][o:o + n].tobytes()


def make_block(pkts, first=48, pad=8):
    """A TPACKET_V3 block: tpacket_block_desc, then tpacket3_hdr + sockaddr_ll
    room + frame per packet, 16-byte aligned (linux/if_packet.h)."""
    hdrs, body, off = [], b"", first
    for k, p in enumerate(pkts):
        mac = 48 + 20 + pad                  # header, sockaddr_ll, padding
        size = (mac + len(p) + 15) & ~15
        nxt = size if k + 1 < len(pkts) else 0
        h = struct.pack("<IIIIIIHH", nxt, 500 + k, 1000 * k, len(p), len(p) + 4, 1, mac, 48) + bytes(20)
        frame = h + bytes(mac - len(h)) + p
        frame += bytes(size - len(frame))
        hdrs.append((off, mac))
        body += frame
        off += size
    bd = struct.pack("<II", 3, 0) + struct.pack("<IIIIQ", 1, len(pkts), first, first + len(body), 7) + bytes(16)
    bd += bytes(first - len(bd))
    return np.frombuffer(bd + body, np.uint8).copy(), hdrs


def test_tpacket3_block_walk():
    pk = packets(40, seed=5)[3:]
    blk, hdrs = make_block(pk)
    desc, ts = mercury_amd.tpacket3_block(blk, max_pkts=64)
    assert len(desc) == len(pk)
    for k, (d, (off, mac)) in enumerate(zip(desc, hdrs)):
        assert int(d["offset"]) == off + mac and int(d["linktype"]) == 1
        assert blk[int(d["offset"]):int(d["offset"]) + int(d["caplen"])].tobytes() == pk[k]
        assert int(ts[k]) == (500 + k) * 10**9 + 1000 * k
    with pytest.raises(mercury_amd.MercuryAmdError):
        mercury_amd.tpacket3_block(blk[:200], max_pkts=64)       # headers beyond the block
    with pytest.raises(mercury_amd.MercuryAmdError):
        mercury_amd.tpacket3_block(blk, max_pkts=4)


@pytest.mark.gpu
def test_pcap_ingest_to_device(tmp_path):
    """pcap file -> mfp_pcap batches -> device fingerprints == the reference's
    (tests/golden/cases/binmix.fp0: synthetic + fuzzed packets)."""
    from tests import cases
    pk = cases.binmix_case()
    p = tmp_path / "m.pcap"
    write_pcap(p, [b for _, b in pk])
    ctx = mercury_amd.Context("tls,dtls,ssh,http,tcp,tcp.syn_ack", device=0)
    got = []
    with mercury_amd.PcapReader(p) as r:
        for arena, desc, _ in r:
            rec, fp = ctx.process_host(arena, desc)
            got += mercury_amd.fingerprints(rec, fp)
    ctx.close()
    want = [row[3] for row in cases.load_golden("binmix", 0, "fp")]
    assert got == want and sum(1 for s in got if s) > 5000


@pytest.mark.parametrize("big_endian", [False, True])
def test_pcap_from_a_pipe_equals_the_file(tmp_path, big_endian):
    """A regular file is mapped whole; a pipe (or any stream) goes through the
    reader's block buffer (mfp_pcap.cpp): the same packets, times and
    truncation (a 70 000-byte record, BUFLEN = 65 536) either way, including
    records that straddle the buffer's refills."""
    import threading
    pk = packets(2500, seed=7) + [bytes(range(256)) * 274]          # the last: 70 144 bytes
    p = tmp_path / "a.pcap"
    write_pcap(p, pk, big_endian=big_endian, network_field=(1 if not big_endian else 0x00010000))
    want = read_all(p, max_pkts=64, arena_bytes=4 << 20)
    fifo = tmp_path / "a.fifo"
    os.mkfifo(fifo)
    blob = open(p, "rb").read()

    def feed():
        with open(fifo, "wb") as f:
            for k in range(0, len(blob), 100_003):    # odd-sized writes
                f.write(blob[k:k + 100_003])
    t = threading.Thread(target=feed)
    t.start()
    got = read_all(fifo, max_pkts=64, arena_bytes=4 << 20)
    t.join()
    assert got == want
    assert len(got[1]) == len(pk) and got[1][-1] == pk[-1][:65536]
