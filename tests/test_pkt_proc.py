"""The batch packet processors (include/mfp_pkt_proc.h,
mercury_amd/csrc/mfp_pktproc.cpp) behind the reference's pkt_proc plugin
interface (src/pkt_proc.hpp:26-33), driven packet by packet through apply()
as pcap_file_dispatch_pkt_processor (src/pcap_file_io.c:470-512) drives the
reference's processors:

* MFP_PKT_PROC_JSON in place of pkt_proc_json_writer_llq
  (src/pkt_processing.h:129-173): the whole output byte-identical to the
  reference's write_json text (tests/golden/json_*.txt.gz, reasm_json_*,
  json_an_*), with "analysis" objects and reassembly;
* MFP_PKT_PROC_FILTER_PCAP in place of pkt_proc_filter_pcap_writer_llq
  (`mercury -w`, src/pkt_processing.h:230-259): the whole pcap file
  byte-identical to the reference's (tests/golden/pcapw_*.pcap.gz from
  tests/golden/make_golden_pcapw.py, the driver's "pcapw" mode), including
  the packets written only because they fed the reassembler (dump_pkt,
  pkt_proc.cc:1842-1845) and the Ethernet-only parse of other link types;
* the `mercury-amd` driver binary (mercury_amd/csrc/mfp_drv.cpp) on pcap
  files, both outputs;
* CPU: the C++ pkt_proc subclasses (include/mercury_amd_pkt_proc.hpp) compile
  against the reference's own src/pkt_proc.hpp when that tree is present, and
  against their standalone declaration; the pcap file header.
Batch sizes are small (7 ... 1000 packets) so every stream crosses many
batches: flow state, dump_pkt and the prevalence LRU carry across them.
"""
import gzip
import json
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import mercury_amd
from mercury_amd import api

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
INC = os.path.join(ROOT, "include")
REF_SRC = "/root/reference/src"
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"
TS = 1700000000
MANIFEST = json.load(open(os.path.join(GOLD, "pcapw_manifest.json")))
DRV = os.path.join(ROOT, "mercury_amd", "mercury-amd")


def _gold_json(name):
    with gzip.open(os.path.join(GOLD, name), "rb") as f:
        lines = f.read().split(b"\n")[:-1]
    return b"".join(l + b"\n" for l in lines if l)


def _gold_pcap(name):
    with gzip.open(os.path.join(GOLD, f"pcapw_{name}.pcap.gz"), "rb") as f:
        return f.read()


def _npz(name):
    z = np.load(os.path.join(GOLD, name))
    return z["arena"], z["desc"], (z["ts"].astype(np.uint64) if "ts" in z else None)


def _packets(arena, desc):
    for d in desc:
        o, n = int(d["offset"]), int(d["caplen"])
        yield bytes(arena[o:o + n]), int(d["linktype"])


def _reasm_stream():
    from tests import test_reassembly
    return test_reassembly.load_stream()


def _stream(name):
    """(arena, desc, ts_sec or None) of a golden case."""
    from tests import synth
    if name == "ref":
        return _npz("ref_packets.npz")
    if name == "synth":
        return synth.batch(4000, seed=0x5EED0003) + (None,)
    if name == "reasm_r0":
        return _reasm_stream() + (None,)
    if name == "reasm_timed":
        return _npz("reasm_timed_packets.npz")
    if name == "dtls_d0":
        return _npz("dtls_reasm_packets.npz")
    if name == "quic_q0":
        return _npz("quic_reasm_packets.npz")
    if name in ("quic", "stun_ovpn", "tunnel"):       # (their npz carry a "sources" column, no times)
        z = np.load(os.path.join(GOLD, f"{name}_packets.npz"))
        return z["arena"], z["desc"], None
    raise KeyError(name)


def _run(config, kind, arena, desc, ts=None, batch=1000, **kw):
    ctx = mercury_amd.Context(config, device=0)
    try:
        p = mercury_amd.PacketProcessor(ctx, kind, batch_pkts=batch, **kw)
        try:
            for i, (pkt, lt) in enumerate(_packets(arena, desc)):
                p.apply(pkt, ts_sec=int(ts[i]) if ts is not None else TS, linktype=lt)
            p.finalize()
            st = p.stats()
            out = bytes(p.out)
        finally:
            p.close()
    finally:
        ctx.close()
    assert st["packets"] == len(desc) and st["skipped"] == 0
    return out, st


def _first_diff(a, b):
    n = min(len(a), len(b))
    i = next((k for k in range(n) if a[k] != b[k]), n)
    return f"first difference at byte {i} of {len(a)} / {len(b)}: {a[max(0, i - 60):i + 60]!r} vs {b[max(0, i - 60):i + 60]!r}"


# ---------------------------------------------------------------- CPU tests

def _compile(tu, flags):
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.cc")
        with open(src, "w") as f:
            f.write(tu)
        r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-c", src, "-o", os.path.join(d, "t.o")] + flags,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


TU = """
#include "mercury_amd_pkt_proc.hpp"
// the factory's choice (pkt_proc_new_from_config src/pkt_processing.cc:14-52)
// with the device processors in place of the reference's two
struct pkt_proc *make(mfp_context ctx, bool write_pcap, FILE *out) {
    if (write_pcap) {
        mercury_amd::write_pcap_header(out);
        return new mercury_amd::pkt_proc_gpu_filter_pcap_writer(ctx, out);
    }
    return new mercury_amd::pkt_proc_gpu_json_writer(ctx, out);
}
void drive(struct pkt_proc *p, struct packet_info *pi, uint8_t *pkt) { p->apply(pi, pkt); p->flush(); p->finalize(); }
"""


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "pkt_proc.hpp")), reason="reference tree absent")
def test_subclasses_compile_against_reference_pkt_proc():
    """The subclasses derive from the reference's own struct pkt_proc."""
    _compile(TU + '\nstatic_assert(sizeof(packet_info::linktype) == 2, "");\n', ["-I" + REF_SRC, "-I" + INC])


def test_subclasses_compile_standalone():
    _compile(TU, ["-I" + INC])


def test_pcap_file_header():
    """write_pcap_file_header (pcap_file_io.c:88-104), as the reference's
    output file starts."""
    h = mercury_amd.pcap_file_header()
    assert h == struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1)
    for name in MANIFEST["cases"]:
        assert _gold_pcap(name)[:24] == h


def test_golden_pcapw_shapes():
    """The goldens: every record's incl_len == orig_len, the counts of the
    manifest, and (no reassembly) exactly the packets with a JSON record."""
    for name, m in MANIFEST["cases"].items():
        blob = _gold_pcap(name)
        o, k = 24, 0
        while o < len(blob):
            s, u, incl, orig = struct.unpack_from("<IIII", blob, o)
            assert incl == orig and u == 0
            o += 16 + incl
            k += 1
        assert o == len(blob) and k == m["written"]
        if "reassembly" not in m["config"]:
            assert m["dump_only"] == 0
        else:
            assert m["dump_only"] > 0


def test_driver_built():
    assert os.access(DRV, os.X_OK), "mercury_amd/mercury-amd missing: run __graft_entry__.build()"
    r = subprocess.run([DRV], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


# ---------------------------------------------------------------- GPU tests

@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", [("ref", 1000), ("synth", 333), ("reasm_r0", 97), ("reasm_timed", 7),
                                        ("dtls_d0", 13), ("quic_q0", 50)])
def test_filter_pcap_vs_reference(name, batch):
    arena, desc, ts = _stream(name)
    out, st = _run(MANIFEST["cases"][name]["config"], api.PKT_PROC_FILTER_PCAP, arena, desc, ts, batch=batch)
    want = _gold_pcap(name)[24:]
    assert out == want, _first_diff(out, want)
    assert st["records"] == MANIFEST["cases"][name]["written"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,golden,config,batch", [
    ("ref", "json_ref.txt.gz", CONTRACT, 1000),
    ("synth", "json_synth.txt.gz", CONTRACT, 129),
    ("reasm_r0", "reasm_json_r0.txt.gz", "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly", 97),
    ("reasm_timed", "reasm_timed_json.txt.gz", "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly", 7),
    ("dtls_d0", "dtls_reasm_json_d0.txt.gz", "select=dtls;reassembly", 13),
    ("quic_q0", "quic_reasm_json_q0.txt.gz", "select=quic;reassembly", 50),
    ("quic", "quic_json_mix.txt.gz", "select=tls,dtls,ssh,http,tcp,tcp.syn_ack,quic;format=tls/1,quic/1", 300),
    ("stun_ovpn", "stun_ovpn_json_mix.txt.gz",
     "select=tls,dtls,ssh,http,tcp,tcp.syn_ack,stun,openvpn_tcp;format=tls/1", 700),
    ("tunnel", "tunnel_json_t0.txt.gz", "tls,dtls,ssh,http,tcp,tcp.syn_ack,quic,gre,vxlan,geneve", 111),
])
def test_json_writer_vs_reference(name, golden, config, batch):
    arena, desc, ts = _stream(name)
    out, st = _run(config, api.PKT_PROC_JSON, arena, desc, ts, batch=batch, json_threads=3)
    want = _gold_json(golden)
    assert out == want, _first_diff(out, want)
    assert st["records"] == want.count(b"\n")


@pytest.mark.gpu
@pytest.mark.parametrize("name,golden,res", [("synth", "json_an_synth.txt.gz", "synth_resources.tgz"),
                                              ("ref", "json_an_ref.txt.gz", "resources-test.tgz")])
def test_json_writer_analysis_vs_reference(name, golden, res):
    """--analysis: the "analysis" objects (report_os on, as the goldens were
    made), the prevalence LRU in stream order across batches."""
    arena, desc, ts = _stream(name)
    cfg = f"select={CONTRACT};resources={os.path.join(GOLD, res)};analysis;report_os"
    out, _ = _run(cfg, api.PKT_PROC_JSON, arena, desc, ts, batch=501)
    want = _gold_json(golden)
    assert out == want, _first_diff(out, want)


@pytest.mark.gpu
def test_json_writer_reassembly_analysis_vs_reference():
    arena, desc = _reasm_stream()
    cfg = f"select=tls,ssh,http,tcp,tcp.syn_ack;reassembly;resources={os.path.join(GOLD, 'resources-test.tgz')};analysis"
    out, _ = _run(cfg, api.PKT_PROC_JSON, arena, desc, None, batch=211)
    want = _gold_json("reasm_json_an.txt.gz")
    assert out == want, _first_diff(out, want)


@pytest.mark.gpu
def test_flush_timeout_and_drain():
    """flush() hands a partial batch over without waiting; a batch whose first
    packet waited flush_us is handed over from apply(); drain() waits; the
    output is the same stream whatever the cut."""
    import time
    from tests import synth
    arena, desc = synth.batch(4000, seed=0x5EED0003)
    desc = desc[:600]
    ctx = mercury_amd.Context(CONTRACT, device=0)
    p = mercury_amd.PacketProcessor(ctx, api.PKT_PROC_JSON, batch_pkts=100000, flush_us=1000)
    try:
        pk = list(_packets(arena, desc))
        for i, (b, lt) in enumerate(pk):
            p.apply(b, ts_sec=TS, linktype=lt)
            if i == 100:
                p.flush()
            if i in (200, 300):
                time.sleep(0.01)        # the next multiple of 64 packets trips the timeout
        p.drain()
        st = p.stats()
        assert st["batches"] >= 3 and st["packets"] == len(desc)
        p.finalize()
        got = bytes(p.out)
    finally:
        p.close()
        ctx.close()
    gold = _gold_json("json_synth.txt.gz")   # the first 600 packets' lines
    with gzip.open(os.path.join(GOLD, "json_synth.txt.gz"), "rb") as f:
        lines = f.read().split(b"\n")[:600]
    want = b"".join(l + b"\n" for l in lines if l)
    assert got == want and gold.startswith(want)


@pytest.mark.gpu
def test_refuses_analysis_mode_context():
    ctx = mercury_amd.Context(CONTRACT, device=0, mode=api.MODE_ANALYSIS)
    try:
        with pytest.raises(mercury_amd.MercuryAmdError, match="MFP_MODE_WRITE_JSON"):
            mercury_amd.PacketProcessor(ctx, api.PKT_PROC_JSON)
    finally:
        ctx.close()


def _write_pcap(path, arena, desc, ts):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, (b, _) in enumerate(_packets(arena, desc)):
            f.write(struct.pack("<IIII", int(ts[i]) if ts is not None else TS, 0, len(b), len(b)))
            f.write(b)


@pytest.mark.gpu
@pytest.mark.parametrize("name,golden,config", [
    ("synth", "json_synth.txt.gz", CONTRACT),
    ("reasm_timed", "reasm_timed_json.txt.gz", "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly"),
])
def test_driver_pcap_to_json_and_pcap(name, golden, config, tmp_path):
    """mercury-amd -r IN -f OUT.json / -w OUT.pcap: the reference's bytes."""
    arena, desc, ts = _stream(name)
    src = str(tmp_path / "in.pcap")
    _write_pcap(src, arena, desc, ts)
    for flag, want in (("-f", _gold_json(golden)), ("-w", _gold_pcap(name))):
        out = str(tmp_path / ("out" + flag))
        r = subprocess.run([DRV, "-r", src, flag, out, "-c", config, "-b", "50"], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        stats = json.loads(r.stderr.strip().splitlines()[-1])
        assert stats["packets"] == len(desc) and stats["skipped"] == 0
        got = open(out, "rb").read()
        assert got == want, (flag, _first_diff(got, want))
