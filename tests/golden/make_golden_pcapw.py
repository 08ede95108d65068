"""Golden output of the REFERENCE's filtered pcap writer (`mercury -r in -w out`:
pkt_proc_filter_pcap_writer_llq, src/pkt_processing.h:230-259) for the batch
packet processor MFP_PKT_PROC_FILTER_PCAP (mercury_amd/csrc/mfp_pktproc.cpp).

Run in the dev container (needs oracle/_ref built by oracle/Makefile.ref):

    python tests/golden/make_golden_pcapw.py

The driver's "pcapw" mode (oracle/ref_driver.cc) runs each packet through the
reference processor's Ethernet write_json and writes it, in classic pcap
format behind the output file's header, when a record was written or
dump_pkt() is set (the packet fed the reassembler).  Outputs (committed),
each the whole pcap file, gzipped:
  pcapw_ref.pcap.gz          ref_packets.npz (65 unit-test pcaps, every link
                             type: the writer reads each as Ethernet)
  pcapw_synth.pcap.gz        synth.batch(4000, seed=0x5EED0003)
  pcapw_reasm_r0.pcap.gz     the TCP reassembly stream of test_reassembly.py
                             (ref packets + reasm_packets.npz), "reassembly"
  pcapw_reasm_timed.pcap.gz  reasm_timed_packets.npz with its capture times
  pcapw_dtls_d0.pcap.gz      dtls_reasm_packets.npz, select=dtls;reassembly
  pcapw_quic_q0.pcap.gz      quic_reasm_packets.npz, select=quic;reassembly
  pcapw_manifest.json        configurations and counts (records written,
                             packets written only for dump_pkt)
"""
import gzip
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"


def load_npz(name):
    z = np.load(os.path.join(HERE, name))
    return z["arena"], z["desc"], (z["ts"].astype(np.uint64) if "ts" in z else None)


def reasm_stream():
    z = np.load(os.path.join(HERE, "ref_packets.npz"))
    pk = [(int(d["linktype"]), bytes(z["arena"][int(d["offset"]):int(d["offset"]) + int(d["caplen"])]))
          for d in z["desc"]]
    s = np.load(os.path.join(HERE, "reasm_packets.npz"))
    syn = [(1, bytes(s["arena"][int(d["offset"]):int(d["offset"]) + int(d["caplen"])])) for d in s["desc"]]
    return pcaplib.make_batch(pk + syn)


def run(mode, arena, desc, config, ts_sec=None):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "b.mfpb")
        pcaplib.write_mfpb(p, arena, desc)
        env = dict(os.environ)
        if ts_sec is not None:
            tf = os.path.join(d, "ts.bin")
            np.asarray(ts_sec, dtype=np.uint64).tofile(tf)
            env["MERC_TS_FILE"] = tf
        return subprocess.run([REF, mode, p, config, "-"], capture_output=True, check=True, env=env).stdout


def pcap_records(blob):
    """[(ts_sec, ts_usec, bytes)] of a pcap file (after its 24-byte header)."""
    out, o = [], 24
    while o < len(blob):
        s, u, incl, orig = struct.unpack_from("<IIII", blob, o)
        assert incl == orig
        out.append((s, u, blob[o + 16:o + 16 + incl]))
        o += 16 + incl
    assert o == len(blob)
    return out


def main():
    cases = {
        "ref": (load_npz("ref_packets.npz")[:2], CONTRACT, None),
        "synth": (synth.batch(4000, seed=0x5EED0003), CONTRACT, None),
        "reasm_r0": (reasm_stream(), "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly", None),
        "reasm_timed": (load_npz("reasm_timed_packets.npz")[:2], "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly",
                        load_npz("reasm_timed_packets.npz")[2]),
        "dtls_d0": (load_npz("dtls_reasm_packets.npz")[:2], "select=dtls;reassembly", None),
        "quic_q0": (load_npz("quic_reasm_packets.npz")[:2], "select=quic;reassembly", None),
    }
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv pcapw <batch> <config> - (ts 1700000000 unless MERC_TS_FILE)",
                "cases": {}}
    for name, ((arena, desc), config, ts) in cases.items():
        blob = run("pcapw", arena, desc, config, ts)
        recs = pcap_records(blob)
        # the packets that wrote a JSON record (the reference's write_json_linktype
        # would differ for non-Ethernet link types: count with the Ethernet form
        # by forcing linktype 1, as the filter does)
        d1 = desc.copy()
        d1["linktype"] = 1
        lines = run("json", arena, d1, config, ts).split(b"\n")[:-1]
        emitted = sum(1 for l in lines if l)
        with gzip.GzipFile(os.path.join(HERE, f"pcapw_{name}.pcap.gz"), "wb", mtime=0) as f:
            f.write(blob)
        manifest["cases"][name] = {"config": config, "packets": int(len(desc)), "written": len(recs),
                                   "json_records": emitted, "dump_only": len(recs) - emitted,
                                   "timestamps": "MERC_TS_FILE" if ts is not None else 1700000000}
        print(name, manifest["cases"][name])
    with open(os.path.join(HERE, "pcapw_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
