"""Selections that name protocols outside the device path -- "all" (the
reference CLI's default) and a mixed list -- against the REFERENCE (libmerc
2.18.0 built by oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv); run
in the dev container:

    python tests/golden/make_golden_all.py

For a selection C the reference writes records for this path's protocols and
for the others.  The device path must write exactly the reference's records of
its own protocols and nothing for the others -- also where another protocol's
matcher or port claims a packet this path would otherwise have parsed.  The
expected output is therefore, per packet:

    the reference's record under C, when it is the record the reference writes
    under C's own protocols alone (C restricted to this path), else nothing.

Packets: the reference's test pcaps (tests/golden/ref_packets.npz plus the DNS,
mDNS and HTTP capture pcaps), the QUIC, STUN/OpenVPN and tunnel fixtures'
packets, and tests/other_synth.py's crafted packets (every matcher and port
that comes first).

Outputs (committed):
  all_packets.npz            the packets (+ sources)
  all_json_<cfg>.txt.gz      expected write_json text per packet ("" = none)
  all_fp_<cfg>.tsv.gz        expected fp rows: idx emit fp_type truncated fp
  all_manifest.json          configurations, counts (records the reference
                             writes for other protocols, records claimed away)
"""
import gzip
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import other_synth, pcaplib  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

OWN = "tls,dtls,ssh,http,tcp,tcp.syn_ack,quic,stun,openvpn_tcp,gre,vxlan,geneve"
CONFIGS = {
    "all": ("all", OWN),
    "mix": ("tls,http,quic,stun,dtls,dns,rdp,telnet,smtp,socks,ipsec,tftp,vxlan,geneve,openvpn_tcp,mysql",
            "tls,http,quic,stun,dtls,vxlan,geneve,openvpn_tcp"),
    "all_fmt1": ("all;format=tls/1", "select=" + OWN + ";format=tls/1"),
}
EXTRA_PCAPS = ["dns_packet.capture2.pcap", "mdns_capture.pcap", "http_request.capture2.pcap"]


def run(mode, path, cfg):
    return subprocess.run([REF, mode, path, cfg, "-"], capture_output=True, check=True).stdout


def gz(path, data):
    with open(path, "wb") as f:
        f.write(gzip.compress(data, mtime=0))


def main():
    pk, sources = [], []
    z = np.load(os.path.join(HERE, "ref_packets.npz"))
    for i, d in enumerate(z["desc"]):
        off, cl = int(d["offset"]), int(d["caplen"])
        pk.append((int(d["linktype"]), z["arena"][off:off + cl].tobytes()))
        sources.append(str(z["sources"][i]))
    for name in EXTRA_PCAPS:
        for i, p in enumerate(pcaplib.read_pcap(os.path.join("/root/reference/unit_tests/pcaps", name))[:300]):
            pk.append(p)
            sources.append(f"{name}:{i}")
    for fix in ("quic_packets.npz", "tunnel_packets.npz"):
        y = np.load(os.path.join(HERE, fix))
        for i, d in enumerate(y["desc"][:600]):
            off, cl = int(d["offset"]), int(d["caplen"])
            pk.append((int(d["linktype"]), y["arena"][off:off + cl].tobytes()))
            sources.append(f"{fix}:{i}")
    for lab, p in other_synth.scenarios():
        pk.append((1, p))
        sources.append(f"other:{lab}")
    arena, desc = pcaplib.make_batch(pk)
    np.savez_compressed(os.path.join(HERE, "all_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U64"))
    tmp = "/tmp/mfp_all.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {"packets": len(desc)}
    for key, (cfg, own) in CONFIGS.items():
        js_c = run("json", tmp, cfg).split(b"\n")[:len(desc)]
        js_o = run("json", tmp, own).split(b"\n")[:len(desc)]
        fp_c = run("fp", tmp, cfg).split(b"\n")[:len(desc)]
        fp_o = run("fp", tmp, own).split(b"\n")[:len(desc)]
        exp_js, exp_fp = [], []
        other, claimed = 0, 0
        for i in range(len(desc)):
            same = js_c[i] == js_o[i]
            exp_js.append(js_c[i] if same else b"")
            exp_fp.append(fp_c[i] if fp_c[i] == fp_o[i] else f"{i}\t0\t0\t0\t".encode())
            other += bool(js_c[i]) and not same
            claimed += bool(js_o[i]) and not same
        gz(os.path.join(HERE, f"all_json_{key}.txt.gz"), b"\n".join(exp_js) + b"\n")
        gz(os.path.join(HERE, f"all_fp_{key}.tsv.gz"), b"\n".join(exp_fp) + b"\n")
        counts[key] = {"config": cfg, "own": own, "records": sum(bool(x) for x in exp_js),
                       "other_protocol_records": other, "claimed_from_own": claimed}
    os.unlink(tmp)
    json.dump(counts, open(os.path.join(HERE, "all_manifest.json"), "w"), indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
