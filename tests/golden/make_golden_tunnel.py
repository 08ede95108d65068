"""Decapsulation fixtures (GRE / VXLAN / Geneve / IP-in-IP, pkt_proc.cc:959-1049)
from the REFERENCE (libmerc 2.18.0 built by oracle/Makefile.ref, driven by
oracle/_ref/merc_ref_drv); run in the dev container:

    python tests/golden/make_golden_tunnel.py

Outputs (committed):
  tunnel_packets.npz        every packet of the reference's tunnel pcaps
                            (unit_tests/pcaps/{gre,vxlan,geneve,ip_encapsulation}.pcap)
                            and the scenarios of tests/tunnel_synth.py
  tunnel_fp_<cfg>.tsv.gz    reference output per packet (write_json path):
                            idx, emit, fp_type, truncated, fingerprint
  tunnel_json_<cfg>.txt.gz  the write_json record text per packet (t0, vx, none)
  tunnel_manifest.json      configurations, sources, counts
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
from tests import pcaplib, tunnel_synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

PCAPS = ["gre.pcap", "vxlan.pcap", "geneve.pcap", "ip_encapsulation.pcap"]
BASE = "tls,dtls,ssh,http,tcp,tcp.syn_ack,quic"
CONFIGS = {
    "t0": f"{BASE},gre,vxlan,geneve",                       # every decapsulation
    "t1": f"select={BASE},gre,vxlan,geneve;format=tls/1",
    "vx": f"{BASE},vxlan",                                   # one tunnel type only
    "none": BASE,                                           # IP-in-IP only (always walked)
}


JSON_KEYS = ["t0", "vx", "none"]


def ref_fp(path, cfg):
    return subprocess.run([REF, "fp", path, cfg, "-"], capture_output=True, check=True).stdout


def main():
    keep, sources = [], []
    for name in PCAPS:
        for i, p in enumerate(pcaplib.read_pcap(os.path.join("/root/reference/unit_tests/pcaps", name))):
            keep.append(p)
            sources.append(f"{name}:{i}")
    for label, p in tunnel_synth.scenarios():
        keep.append((1, p))
        sources.append(f"synth:{label}")
    arena, desc = pcaplib.make_batch(keep)
    np.savez_compressed(os.path.join(HERE, "tunnel_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U64"))
    tmp = "/tmp/tunnel_golden.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {}
    for key, cfg in CONFIGS.items():
        out = ref_fp(tmp, cfg)
        with gzip.open(os.path.join(HERE, f"tunnel_fp_{key}.tsv.gz"), "wb") as f:
            f.write(out)
        rows = [l.split(b"\t") for l in out.splitlines()]
        counts[key] = {"emit": sum(int(r[1]) for r in rows), "fingerprints": sum(r[2] != b"0" for r in rows),
                       "truncated": sum(int(r[3]) for r in rows)}
    # the whole write_json record text (encapsulations arrays, QUIC objects)
    for key in JSON_KEYS:
        js = subprocess.run([REF, "json", tmp, CONFIGS[key], "-"], capture_output=True,
                            check=True).stdout.decode("latin-1")
        lines = js.split("\n")[:len(desc)]
        with gzip.open(os.path.join(HERE, f"tunnel_json_{key}.txt.gz"), "wt", encoding="latin-1") as f:
            f.write("\n".join(lines) + "\n")
        counts[key]["json_lines"] = sum(1 for l in lines if l)
        counts[key]["encapsulations"] = sum('"encapsulations"' in l for l in lines)
    os.unlink(tmp)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp <batch> <config> -", "configs": CONFIGS,
                "packets": len(keep), "pcaps": PCAPS, "synthetic": "tests/tunnel_synth.py scenarios(seed=0x5EED000A)",
                "counts": counts}
    with open(os.path.join(HERE, "tunnel_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
