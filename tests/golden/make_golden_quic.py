"""QUIC Initial fixtures from the REFERENCE (libmerc 2.18.0 built by
oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv); run in the dev
container:

    python tests/golden/make_golden_quic.py

Outputs (committed):
  quic_packets.npz        packets of the reference's QUIC test pcaps
                          (unit_tests/pcaps/quic*.pcap: at most 150 each, every
                          one the reference emits a fingerprint for first) and
                          the synthetic scenarios of tests/quic_synth.py
  quic_fp_<cfg>.tsv.gz    reference output per packet (write_json path):
                          idx, emit, fp_type, truncated, fingerprint
  quic_manifest.json      configurations, sources, counts
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
from tests import pcaplib, quic_synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

PCAPS = ["quic_init.capture2.pcap", "quic_decry.pcap", "quic_v2.pcap", "quic_ppp.pcap", "quic_reordered_frames.pcap",
         "quic_fragmented.pcap", "quic-crypto-packets.pcap"]
PER_PCAP = 150
# name -> reference packet_filter_cfg
CONFIGS = {
    "q0": "quic",
    "q1": "select=quic;format=quic/1",
    "mix": "select=tls,dtls,ssh,http,tcp,tcp.syn_ack,quic;format=tls/1,quic/1",
}


def ref_fp(path, cfg):
    return subprocess.run([REF, "fp", path, cfg, "-"], capture_output=True, check=True).stdout


def main():
    keep, sources = [], []
    for name in PCAPS:
        fn = os.path.join("/root/reference/unit_tests/pcaps", name)
        pkts = pcaplib.read_pcap(fn)
        out = ref_fp(fn, CONFIGS["q0"]).decode("latin-1").splitlines()
        has_fp = [int(l.split("\t")[2]) != 0 for l in out]
        sel = [i for i in range(len(pkts)) if has_fp[i]][:PER_PCAP]
        sel += [i for i in range(len(pkts)) if not has_fp[i]][:max(0, PER_PCAP - len(sel))]
        for i in sorted(sel):
            keep.append(pkts[i])
            sources.append(f"{name}:{i}")
    for label, p in quic_synth.scenarios():
        keep.append((1, p))
        sources.append(f"synth:{label}")
    arena, desc = pcaplib.make_batch(keep)
    np.savez_compressed(os.path.join(HERE, "quic_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U64"))
    tmp = "/tmp/quic_golden.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {}
    for key, cfg in CONFIGS.items():
        out = ref_fp(tmp, cfg)
        with gzip.open(os.path.join(HERE, f"quic_fp_{key}.tsv.gz"), "wb") as f:
            f.write(out)
        rows = [l.split(b"\t") for l in out.splitlines()]
        counts[key] = {"emit": sum(int(r[1]) for r in rows), "quic_fp": sum(r[2] == b"12" for r in rows),
                       "truncated": sum(int(r[3]) for r in rows)}
    # the whole write_json record text ("tls" and "quic" objects)
    for key in ("q0", "mix"):
        js = subprocess.run([REF, "json", tmp, CONFIGS[key], "-"], capture_output=True,
                            check=True).stdout.decode("latin-1")
        lines = js.split("\n")[:len(desc)]
        with gzip.open(os.path.join(HERE, f"quic_json_{key}.txt.gz"), "wt", encoding="latin-1") as f:
            f.write("\n".join(lines) + "\n")
        counts[key]["json_lines"] = sum(1 for l in lines if l)
        counts[key]["quic_objects"] = sum('"quic":{' in l for l in lines)
    os.unlink(tmp)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp <batch> <config> -", "configs": CONFIGS,
                "packets": len(keep), "pcaps": PCAPS, "per_pcap": PER_PCAP,
                "synthetic": "tests/quic_synth.py scenarios(seed=0x5EED0009, n_random=600)", "counts": counts}
    with open(os.path.join(HERE, "quic_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
