"""TCP reassembly fixtures from the REFERENCE (libmerc 2.18.0 built by
oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv) with "reassembly"
in the configuration; run in the dev container:

    python tests/golden/make_golden_reasm.py

One packet stream, processed in order by one reference processor (so flow
state carries from packet to packet): every packet of the reference pcaps of
ref_packets.npz (65 unit-test pcaps), then the synthetic streams of
tests/reasm_synth.py.

Outputs (committed):
  reasm_packets.npz        the synthetic packets (the pcap packets come from
                           ref_packets.npz)
  reasm_fp_<cfg>.tsv.gz    write_json path per packet: idx, emit, fp_type,
                           truncated, fingerprint
  reasm_props_<cfg>.txt.gz the record's "reassembly_properties" object text
                           per packet ("" when none)
  reasm_json_<cfg>.txt.gz  the record's whole JSON line per packet
  reasm_manifest.json      configurations, counts
"""
import gzip
import json
import os
import re
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, reasm_synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

CONFIGS = {
    "r0": "select=tls,ssh,http,tcp,tcp.syn_ack;reassembly",
    "r1": "select=tls,ssh,http;format=tls/1;reassembly",
}
PROPS = re.compile(r'"reassembly_properties":(\{[^}]*\})')


def stream():
    z = np.load(os.path.join(HERE, "ref_packets.npz"))
    pk = [(int(d["linktype"]), bytes(z["arena"][int(d["offset"]):int(d["offset"]) + int(d["caplen"])]))
          for d in z["desc"]]
    syn = reasm_synth.scenarios()
    return pk, syn


def main():
    pk, syn = stream()
    arena_s, desc_s = pcaplib.make_batch([(1, p) for _, p in syn])
    np.savez_compressed(os.path.join(HERE, "reasm_packets.npz"), arena=arena_s, desc=desc_s,
                        sources=np.array([lab for lab, _ in syn], dtype="U48"))
    arena, desc = pcaplib.make_batch(pk + [(1, p) for _, p in syn])
    tmp = "/tmp/reasm_golden.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {}
    for key, cfg in CONFIGS.items():
        out = subprocess.run([REF, "fp", tmp, cfg, "-"], capture_output=True, check=True).stdout
        with gzip.open(os.path.join(HERE, f"reasm_fp_{key}.tsv.gz"), "wb") as f:
            f.write(out)
        js = subprocess.run([REF, "json", tmp, cfg, "-"], capture_output=True, check=True).stdout.decode("latin-1")
        lines = js.split("\n")[:len(desc)]
        props = []
        for l in lines:
            m = PROPS.search(l)
            props.append(m.group(1) if m else "")
        with gzip.open(os.path.join(HERE, f"reasm_props_{key}.txt.gz"), "wt", encoding="latin-1") as f:
            f.write("\n".join(props) + "\n")
        with gzip.open(os.path.join(HERE, f"reasm_json_{key}.txt.gz"), "wt", encoding="latin-1") as f:
            f.write("\n".join(lines) + "\n")
        rows = [l.split(b"\t") for l in out.splitlines()]
        counts[key] = {"emit": sum(int(r[1]) for r in rows), "fp": sum(r[2] != b"0" for r in rows),
                       "reassembled": sum('"reassembled":true' in p for p in props),
                       "truncated": sum(int(r[3]) for r in rows),
                       "overlaps": sum("overlap" in p for p in props)}
    # with --analysis (the reference's test archive): the whole JSON text
    res = os.path.join(HERE, "resources-test.tgz")
    js = subprocess.run([REF, "json", tmp, CONFIGS["r0"], res], capture_output=True, check=True).stdout.decode("latin-1")
    with gzip.open(os.path.join(HERE, "reasm_json_an.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(js.split("\n")[:len(desc)]) + "\n")
    counts["an"] = {"analysis_objects": js.count('"analysis":')}
    os.unlink(tmp)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp|json <stream> <config> - (fixed ts 1700000000)",
                "configs": CONFIGS, "packets": len(desc), "pcap_packets": len(pk), "synthetic": len(syn),
                "synthetic_source": "tests/reasm_synth.py scenarios(seed=0x5EED000F)", "counts": counts}
    with open(os.path.join(HERE, "reasm_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
