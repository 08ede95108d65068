"""QUIC CRYPTO-frame reassembly fixtures from the REFERENCE (libmerc 2.18.0
built by oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv) with
"reassembly" in the configuration; run in the dev container:

    python tests/golden/make_golden_quic_reasm.py

One packet stream, processed in order by one reference processor: the
reference's multi-datagram QUIC pcaps (unit_tests/pcaps/quic_fragmented,
quic_reordered_frames, quic-crypto-packets, quic_init.capture2), then the
synthetic streams of tests/quic_reasm_synth.py (scenarios, then stale_scenarios).

Outputs (committed):
  quic_reasm_packets.npz       the whole stream (pcap + synthetic packets)
  quic_reasm_fp_<cfg>.tsv.gz   write_json path per packet: idx, emit, fp_type,
                               truncated, fingerprint
  quic_reasm_json_<cfg>.txt.gz the record's JSON line per packet ("" = none)
  quic_reasm_an.tsv.gz         the analysis_context path ("anr") with
                               more_pkts_needed, config AN_CONFIG
  quic_reasm_timed_*.gz        a timed stream (quic_reasm_synth.timed_scenarios)
  quic_reasm_manifest.json     configurations, counts
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
from tests import pcaplib, quic_reasm_synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

PCAPS = ["quic_fragmented.pcap", "quic_reordered_frames.pcap", "quic-crypto-packets.pcap", "quic_init.capture2.pcap"]
PER_PCAP = 200
CONFIGS = {"q0": "select=quic;reassembly", "q1": "select=quic,tls;format=quic/1;reassembly"}
AN_CONFIG = "select=quic;reassembly"


def run(mode, path, cfg, res="-", env=None):
    return subprocess.run([REF, mode, path, cfg, res], capture_output=True, check=True, env=env).stdout


def main():
    pk = []
    for name in PCAPS:
        pk += pcaplib.read_pcap(os.path.join("/root/reference/unit_tests/pcaps", name))[:PER_PCAP]
    syn = quic_reasm_synth.scenarios() + quic_reasm_synth.stale_scenarios()
    pkts = pk + [(1, p) for _, p in syn]
    arena, desc = pcaplib.make_batch(pkts)
    sources = [f"pcap.{i}" for i in range(len(pk))] + [lab for lab, _ in syn]
    np.savez_compressed(os.path.join(HERE, "quic_reasm_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U48"))
    tmp = "/tmp/quic_reasm.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {"packets": len(desc), "pcap_packets": len(pk)}
    for key, cfg in CONFIGS.items():
        out = run("fp", tmp, cfg)
        with gzip.open(os.path.join(HERE, f"quic_reasm_fp_{key}.tsv.gz"), "wb") as f:
            f.write(out)
        lines = run("json", tmp, cfg).decode("latin-1").split("\n")[:len(desc)]
        with gzip.open(os.path.join(HERE, f"quic_reasm_json_{key}.txt.gz"), "wt", encoding="latin-1") as f:
            f.write("\n".join(lines) + "\n")
        rows = [l.split(b"\t") for l in out.splitlines()]
        counts[key] = {"emit": sum(int(r[1]) for r in rows), "fp": sum(r[2] != b"0" for r in rows),
                       "reassembled": sum('"reassembled":true' in l for l in lines),
                       "truncated_flows": sum('"reassembled":true' in l and '"truncated"' in l for l in lines)}
    res = os.path.join(HERE, "quic_resources.tgz")
    an = run("anr", tmp, AN_CONFIG, res)
    with gzip.open(os.path.join(HERE, "quic_reasm_an.tsv.gz"), "wb") as f:
        f.write(an)
    rows = [l.split(b"\t") for l in an.splitlines()]
    counts["an_path"] = {"valid": sum(int(r[1]) for r in rows), "more": sum(int(r[8]) for r in rows)}
    # the timed stream
    timed = quic_reasm_synth.timed_scenarios()
    arena_t, desc_t = pcaplib.make_batch([(1, p) for _, p, _ in timed])
    ts = np.array([t for _, _, t in timed], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "quic_reasm_timed_packets.npz"), arena=arena_t, desc=desc_t, ts=ts,
                        sources=np.array([lab for lab, _, _ in timed], dtype="U48"))
    pcaplib.write_mfpb(tmp, arena_t, desc_t)
    tsf = "/tmp/quic_reasm_timed.ts"
    ts.astype("<u8").tofile(tsf)
    env = dict(os.environ, MERC_TS_FILE=tsf)
    lines = run("json", tmp, CONFIGS["q0"], env=env).decode("latin-1").split("\n")[:len(desc_t)]
    with gzip.open(os.path.join(HERE, "quic_reasm_timed_json.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(lines) + "\n")
    counts["timed"] = {"packets": len(desc_t), "reassembled": sum('"reassembled":true' in l for l in lines),
                       "timeout": sum('"timeout":true' in l for l in lines)}
    os.unlink(tmp)
    os.unlink(tsf)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp|json|anr <stream> <config> (fixed ts 1700000000)",
                "pcaps": PCAPS, "per_pcap": PER_PCAP, "configs": CONFIGS, "an_config": AN_CONFIG,
                "synthetic_source": "tests/quic_reasm_synth.py scenarios(seed=0x5EED0016), "
                                    "timed_scenarios(seed=0x5EED0017), MERC_TS_FILE",
                "counts": counts}
    with open(os.path.join(HERE, "quic_reasm_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
