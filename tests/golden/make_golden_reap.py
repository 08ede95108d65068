"""Reassembly reaping-order fixtures from the REFERENCE (libmerc 2.18.0 built
by oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv, "reassembly"
configured, per-packet capture times through MERC_TS_FILE); run in the dev
container:

    python tests/golden/make_golden_reap.py

The stream (tests/reasm_synth.py reap_scenarios) fills the flow table past
its 10 000 entries so that every new flow makes active_reap drop two flows
from the persistent iterator, completes the survivors (which keep reaping),
then stalls 64 flows past the 15 s timeout and lets passive_reap walk them
while new flows arrive: which flows survive to complete depends only on the
table's iteration order (reassembly.hpp:596-655, std::hash<key>
flow_key.h:257-317).

Outputs (committed):
  reap_packets.npz       the stream, with per-packet capture times (seconds)
  reap_fp.tsv.gz         write_json path per packet: idx, emit, fp_type,
                         truncated, fingerprint (config CONFIG)
  reap_props.txt.gz      the record's "reassembly_properties" object per packet
  reap_manifest.json     configuration, counts
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

CONFIG = "select=tls;reassembly"
PROPS = re.compile(r'"reassembly_properties":(\{[^}]*\})')


def main():
    items = reasm_synth.reap_scenarios()
    arena, desc = pcaplib.make_batch([(1, p) for _, p, _ in items])
    ts = np.array([t for _, _, t in items], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "reap_packets.npz"), arena=arena, desc=desc, ts=ts,
                        phase=np.array([lab for lab, _, _ in items], dtype="U8"))
    tmp, tsf = "/tmp/reap.mfpb", "/tmp/reap.ts"
    pcaplib.write_mfpb(tmp, arena, desc)
    ts.astype("<u8").tofile(tsf)
    env = dict(os.environ, MERC_TS_FILE=tsf)
    out = subprocess.run([REF, "fp", tmp, CONFIG, "-"], capture_output=True, check=True, env=env).stdout
    with gzip.open(os.path.join(HERE, "reap_fp.tsv.gz"), "wb") as f:
        f.write(out)
    js = subprocess.run([REF, "json", tmp, CONFIG, "-"], capture_output=True, check=True, env=env).stdout
    lines = js.decode("latin-1").split("\n")[:len(desc)]
    props = [(m.group(1) if m else "") for m in (PROPS.search(l) for l in lines)]
    with gzip.open(os.path.join(HERE, "reap_props.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(props) + "\n")
    os.unlink(tmp)
    os.unlink(tsf)
    rows = [l.split(b"\t") for l in out.splitlines()]
    phases = [lab for lab, _, _ in items]
    counts = {"packets": len(desc), "emit": sum(int(r[1]) for r in rows),
              "reassembled": sum('"reassembled":true' in p for p in props),
              "timeout": sum('"timeout":true' in p for p in props)}
    for ph in sorted(set(phases)):
        counts[ph] = sum('"reassembled":true' in p for p, q in zip(props, phases) if q == ph)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp|json <stream> <config> with MERC_TS_FILE",
                "config": CONFIG, "synthetic_source": "tests/reasm_synth.py reap_scenarios(seed=0x5EED0018)",
                "counts": counts}
    with open(os.path.join(HERE, "reap_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
