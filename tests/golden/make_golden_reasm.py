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
  reasm_an_r0.tsv.gz       the analysis_context path ("anr": valid, type,
                           status, process, score, malware, p_malware,
                           more_pkts_needed, fingerprint) with config AN_CONFIG
                           and the reference's test archive
  reasm_timed_packets.npz  a second stream with per-packet capture times
                           (tests/reasm_synth.py timed_scenarios), run by its
                           own processor: reasm_timed_fp.tsv.gz,
                           reasm_timed_props.txt.gz, reasm_timed_json.txt.gz
                           (config r0) and reasm_timed_an.tsv.gz ("anr")
  reasm_tunnel_packets.npz ClientHellos split inside tunnels
                           (reasm_synth.tunnel_scenarios); their JSON text
                           with TUNNEL_CONFIG: reasm_tunnel_json.txt.gz
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
AN_CONFIG = "select=tls,ssh,http;reassembly"
TUNNEL_CONFIG = "select=tls,ssh,http,gre,vxlan,geneve;reassembly"
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
    an = subprocess.run([REF, "anr", tmp, AN_CONFIG, res], capture_output=True, check=True).stdout
    with gzip.open(os.path.join(HERE, "reasm_an_r0.tsv.gz"), "wb") as f:
        f.write(an)
    rows = [l.split(b"\t") for l in an.splitlines()]
    counts["an_path"] = {"valid": sum(int(r[1]) for r in rows), "more": sum(int(r[8]) for r in rows)}
    os.unlink(tmp)
    # the timed stream
    timed = reasm_synth.timed_scenarios()
    arena_t, desc_t = pcaplib.make_batch([(1, p) for _, p, _ in timed])
    ts = np.array([t for _, _, t in timed], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "reasm_timed_packets.npz"), arena=arena_t, desc=desc_t, ts=ts,
                        sources=np.array([lab for lab, _, _ in timed], dtype="U48"))
    pcaplib.write_mfpb(tmp, arena_t, desc_t)
    tsf = "/tmp/reasm_timed.ts"
    ts.astype("<u8").tofile(tsf)
    env = dict(os.environ, MERC_TS_FILE=tsf)
    out = subprocess.run([REF, "fp", tmp, CONFIGS["r0"], "-"], capture_output=True, check=True, env=env).stdout
    with gzip.open(os.path.join(HERE, "reasm_timed_fp.tsv.gz"), "wb") as f:
        f.write(out)
    js = subprocess.run([REF, "json", tmp, CONFIGS["r0"], "-"], capture_output=True, check=True,
                        env=env).stdout.decode("latin-1")
    lines = js.split("\n")[:len(desc_t)]
    props = [(PROPS.search(l).group(1) if PROPS.search(l) else "") for l in lines]
    with gzip.open(os.path.join(HERE, "reasm_timed_props.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(props) + "\n")
    with gzip.open(os.path.join(HERE, "reasm_timed_json.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(lines) + "\n")
    an = subprocess.run([REF, "anr", tmp, AN_CONFIG, res], capture_output=True, check=True, env=env).stdout
    with gzip.open(os.path.join(HERE, "reasm_timed_an.tsv.gz"), "wb") as f:
        f.write(an)
    rows = [l.split(b"\t") for l in an.splitlines()]
    counts["timed"] = {"packets": len(desc_t), "reassembled": sum('"reassembled":true' in p for p in props),
                       "timeout": sum("timeout" in p for p in props),
                       "an_valid": sum(int(r[1]) for r in rows), "an_more": sum(int(r[8]) for r in rows)}
    # tunnelled split ClientHellos (the reassembled record keeps its "encapsulations")
    tun = reasm_synth.tunnel_scenarios()
    arena_u, desc_u = pcaplib.make_batch([(1, p) for _, p in tun])
    np.savez_compressed(os.path.join(HERE, "reasm_tunnel_packets.npz"), arena=arena_u, desc=desc_u,
                        sources=np.array([lab for lab, _ in tun], dtype="U48"))
    pcaplib.write_mfpb(tmp, arena_u, desc_u)
    js = subprocess.run([REF, "json", tmp, TUNNEL_CONFIG, "-"], capture_output=True,
                        check=True).stdout.decode("latin-1")
    lines = js.split("\n")[:len(desc_u)]
    with gzip.open(os.path.join(HERE, "reasm_tunnel_json.txt.gz"), "wt", encoding="latin-1") as f:
        f.write("\n".join(lines) + "\n")
    counts["tunnel"] = {"packets": len(desc_u), "reassembled": sum('"reassembled":true' in l for l in lines),
                        "encapsulated": sum('"encapsulations"' in l for l in lines)}
    os.unlink(tmp)
    os.unlink(tsf)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp|json <stream> <config> - (fixed ts 1700000000)",
                "configs": CONFIGS, "an_config": AN_CONFIG, "tunnel_config": TUNNEL_CONFIG, "packets": len(desc), "pcap_packets": len(pk), "synthetic": len(syn),
                "synthetic_source": "tests/reasm_synth.py scenarios(seed=0x5EED000F)",
                "timed_source": "tests/reasm_synth.py timed_scenarios(seed=0x5EED0010), MERC_TS_FILE", "counts": counts}
    with open(os.path.join(HERE, "reasm_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
