"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the dev container (needs /root/reference and oracle/_ref built by
oracle/Makefile.ref):

    python tests/golden/make_golden.py

Outputs (committed):
  ref_packets.npz        packets taken from the reference's own test pcaps
                         (unit_tests/pcaps/*.pcap, test/data/*.pcap): all
                         packets of the small captures, and for the large ones
                         every packet the reference emits a record for plus
                         every 10th other packet
  ref_fp_fmt{0,1,2}.tsv.gz  reference output per packet (write_json path):
                         idx, emit, fp_type, truncated, fingerprint
  manifest.json          what produced them
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
from tests import pcaplib  # noqa: E402
from oracle.compare_ref import REF, ref_config  # noqa: E402

REFDIR = "/root/reference"
SKIP = {"dns_packet.capture2.pcap", "http_request.capture2.pcap", "mdns_capture.pcap",
        "quic-crypto-packets.pcap"}
BIG = 20000  # bytes: captures above this are subsampled


def main():
    files = sorted(os.path.join(REFDIR, "unit_tests/pcaps", f) for f in os.listdir(os.path.join(REFDIR, "unit_tests/pcaps")))
    # test/data/top_100_fingerprints.pcap is byte-identical to the unit_tests copy
    files += [os.path.join(REFDIR, "test/data", f) for f in ("new-stats-telemetry-test.pcap", "test_decrypt.pcap")]
    keep = []
    sources = []
    for fn in files:
        base = os.path.basename(fn)
        if base in SKIP or not fn.endswith(".pcap"):
            continue
        pkts = pcaplib.read_pcap(fn)
        if os.path.getsize(fn) > BIG:
            out = subprocess.run([REF, "fp", fn, ref_config(0), "-"], capture_output=True, check=True).stdout
            emit = [int(l.split(b"\t")[1]) for l in out.splitlines()]
            sel = [i for i in range(len(pkts)) if emit[i] or i % 10 == 0]
        else:
            sel = list(range(len(pkts)))
        for i in sel:
            keep.append(pkts[i])
            sources.append(f"{base}:{i}")
    arena, desc = pcaplib.make_batch(keep)
    np.savez_compressed(os.path.join(HERE, "ref_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U64"))
    tmp = os.path.join("/tmp", "golden.mfpb")
    pcaplib.write_mfpb(tmp, arena, desc)
    for fmt in (0, 1, 2):
        out = subprocess.run([REF, "fp", tmp, ref_config(fmt), "-"], capture_output=True, check=True).stdout
        with gzip.open(os.path.join(HERE, f"ref_fp_fmt{fmt}.tsv.gz"), "wb") as f:
            f.write(out)
    os.unlink(tmp)
    manifest = {
        "reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
        "driver": "oracle/_ref/merc_ref_drv fp <batch> <config> -",
        "configs": {str(f): ref_config(f) for f in (0, 1, 2)},
        "packets": len(keep),
        "pcaps": sorted({s.split(":")[0] for s in sources}),
    }
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(keep)} packets, arena {len(arena)} bytes")


if __name__ == "__main__":
    main()
