"""Reference outputs for the GPU parity cases of tests/cases.py (fuzzed
packets, edge cases, kernel-assignment mixes, synthetic batches, the
analysis_context path, the reference's own fuzzing seeds), produced by the
REFERENCE (oracle/_ref/merc_ref_drv, libmerc 2.18.0 compiled from
/root/reference).  Dev container only:

    python tests/golden/make_golden_cases.py

Also copies the reference's fuzzing seeds (test/fuzz/{tls_client_hello,
http_request,http_response}/corpus, data files) into fuzz_corpus.npz.
Outputs (committed): cases/<case>.<mode><fmt>.tsv.gz, cases/manifest.json.
"""
import gzip
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from oracle.compare_ref import REF, ref_config  # noqa: E402
from tests import cases, pcaplib  # noqa: E402


def main():
    os.makedirs(os.path.join(HERE, "cases"), exist_ok=True)
    man = {"reference": "oracle/_ref/merc_ref_drv (libmerc 2.18.0 compiled from /root/reference)", "cases": {}}
    for name, (build, runs) in cases.CASES.items():
        pk = build()
        a, d = pcaplib.make_batch(pk)
        tmp = f"/tmp/golden_case_{name}.mfpb"
        pcaplib.write_mfpb(tmp, a, d)
        for fmt, mode in runs:
            res = cases.META_RESOURCES if mode == "meta" else "-"
            out = subprocess.run([REF, mode, tmp, ref_config(fmt), res], capture_output=True, check=True).stdout
            with gzip.GzipFile(cases.golden_path(name, fmt, mode), "wb", mtime=0) as g:
                g.write(out)
        os.unlink(tmp)
        man["cases"][name] = {"packets": len(pk), "runs": [f"{m}{f}" for f, m in runs],
                              "batch_sha256": hashlib.sha256(a.tobytes() + d.tobytes()).hexdigest()}
        print(name, len(pk))
    json.dump(man, open(os.path.join(HERE, "cases", "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
