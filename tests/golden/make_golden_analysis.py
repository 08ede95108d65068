"""Golden vectors for the --analysis classifier, produced by the REFERENCE
(oracle/_ref/merc_ref_drv "an": libmerc get_analysis_context with
do_analysis and a resource archive).  Dev container only:

    python tests/golden/make_golden_analysis.py

Outputs (committed):
  synth_resources.tgz   synthetic archive in the reference's format (tests/synth_db.py)
  resources-test.tgz    the reference's own test archive (test/data/resources-test.tgz, a data file)
  an_synth.tsv.gz       reference results for synth.batch(N_SYNTH, seed=SEED_SYNTH) with synth_resources.tgz
  an_ref.tsv.gz         reference results for ref_packets.npz with resources-test.tgz
  an_survey.tsv.gz      reference results for the same synthetic batch with the SURVEY-sized
                        archive (tests/synth_db.py build_survey(): ~20k fingerprints, P up to
                        256, ~100k pyasn prefixes; regenerated, not committed -- its sha256 is
                        in the manifest)
  an_manifest.json      what produced them (plus a checksum of the regenerated batch)
Columns: idx  valid  fp_type  status  process  score  malware  p_malware
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth, synth_db  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")
SELECT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"
N_SYNTH = 12000
SEED_SYNTH = 0x5EED0003   # same template pool as the synthetic archive


def run_ref(batch_path, resources):
    out = subprocess.run([REF, "an", batch_path, SELECT, resources], capture_output=True, check=True).stdout
    lines = []
    for line in out.decode("latin-1").splitlines():
        f = line.split("\t")
        lines.append("\t".join(f[:8]))
    return "\n".join(lines) + "\n"


def batch_digest(arena, desc):
    h = hashlib.sha256()
    h.update(arena.tobytes())
    h.update(desc.tobytes())
    return h.hexdigest()


def main():
    data, info = synth_db.build()
    with open(os.path.join(HERE, "synth_resources.tgz"), "wb") as f:
        f.write(data)
    shutil.copy("/root/reference/test/data/resources-test.tgz", os.path.join(HERE, "resources-test.tgz"))

    a, d = synth.batch(N_SYNTH, seed=SEED_SYNTH, workload="mixed", n_templates=4096)
    tmp = "/tmp/golden_an.mfpb"
    pcaplib.write_mfpb(tmp, a, d)
    with gzip.open(os.path.join(HERE, "an_synth.tsv.gz"), "wt", encoding="latin-1") as f:
        f.write(run_ref(tmp, os.path.join(HERE, "synth_resources.tgz")))

    survey = synth_db.build_survey()
    with gzip.open(os.path.join(HERE, "an_survey.tsv.gz"), "wt", encoding="latin-1") as f:
        f.write(run_ref(tmp, survey))

    z = np.load(os.path.join(HERE, "ref_packets.npz"))
    pcaplib.write_mfpb(tmp, z["arena"], z["desc"])
    with gzip.open(os.path.join(HERE, "an_ref.tsv.gz"), "wt", encoding="latin-1") as f:
        f.write(run_ref(tmp, os.path.join(HERE, "resources-test.tgz")))
    os.unlink(tmp)

    manifest = {
        "reference": "cisco/mercury 2.18.0 libmerc (oracle/Makefile.ref), merc_ref_drv an <batch> <select> <resources>",
        "select": SELECT,
        "synth": {"n": N_SYNTH, "seed": SEED_SYNTH, "workload": "mixed", "n_templates": 4096,
                  "sha256": batch_digest(a, d), "db": info},
        "ref": {"packets": "ref_packets.npz", "resources": "resources-test.tgz (test/data of the reference)"},
        "survey": {"archive": "tests/golden/_gen/survey_resources.tgz (tests/synth_db.py build_survey)",
                   "params": {k: v for k, v in synth_db.SURVEY.items()},
                   "tar_sha256": hashlib.sha256(gzip.decompress(open(survey, "rb").read())).hexdigest()},
        "columns": ["idx", "valid", "fp_type", "status", "process", "score", "malware", "p_malware"],
    }
    with open(os.path.join(HERE, "an_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(manifest["synth"])


if __name__ == "__main__":
    main()
