"""Golden output of the REFERENCE for bench.py's timed workload (config 4), so
the benchmark checks the records it times (bench.py `check_step_output`,
`check_diverse_statuses`).  Dev container only (needs oracle/_ref and the
SURVEY-sized archive, tests/synth_db.py build_survey):

    python tests/golden/make_golden_bench.py

bench.py's device batch is its rank's 1 000 000 unique packets
(synth.batch(1M, seed=0x5EED0003, workload="mixed", n_templates=4096,
draw_seed=0x5EED0004) on rank 0) tiled to 50 M.  The reference (oracle/_ref,
merc_ref_drv, write_json path with the classifier) runs:

* bench_sample.npz: the unique packets twice in a row (MERC_TILE=0:2M,
  "wjan" mode) and reports the SECOND period's records at 24 000 seeded
  indices: emit flag, fingerprint type and string, analysis validity, status,
  process, score, malware, p_malware.  The timed steps come after warm-up
  steps over the same packets, so every unknown-TLS fingerprint has been seen
  before -- exactly the second period's state (the period has far fewer
  distinct unknown fingerprints than the LRU's 100 000 entries, so nothing is
  evicted and membership alone decides the status).
* bench_diverse_status.bin.gz: the unique packets once, then the diversity
  leg's first step -- the diverse unique set (the same draw with
  diverse_tls=1.0) tiled to 50 M ("stat" mode) -- one bit per unknown-TLS
  sighting of that step (1 = unlabeled, 0 = randomized), in stream order:
  17.5 M decisions of the 100 000-entry LRU, evictions included.  After the
  main leg's steps the LRU holds the main set's unknown fingerprints in the
  order of their last sighting in one period, the state the single first
  period leaves.
* bench_manifest.json: the parameters and counts.
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth, synth_db  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

U = 1_000_000
N = 50_000_000
SEED, DRAW = 0x5EED0003, 0x5EED0003 + 1
SAMPLE_SEED = 0x5EED0B1C
N_SAMPLE = 24_000
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"


def unique(diverse=0.0):
    return synth.batch(U, seed=SEED, workload="mixed", n_templates=4096, draw_seed=DRAW, diverse_tls=diverse)


def run(mode, arena, desc, cfg, res, env):
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        p = os.path.join(d, "b.mfpb")
        pcaplib.write_mfpb(p, arena, desc)
        e = dict(os.environ)
        for k, v in env.items():
            if isinstance(v, np.ndarray):
                f = os.path.join(d, k + ".bin")
                v.astype("<u8").tofile(f)
                v = f
            e[k] = str(v)
        r = subprocess.run([REF, mode, p, cfg, res], capture_output=True, check=True, env=e)
        return r.stdout, r.stderr.decode("latin-1")


def main():
    res = synth_db.build_survey()
    cfg = CONTRACT          # a bare list: resources come as the driver's own argument
    t0 = time.time()
    ua, ud = unique()
    rng = np.random.default_rng(SAMPLE_SEED)
    rows = np.sort(rng.choice(U, N_SAMPLE, replace=False)).astype(np.uint64)
    out, _ = run("wjan", ua, ud, cfg, res, {"MERC_TILE": f"0:{2 * U}", "MERC_ROWS_FILE": rows + np.uint64(U)})
    lines = out.decode("latin-1").split("\n")[:-1]
    assert len(lines) == N_SAMPLE, len(lines)
    fps, fp_idx, procs, proc_idx = {}, [], {}, []
    cols = {k: [] for k in ("emit", "fp_type", "valid", "status", "malware")}
    score, pmal = [], []
    for ln, r in zip(lines, rows):
        p = ln.split("\t")
        assert int(p[0]) == int(r) + U
        for k, j in (("emit", 1), ("fp_type", 2), ("valid", 3), ("status", 4), ("malware", 7)):
            cols[k].append(int(p[j]))
        proc_idx.append(procs.setdefault(p[5], len(procs)))
        score.append(float(p[6]))
        pmal.append(float(p[8]))
        fp_idx.append(fps.setdefault(p[9] if len(p) > 9 else "", len(fps)))
    fp_list = sorted(fps, key=fps.get)
    blob = "".join(fp_list).encode("latin-1")
    ends = np.cumsum([len(s.encode("latin-1")) for s in fp_list]).astype(np.uint64)
    names = "\n".join(sorted(procs, key=procs.get)).encode()
    np.savez_compressed(os.path.join(HERE, "bench_sample.npz"), rows=rows,
                        **{k: np.array(v, np.uint8) for k, v in cols.items()},
                        score=np.array(score), p_malware=np.array(pmal),
                        fp_idx=np.array(fp_idx, np.uint32), fp_blob=np.frombuffer(blob, np.uint8), fp_ends=ends,
                        proc_idx=np.array(proc_idx, np.uint32), proc_names=np.frombuffer(names, np.uint8))
    t1 = time.time()
    print(f"sample: {N_SAMPLE} rows, {len(fp_list)} distinct fingerprints, {len(procs)} processes ({t1 - t0:.0f} s)")

    da, dd = unique(diverse=1.0)
    arena = np.concatenate([ua, da])
    d2 = dd.copy()
    d2["offset"] += np.uint64(len(ua))
    desc = np.concatenate([ud, d2])
    del ua, da
    bits, err = run("stat", arena, desc, cfg, res, {"MERC_TILE": f"{U}:{U + N}"})
    sightings = int(err.split("sightings ")[-1].split()[0])
    assert (sightings + 7) // 8 == len(bits)
    with gzip.GzipFile(os.path.join(HERE, "bench_diverse_status.bin.gz"), "wb", mtime=0) as f:
        f.write(bits)
    t2 = time.time()
    unl = int(np.unpackbits(np.frombuffer(bits, np.uint8)).sum())
    manifest = {
        "reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
        "driver": "oracle/_ref/merc_ref_drv wjan|stat (MERC_TILE, MERC_ROWS_FILE), write_json path + classifier",
        "unique": U, "packets": N, "seed": SEED, "draw_seed": DRAW, "n_templates": 4096, "workload": "mixed",
        "config": "select=" + cfg + ";resources=<synth_db.build_survey()>;analysis", "sample_seed": SAMPLE_SEED,
        "sample_rows": N_SAMPLE, "sample_distinct_fingerprints": len(fp_list),
        "diverse_tls": 1.0, "diverse_bytes": len(bits), "diverse_sightings": sightings,
        "diverse_unlabeled_bits": unl,
        "seconds": {"sample": round(t1 - t0, 1), "diverse": round(t2 - t1, 1)},
    }
    with open(os.path.join(HERE, "bench_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(manifest)


if __name__ == "__main__":
    main()
