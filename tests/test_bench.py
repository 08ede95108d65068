"""bench.py's launch contract on the CPU: `python bench.py --gpus N` starts N
rank processes itself (torch.distributed.run environment, gloo control group)
before anything touches the GPU, and the per-kernel byte accounting."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))



@pytest.mark.parametrize("world", [2, 8])
def test_bench_spawns_ranks_dry_run(world):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["dry_run"] and line["n_gpus"] == world and line["backend"] == "gloo"
    assert sorted(r["rank"] for r in line["ranks"]) == list(range(world))
    assert sorted(r["local_rank"] for r in line["ranks"]) == list(range(world))
    assert len({r["pid"] for r in line["ranks"]}) == world


def test_bench_under_launcher_env_uses_world_size():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                         capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["n_gpus"] == 1   # a launcher's WORLD_SIZE wins


def test_kernel_bytes_accounting():
    sys.path.insert(0, ROOT)
    import bench
    from mercury_amd.api import ANALYSIS_DTYPE, DESC_DTYPE, RECORD_DTYPE
    rec = np.zeros(3, RECORD_DTYPE)
    desc = np.zeros(3, DESC_DTYPE)
    desc["caplen"] = [600, 200, 60]
    rec["msg"] = [1, 6, 8]            # TLS CH, HTTP request, SYN
    rec["fp_len"] = [300, 100, 40]
    rec["flags"] = [0, 4, 0]
    rec["sni_len"] = [20, 0xffff, 0xffff]
    rec["ua_len"] = 0xffff
    an = np.zeros(3, ANALYSIS_DTYPE)
    an["flags"] = [1, 0, 0]
    an["process"] = [7, 0xFFFFFFFF, 0xFFFFFFFF]
    st = {"work_items": 1, "lane_scored": 1, "feature_slots": 5, "lane_priors": 4, "lane_updates": 10,
          "pending": 0, "deferred": 0, "seen_merges": 0}
    tb = {}
    kb = bench.kernel_bytes(rec, desc, an, an_stats=st, tables=tb)
    assert kb["k_fp_tls1/tls_ch"] == 4 + 16 + 600 + 32 + 300
    assert kb["k_fp_seg/http_req"] == 4 + 16 + 200 + 32 + 100 + 8
    assert kb["k_fingerprint/tcp_syn"] == 4 + 16 + 60 + 32 + 40
    assert kb["k_classify"] == 3 * (16 + 5) + 128 + 128 + 60
    assert kb["k_analyze"] == 3 * (32 + 32) + (8 + 300) + 16 + 8   # record + 32-B analysis record
    assert kb["k_an_features"] == (16 + 32 + 16 + 40) + 20 + 64
    assert kb["k_an_score"] == 64 + 32 + 32
    assert kb["k_seen_scan"] == 8
    # the archive's tables: the verified strings' pool copies, feature slots, priors and update lists
    assert tb == {"k_analyze": 300, "k_an_features": 20 + 32 * 5, "k_an_score": 8 * 4 + 12 * 10, "k_analyze_wave": 0}


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _sample_records():
    """Records, analysis results and a fingerprint arena that reproduce the
    reference golden of bench_sample.npz at the positions check_step_output
    samples (the CPU stand-in for the device outputs)."""
    import torch
    from mercury_amd.api import ANALYSIS_DTYPE, RECORD_DTYPE
    b = _bench()
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "bench_sample.npz")))
    m = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_manifest.json")))
    u, n = m["unique"], m["packets"]
    rows = g["rows"].astype(np.int64)
    k = np.random.default_rng(0x5EED0B1D).integers(0, n // u, len(rows))
    idx = rows + k * u
    ends = np.concatenate([[0], g["fp_ends"].astype(np.int64)])
    blob = g["fp_blob"].tobytes()
    names = g["proc_names"].tobytes().decode().split("\n")
    # a small "step": only the sampled positions are filled (the checker reads only them)
    rec = np.zeros(int(idx.max()) + 1, RECORD_DTYPE)
    an = np.zeros(len(rec), ANALYSIS_DTYPE)
    fp = bytearray()
    ids = {name: i for i, name in enumerate(names)}

    class Ctx:
        def process_name(self, pid):
            return "" if pid == 0xFFFFFFFF else names[pid]
    for j, i in enumerate(idx):
        fi = int(g["fp_idx"][j])
        s = blob[ends[fi]:ends[fi + 1]]
        rec[i]["fp_offset"], rec[i]["fp_len"] = len(fp), len(s)
        fp += s
        rec[i]["fp_type"] = g["fp_type"][j]
        rec[i]["flags"] = g["emit"][j]
        if g["valid"][j]:
            nm = names[int(g["proc_idx"][j])]
            an[i]["flags"] = 1 | (2 * int(g["malware"][j])) | 4
            an[i]["status"] = g["status"][j]
            an[i]["process"] = ids[nm] if nm else 0xFFFFFFFF
            an[i]["score"] = g["score"][j]
            an[i]["malware_prob"] = g["p_malware"][j]
    return b, Ctx(), rec, an, torch.frombuffer(bytes(fp) + b"\0", dtype=torch.uint8), n, u, idx


def test_bench_output_check_accepts_reference_and_catches_a_byte():
    """check_step_output: the golden's own records pass; one flipped
    fingerprint byte, status or score fails the line."""
    import torch
    b, ctx, rec, an, d_fp, n, u, idx = _sample_records()
    r = b.check_step_output(torch, ctx, rec, an, d_fp, n, u)
    assert r["ok"] and r["records_checked"] == 24000 and r["classified_checked"] > 1000, r
    fp2 = d_fp.clone()
    j = int(np.flatnonzero(rec["fp_len"][idx] > 0)[0])
    fp2[int(rec["fp_offset"][idx[j]])] ^= 1
    assert not b.check_step_output(torch, ctx, rec, an, fp2, n, u)["ok"]
    v = int(idx[np.flatnonzero(an["flags"][idx] & 1)[0]])
    an2 = an.copy()
    an2["score"][v] += 1e-5
    assert not b.check_step_output(torch, ctx, rec, an2, d_fp, n, u)["ok"]
    an3 = an.copy()
    an3["status"][v] ^= 1
    assert not b.check_step_output(torch, ctx, rec, an3, d_fp, n, u)["ok"]


def test_bench_diverse_check():
    """check_diverse_statuses over the reference's 17.5 M decisions: the same
    bits pass, one flipped decision fails."""
    import gzip
    from mercury_amd.api import ANALYSIS_DTYPE
    b = _bench()
    m = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_manifest.json")))
    with gzip.open(os.path.join(ROOT, "tests", "golden", "bench_diverse_status.bin.gz"), "rb") as f:
        bits = np.unpackbits(np.frombuffer(f.read(), np.uint8))[:m["diverse_sightings"]]
    assert m["diverse_sightings"] > 10_000_000 and 0 < bits.sum() < len(bits)
    an = np.zeros(len(bits) + 7, ANALYSIS_DTYPE)      # a few packets that are not sightings
    an["flags"][:len(bits)] = 1
    an["status"][:len(bits)] = np.where(bits == 1, 3, 2)
    an["flags"][len(bits):] = 1
    an["status"][len(bits):] = 1                       # labeled
    assert b.check_diverse_statuses(an)["ok"]
    an["status"][12345] ^= 1                            # 2 <-> 3
    r = b.check_diverse_statuses(an)
    assert not r["ok"] and r["first_mismatch"] == 12345


def test_bench_golden_applies_only_to_the_default_batch():
    b = _bench()
    m = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_manifest.json")))
    assert b.golden_applies(m["packets"], m["unique"], "mixed", True, "survey", m["draw_seed"])
    assert not b.golden_applies(m["packets"], m["unique"], "mixed", True, "survey", m["draw_seed"] + 7919)   # rank 1
    assert not b.golden_applies(10_000_000, m["unique"], "mixed", True, "survey", m["draw_seed"])
    assert not b.golden_applies(m["packets"], m["unique"], "mixed", False, "survey", m["draw_seed"])
