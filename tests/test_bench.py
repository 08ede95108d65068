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
    kb = bench.kernel_bytes(rec, desc, an, an_stats=st)
    assert kb["k_fp_tls1/tls_ch"] == 4 + 16 + 600 + 32 + 300
    assert kb["k_fp_seg/http_req"] == 4 + 16 + 200 + 32 + 100 + 8
    assert kb["k_fingerprint/tcp_syn"] == 4 + 16 + 60 + 32 + 40
    assert kb["k_classify"] == 3 * (16 + 5) + 128 + 128 + 60
    assert kb["k_analyze"] == 3 * (32 + 32) + (8 + 2 * 300) + 16 + 8   # record + 32-B analysis record
    assert kb["k_an_features"] == (16 + 32 + 16 + 40) + 2 * 20 + 32 * 5 + 64
    assert kb["k_an_score"] == (64 + 32 + 32) + 8 * 4 + 12 * 10
    assert kb["k_seen_scan"] == 8
