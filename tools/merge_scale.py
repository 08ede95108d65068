"""Per-rank cost of shard.ordered_prevalence_merge's sequence form at the
diversity leg's scale (17.5 M unknown-TLS sightings per rank per step, the
key mix of tests/test_shard.py::_scale_worker), by phase and LRU thread count,
without a process group: what one rank does between the all_gathers.

    python tools/merge_scale.py [--threads 1,4,8,16] [--world 8] [--m 17500000]

Prints one JSON line per thread count (seconds per phase, best of --reps)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))


def keys_for(rank, world, step, m):
    rng = np.random.default_rng(1000 * step + rank)
    keys = rng.integers(0, 350_000, m, dtype=np.int64) + (rank + world * step) * 1_000_000
    hot = rng.random(m) < 0.02
    keys[hot] = rng.integers(0, 64, int(hot.sum()))
    return (keys.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x5EED)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=None, help="the rank measured (default: the last, the most prior)")
    ap.add_argument("--m", type=int, default=17_500_000)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import mercury_amd
    world, m = args.world, args.m
    rank = world - 1 if args.rank is None else args.rank
    # step 0 sets the LRU (every rank's copy is the same), step 1 is measured
    seqs0 = [keys_for(r, world, 0, m) for r in range(world)]
    seqs1 = [keys_for(r, world, 1, m) for r in range(world)]
    for th in [int(x) for x in args.threads.split(",")]:
        os.environ["MFP_LRU_THREADS"] = str(th)
        best = None
        for _ in range(args.reps):
            prev = mercury_amd.Prevalence(100000)
            sums0 = [prev.summary(s) for s in seqs0]
            prev.advance(np.concatenate(sums0[::-1]))
            sums1 = [prev.summary(s) for s in seqs1]      # the other ranks' summaries (computed there)
            seq = seqs1[rank]
            t0 = time.perf_counter()
            mine = prev.summary(seq)
            t1 = time.perf_counter()
            prior = np.concatenate(sums1[:rank][::-1]) if rank else np.zeros(0, np.uint64)
            seen = prev.resolve_shard(seq, prior)
            t2 = time.perf_counter()
            allsum = list(sums1)
            allsum[rank] = mine
            prev.advance(np.concatenate(allsum[::-1]))
            t3 = time.perf_counter()
            ph = {"summary": t1 - t0, "resolve_shard": t2 - t1, "advance": t3 - t2, "total": t3 - t0}
            if best is None or ph["total"] < best["total"]:
                best = ph
        print(json.dumps({"threads": th, "world": world, "rank": rank, "sightings": m,
                          "randomized": int(len(seq) - int(np.asarray(seen).sum())),
                          **{k: round(v * 1e3, 2) for k, v in best.items()}, "unit": "ms"}), flush=True)


if __name__ == "__main__":
    main()
