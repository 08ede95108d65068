"""The end-to-end leg of bench.py alone (config 5: page-locked host packets ->
mfp_process_pipelined -> page-locked records, strings, classifier results),
for A/B runs and rocprofv3 timelines of the pipeline.

    python tools/e2e_probe.py [--packets 10000000] [--chunk 2000000] [--passes 3] [--no-analysis]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--chunk", type=int, default=2_000_000)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--no-analysis", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    import mercury_amd
    from mercury_amd.api import ANALYSIS_DTYPE, DESC_DTYPE, RECORD_DTYPE
    from tests import synth_db
    analysis = not args.no_analysis
    # the unique set the bench replicates
    ua, ud, d_arena, _, d_desc = bench.build_device_batch(torch, 1_000_000, "mixed", bench.TEMPLATE_SEED["mixed"] + 1,
                                                          1_000_000)
    del d_arena, d_desc
    if analysis:
        cfg = f"select={bench.CONTRACT};resources={synth_db.build_survey()};analysis"
    else:
        cfg = bench.CONTRACT
    ctx = mercury_amd.Context(cfg, device=0)
    u, n = len(ud), args.packets
    span = int(ud["offset"][-1] + ud["caplen"][-1])
    stride = (span + 255) // 256 * 256
    reps = (n + u - 1) // u
    h_arena = torch.empty(stride * reps + 64, dtype=torch.uint8, pin_memory=True)
    av = h_arena.numpy()
    for r in range(reps):
        av[r * stride:r * stride + span] = ua[:span]
    desc = np.tile(ud, reps)[:n].copy()
    desc["offset"] += (np.arange(reps, dtype=np.uint64) * np.uint64(stride)).repeat(u)[:n]
    h_desc = torch.empty(n * 16, dtype=torch.uint8, pin_memory=True)
    h_desc.numpy()[:] = desc.view(np.uint8)
    rec_u, _ = ctx.process_host(ua, ud)
    fp_cap = int((int(rec_u["fp_len"].astype(np.int64).sum()) + 16 * u) * reps * 1.05) + (64 << 20)
    h_rec = torch.empty(n * 32, dtype=torch.uint8, pin_memory=True)
    h_fp = torch.empty(fp_cap, dtype=torch.uint8, pin_memory=True)
    h_an = torch.empty(n * ANALYSIS_DTYPE.itemsize if analysis else 8, dtype=torch.uint8, pin_memory=True)
    out = (h_rec.numpy().view(RECORD_DTYPE), h_fp.numpy(), h_an.numpy().view(ANALYSIS_DTYPE) if analysis else None)
    d = h_desc.numpy().view(DESC_DTYPE)
    ctx.process_pipelined(av, d, chunk=args.chunk, analysis=analysis, out=out)
    t0 = time.perf_counter()
    used = 0
    for _ in range(args.passes):
        _, used, _ = ctx.process_pipelined(av, d, chunk=args.chunk, analysis=analysis, out=out)
    el = time.perf_counter() - t0
    in_bytes = (int(desc["caplen"].astype(np.int64).sum()) + 16 * n) * args.passes
    print(json.dumps({"packets": n * args.passes, "chunk": args.chunk, "analysis": analysis, "seconds": round(el, 4),
                      "mpkt_s": round(n * args.passes / el / 1e6, 2), "h2d_gb_s": round(in_bytes / el / 1e9, 2),
                      "fp_bytes_per_pass": used}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
