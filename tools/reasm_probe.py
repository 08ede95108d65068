"""Where the reassembly leg's time goes (bench.py other_paths "reassembly"):
the same batch (the TCP / DTLS / QUIC reassembly streams x 40, ~58 k packets)
timed as (a) the Python wrapper's whole call, (b) the C call alone with
buffers allocated beforehand, (c) the device walk alone
(mfp_process_batch_host_seg, pass 1), so (b) - (c) is the host flow table
plus the rebuilt messages' device pass.  One JSON line, best of --reps."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import mercury_amd
    from mercury_amd import api
    gold = os.path.join(ROOT, "tests", "golden")
    parts = []
    for npz in ("reasm_packets.npz", "dtls_reasm_packets.npz", "quic_reasm_packets.npz"):
        z = np.load(os.path.join(gold, npz))
        parts.append((z["arena"], z["desc"]))
    arena = np.concatenate([a for a, _ in parts])
    base = np.cumsum([0] + [len(a) for a, _ in parts[:-1]])
    one = np.concatenate([d.copy() for _, d in parts])
    one["offset"] += np.concatenate([np.full(len(d), b, np.uint64) for (_, d), b in zip(parts, base)])
    desc = np.tile(one, 40)
    n = len(desc)
    ts = np.full(n, 1700000000 * 10**9, np.uint64)
    ctx = mercury_amd.Context("select=tls,ssh,http,dtls,quic;reassembly", device=0)
    lib = ctx.lib
    ctx.process_host_reassembly(arena, desc[:len(one)], ts_ns=ts[:len(one)])
    out = {"packets": n}
    best = lambda xs: round(min(xs) * 1e3, 3)   # noqa: E731
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        ctx.process_host_reassembly(arena, desc, ts_ns=ts)
        t.append(time.perf_counter() - t0)
    out["wrapper_ms"] = best(t)
    cap = ctx.fp_arena_bound(desc) + int(lib.mfp_fp_arena_bound(n, n * 8400))
    fp = np.zeros(cap, np.uint8)
    rec = np.zeros(n, api.RECORD_DTYPE)
    props = np.zeros(n, np.uint16)
    od = np.zeros(n, api.DESC_DTYPE)
    seg = np.zeros(n, api.SEG_DTYPE)
    fp[:] = 1
    t, t2 = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        r = lib.mfp_process_batch_reassembly(ctx.h, ctx.reasm, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                             ts.ctypes.data, rec.ctypes.data, fp.ctypes.data, cap, props.ctypes.data,
                                             od.ctypes.data)
        t.append(time.perf_counter() - t0)
        assert r >= 0, api._err(lib)
        t0 = time.perf_counter()
        r = lib.mfp_process_batch_host_seg(ctx.h, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n,
                                           rec.ctypes.data, fp.ctypes.data, cap, seg.ctypes.data)
        t2.append(time.perf_counter() - t0)
        assert r >= 0, api._err(lib)
    out["c_call_ms"] = best(t)
    out["device_walk_ms"] = best(t2)
    out["flow_table_and_pass2_ms"] = round(out["c_call_ms"] - out["device_walk_ms"], 3)
    out["rate_mpkt_s"] = {"wrapper": round(n / out["wrapper_ms"] / 1e3, 3), "c_call": round(n / out["c_call_ms"] / 1e3, 3)}
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
