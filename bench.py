"""bench.py -- device-resident fingerprint throughput of the MI355X path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mixed|tls_ch] [--packets P]

A step is one pass of the hot path (libmercury_amd.so, k_fingerprint) over
one batch of P synthetic packets already resident in HBM (BASELINE.json
config 2: 50 M mixed TLS/HTTP/SSH/TCP packets, protocol identification +
fingerprint; `--workload tls_ch --packets 10000000` is config 1).  Packets
are independent, so for N > 1 every rank processes its own batch (weak
scaling, no data-path collective); the barrier and the max-over-ranks timing
use torch.distributed only for measurement.

Rank 0 prints one JSON line with the roofline of the dominant kernel
(k_fingerprint, HIP events on its stream) and the CPU baseline (the
reference libmerc compiled from /root/reference when oracle/_ref travelled
with the snapshot, else the C oracle port), timed on a bounded sample.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_device_batch(torch, n, workload, seed, unique):
    """Unique packets generated on the host, replicated on the device."""
    from tests import synth
    u = min(unique, n)
    ua, ud = synth.batch(u, seed=seed, workload=workload, n_templates=4096)
    span = int(ud["offset"][-1] + ud["caplen"][-1])
    stride = (span + 64 + 255) // 256 * 256
    reps = (n + u - 1) // u
    host = np.zeros(stride, dtype=np.uint8)
    host[:span] = ua[:span]
    d_unique = torch.from_numpy(host).cuda()
    d_arena = d_unique.repeat(reps)
    desc = np.tile(ud, reps)[:n].copy()
    desc["offset"] += (np.arange(reps, dtype=np.uint64) * np.uint64(stride)).repeat(u)[:n]
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    return ua, ud, d_arena, desc, d_desc


def cpu_baseline(workload, seed, sample_n, threads, seconds):
    """Reference libmerc (oracle/_ref) if present, else the C oracle port."""
    from tests import pcaplib, synth
    a, d = synth.batch(sample_n, seed=seed, workload=workload, n_templates=4096)
    ref = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")
    if os.path.exists(ref):
        with tempfile.NamedTemporaryFile(suffix=".mfpb", delete=False) as t:
            path = t.name
        pcaplib.write_mfpb(path, a, d)
        try:
            out = subprocess.run([ref, "time", path, CONTRACT, "-", str(threads), str(seconds)],
                                 capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
            r = json.loads(out.decode().strip().splitlines()[-1])
            return {"value": r["pps"] / 1e6, "unit": "Mpkt/s", "cores": threads, "kind": "reference",
                    "sample": f"{sample_n} {workload} packets (seed {seed:#x}) looped for {r['seconds']:.1f} s, "
                              f"libmerc write_json, one processor per thread, {r['packets']} packets"}
        finally:
            os.unlink(path)
    from oracle import oracle
    reps = 1
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=1)
    reps = max(1, int(seconds / max(t, 1e-3)))
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=reps)
    return {"value": sample_n * reps / t / 1e6, "unit": "Mpkt/s", "cores": threads, "kind": "port",
            "sample": f"{sample_n} {workload} packets x {reps} passes, C oracle, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="mixed", choices=["mixed", "tls_ch"])
    ap.add_argument("--packets", type=int, default=None)
    ap.add_argument("--unique", type=int, default=1_000_000)
    ap.add_argument("--tls-format", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import mercury_amd

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    workload = args.workload
    n = args.packets or (50_000_000 if workload == "mixed" else 10_000_000)
    seed = 0x5EED0003 if workload == "mixed" else 0x5EED0001
    seed += rank * 7919   # different packets per rank

    t0 = time.time()
    ua, ud, d_arena, desc, d_desc = build_device_batch(torch, n, workload, seed, args.unique)
    log(f"[rank {rank}] batch: {n} packets, {int(desc['caplen'].astype(np.int64).sum()) / 1e9:.2f} GB "
        f"({time.time() - t0:.1f} s to build)")

    cfg = CONTRACT if args.tls_format == 0 else f"select={CONTRACT};format=tls/{args.tls_format}"
    ctx = mercury_amd.Context(cfg, device=torch.cuda.current_device())
    # size the fp arena from the unique set (exact per replica)
    rec_u, fp_u = ctx.process_host(ua, ud)
    reps = (n + len(ud) - 1) // len(ud)
    # strings are 16-byte aligned and each wave reserves 128 KiB chunks
    cap = int(int(rec_u["fp_len"].astype(np.int64).sum() + 16 * len(ud)) * reps * 1.05) + (2 << 30)
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_fp = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap,
                           d_used.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    reserved, overflow, used, n_fallback = [int(x) for x in d_used.cpu()]
    if overflow:
        raise RuntimeError("fp arena overflow")

    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
    caplen_bytes = int(desc["caplen"].astype(np.int64).sum())
    fp_bytes = int(rec["fp_len"].astype(np.int64).sum())
    assert fp_bytes == used
    alg_bytes = caplen_bytes + 16 * n + 32 * n + fp_bytes
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9

    total_pkts = n * world
    value = total_pkts * args.steps / elapsed / 1e6
    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, len(os.sched_getaffinity(0)))
            try:
                cpu = cpu_baseline(workload, seed, 200_000, threads, args.cpu_seconds)
            except Exception as e:   # baseline is reported, never the target
                log(f"cpu baseline failed: {e}")
        n_fp = int((rec["fp_type"] > 0).sum())
        out = {
            "metric": "device-resident Mpkt/s + GB/s, fingerprint+classify, mixed-protocol batch",
            "value": round(value, 3),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": ("config 2: 50M mixed TLS/HTTP/SSH/TCP, protocol-ident + fingerprint (classifier not "
                             "yet on device)") if workload == "mixed" else "config 1: 10M TLS ClientHello, fingerprint",
                "packets_per_gpu": n,
                "unique_packets": len(ud),
                "packet_bytes_per_gpu": caplen_bytes,
                "select": CONTRACT,
                "tls_format": args.tls_format,
                "parallelism": f"shard{world}",
            },
            "gb_per_s": round(caplen_bytes * world * args.steps / elapsed / 1e9, 3),
            "fingerprints_per_step": n_fp,
            "fallback_packets_per_step": n_fallback,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": None,
                "kernel": "k_fingerprint",
                "kernel_ms": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": alg_bytes,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
