"""bench.py -- device-resident fingerprint + classify throughput of the MI355X path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mixed|tls_ch]
                    [--packets P] [--no-analysis]

A step is one pass of the hot path (libmercury_amd.so) over one batch of P
synthetic packets already resident in HBM:

  default       BASELINE config 4: 50 M mixed TLS/HTTP/SSH/TCP packets,
                protocol identification + fingerprint + the --analysis
                process classifier (synthetic resource archive
                tests/golden/synth_resources.tgz, built for this traffic)
  --no-analysis config 3: protocol identification + fingerprint only
  --workload tls_ch --packets 10000000 --no-analysis   config 2

Packets are independent, so for N > 1 every rank processes its own shard
(weak scaling, no data-path collective; all ranks draw from one template pool
so the classifier's label rate is the same on every shard); the barrier and
the max-over-ranks timing use torch.distributed only for measurement.

Rank 0 prints one JSON line.  `roofline` covers the kernels of one step
(timed with HIP events on the stream they run on, mfp_profile_enable) against
the HBM peak; `kernels` breaks the step down per launch.  `roofline.traffic`
comes from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the same command
(profiles/*traffic*.json, tools/pmc_traffic.py) when one matches this
configuration.  `cpu_baseline` is the reference libmerc compiled from
/root/reference (oracle/_ref, travels with the snapshot) or else the C oracle
port, timed on a bounded sample on the host cores.  `end_to_end` is the
H2D/D2H-inclusive rate of the same configuration on --e2e-packets packets in
page-locked host memory (mfp_process_pipelined), reported beside `value`.
"""
import argparse
import glob
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
RESOURCES = os.path.join(ROOT, "tests", "golden", "synth_resources.tgz")
TEMPLATE_SEED = {"mixed": 0x5EED0003, "tls_ch": 0x5EED0001}
N_TEMPLATES = 4096
METRIC = "device-resident Mpkt/s + GB/s, fingerprint+classify, mixed-protocol batch"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_device_batch(torch, n, workload, draw_seed, unique):
    """`unique` distinct packets generated on the host, replicated on the device."""
    from tests import synth
    u = min(unique, n)
    ua, ud = synth.batch(u, seed=TEMPLATE_SEED[workload], workload=workload, n_templates=N_TEMPLATES,
                         draw_seed=draw_seed)
    span = int(ud["offset"][-1] + ud["caplen"][-1])
    stride = (span + 64 + 255) // 256 * 256
    reps = (n + u - 1) // u
    host = np.zeros(stride, dtype=np.uint8)
    host[:span] = ua[:span]
    d_unique = torch.from_numpy(host).cuda()
    d_arena = d_unique.repeat(reps)
    del d_unique
    desc = np.tile(ud, reps)[:n].copy()
    desc["offset"] += (np.arange(reps, dtype=np.uint64) * np.uint64(stride)).repeat(u)[:n]
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    return ua, ud, d_arena, desc, d_desc


def cpu_baseline(workload, draw_seed, sample_n, threads, seconds, analysis):
    """Reference libmerc (oracle/_ref) if present, else the C oracle port."""
    from tests import pcaplib, synth
    a, d = synth.batch(sample_n, seed=TEMPLATE_SEED[workload], workload=workload, n_templates=N_TEMPLATES,
                       draw_seed=draw_seed)
    ref = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")
    if os.path.exists(ref):
        with tempfile.NamedTemporaryFile(suffix=".mfpb", delete=False) as t:
            path = t.name
        pcaplib.write_mfpb(path, a, d)
        try:
            out = subprocess.run([ref, "time", path, CONTRACT, RESOURCES if analysis else "-", str(threads),
                                  str(seconds)],
                                 capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
            r = json.loads(out.decode().strip().splitlines()[-1])
            what = "write_json with --analysis (resources loaded)" if analysis else "write_json"
            return {"value": r["pps"] / 1e6, "unit": "Mpkt/s", "cores": threads, "kind": "reference",
                    "sample": f"{sample_n} {workload} packets looped for {r['seconds']:.1f} s, libmerc {what}, "
                              f"one processor per thread, {r['packets']} packets"}
        finally:
            os.unlink(path)
    if analysis:
        return None   # the C oracle port restates the fingerprint path only
    from oracle import oracle
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=1)
    reps = max(1, int(seconds / max(t, 1e-3)))
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=reps)
    return {"value": sample_n * reps / t / 1e6, "unit": "Mpkt/s", "cores": threads, "kind": "port",
            "sample": f"{sample_n} {workload} packets x {reps} passes, C oracle, {threads} threads"}


def end_to_end(torch, ctx, ua, ud, n, analysis, steps, chunk):
    """Host-resident rate: packets in page-locked host memory, records,
    fingerprints (and classifier results) back in host memory, through
    mfp_process_pipelined (two streams: H2D, kernels, D2H overlapped)."""
    from mercury_amd.api import ANALYSIS_DTYPE, DESC_DTYPE, RECORD_DTYPE
    u = len(ud)
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
    rec_u, fp_u = ctx.process_host(ua, ud)
    fp_cap = int((int(rec_u["fp_len"].astype(np.int64).sum()) + 16 * u) * reps * 1.05) + (64 << 20)
    h_rec = torch.empty(n * 32, dtype=torch.uint8, pin_memory=True)
    h_fp = torch.empty(fp_cap, dtype=torch.uint8, pin_memory=True)
    h_an = torch.empty(n * 24 if analysis else 8, dtype=torch.uint8, pin_memory=True)
    out = (h_rec.numpy().view(RECORD_DTYPE), h_fp.numpy(), h_an.numpy().view(ANALYSIS_DTYPE) if analysis else None)
    d = h_desc.numpy().view(DESC_DTYPE)
    ctx.process_pipelined(av, d, chunk=chunk, analysis=analysis, out=out)   # warm-up (device buffers)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, used, _ = ctx.process_pipelined(av, d, chunk=chunk, analysis=analysis, out=out)
    el = (time.perf_counter() - t0) / steps
    in_bytes = int(desc["caplen"].astype(np.int64).sum()) + 16 * n
    out_bytes = 32 * n + used + (24 * n if analysis else 0)
    res = {"value": round(n / el / 1e6, 3), "unit": "Mpkt/s", "packets": n, "steps": steps, "chunk": chunk,
           "ms_per_step": round(el * 1e3, 3), "h2d_gb_per_s": round(in_bytes / el / 1e9, 3),
           "d2h_gb_per_s": round(out_bytes / el / 1e9, 3), "pinned": True,
           "path": "mfp_process_pipelined: pinned host arena -> 2 HIP streams (H2D | kernels | D2H) -> pinned "
                   "records + fingerprints" + (" + classifier results" if analysis else "")}
    try:
        res["json"] = json_writer_rate(av, d, out[0], out[1], min(n, 2_000_000), 16, analysis)
        jr = res["json"]["value"]
        res["json"]["with_gpu_path_serial_mpkt_s"] = round(1.0 / (1.0 / res["value"] + 1.0 / jr), 3)
        res["json_overlapped"] = json_overlapped(torch, ctx, av, d, n, analysis, chunk, out)
    except Exception as e:
        log(f"json leg failed: {e}")
    return res


def json_overlapped(torch, ctx, av, d, n, analysis, chunk, out_a, batch=2_000_000, threads=16):
    """Whole host path with JSON text: batches of `batch` packets go through
    mfp_process_pipelined while the JSON writer (16 host threads, ctypes
    releases the GIL) formats the previous batch's results; two result sets
    alternate.  Packets in pinned host memory -> JSON text in host memory."""
    import ctypes
    import threading
    from mercury_amd.api import ANALYSIS_DTYPE, RECORD_DTYPE, load_library
    lib = load_library()
    rec_a, fp_a, an_a = out_a
    fp_b = torch.empty(fp_a.nbytes // max(1, n // batch), dtype=torch.uint8, pin_memory=True).numpy()
    rec_b = torch.empty(batch * 32, dtype=torch.uint8, pin_memory=True).numpy().view(RECORD_DTYPE)
    an_b = torch.empty(batch * 24, dtype=torch.uint8, pin_memory=True).numpy().view(ANALYSIS_DTYPE) if analysis else None
    sets = [(rec_a[:batch], fp_a, an_a[:batch] if analysis else None), (rec_b, fp_b, an_b)]
    ts = np.full(batch, 1_700_000_000 * 10**9, np.uint64)
    ends = np.zeros(batch, np.uint64)
    cap = batch * 640
    jbuf = np.empty(cap, np.uint8)
    skipped = ctypes.c_uint64(0)
    total = [0]

    def write(dk, o):
        got = lib.mfp_write_json_batch(av.ctypes.data, dk.ctypes.data, len(dk), o[0].ctypes.data, o[1].ctypes.data,
                                       ts.ctypes.data, jbuf.ctypes.data, cap, ends.ctypes.data,
                                       ctypes.byref(skipped), threads)
        if got < 0:
            raise RuntimeError("mfp_write_json_batch failed")
        total[0] += got

    nb = n // batch
    d0 = np.ascontiguousarray(d[:batch])
    ctx.process_pipelined(av, d0, chunk=chunk, analysis=analysis, out=sets[0])
    write(d0, sets[0])                                   # warm-up (page faults on the text buffer)
    total[0] = 0
    t0 = time.perf_counter()
    prev = None
    for k in range(nb):
        dk = np.ascontiguousarray(d[k * batch:(k + 1) * batch])
        o = sets[k % 2]
        th = threading.Thread(target=write, args=prev) if prev else None
        if th:
            th.start()
        ctx.process_pipelined(av, dk, chunk=chunk, analysis=analysis, out=o)
        if th:
            th.join()
        prev = (dk, o)
    write(*prev)
    el = time.perf_counter() - t0
    return {"value": round(nb * batch / el / 1e6, 3), "unit": "Mpkt/s", "packets": nb * batch, "batch": batch,
            "threads": threads, "json_gb_per_s": round(total[0] / el / 1e9, 3),
            "path": "pinned packets -> mfp_process_pipelined (batch k) || mfp_write_json_batch (batch k-1) -> "
                    "JSON text in host memory"}


def json_writer_rate(arena, desc, rec, fp, n, threads, analysis):
    """Host JSON record assembly (mfp_write_json_batch, the text of
    stateful_pkt_proc::write_json) over the first n results of the end-to-end
    leg, `threads` host threads: Mpkt/s and GB/s of JSON text."""
    import ctypes
    from mercury_amd.api import load_library
    lib = load_library()
    ts = np.full(n, 1_700_000_000 * 10**9, np.uint64)
    ends = np.zeros(n, np.uint64)
    skipped = ctypes.c_uint64(0)
    cap = n * 1024
    buf = np.empty(cap, np.uint8)
    args = (arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data, fp.ctypes.data, ts.ctypes.data,
            buf.ctypes.data, cap, ends.ctypes.data, ctypes.byref(skipped), threads)
    got = lib.mfp_write_json_batch(*args)                 # warm-up (page faults on buf)
    if got < 0:
        raise RuntimeError("mfp_write_json_batch failed")
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        got = lib.mfp_write_json_batch(*args)
    el = (time.perf_counter() - t0) / reps
    return {"value": round(n / el / 1e6, 3), "unit": "Mpkt/s", "packets": n, "threads": threads,
            "json_bytes": int(got), "gb_per_s": round(got / el / 1e9, 3), "records": int((rec["flags"][:n] & 1).sum()),
            "skipped": int(skipped.value),
            "note": "host threads after D2H; text byte-identical to the reference's write_json" +
                    (" minus the 'analysis' object (not built yet)" if analysis else "")}


def find_traffic(cfg_key):
    """Counter-derived HBM bytes per step for this configuration, if profiled."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            t = json.load(open(f))
        except Exception:
            continue
        if t.get("config") == cfg_key:
            best = (f, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="mixed", choices=["mixed", "tls_ch"])
    ap.add_argument("--packets", type=int, default=None)
    ap.add_argument("--unique", type=int, default=1_000_000)
    ap.add_argument("--tls-format", type=int, default=0, help="without --analysis (else the archive's)")
    ap.add_argument("--no-analysis", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-packets", type=int, default=10_000_000,
                    help="host-resident (H2D/D2H-inclusive) leg on this many packets; 0 = skip")
    ap.add_argument("--e2e-chunk", type=int, default=2_000_000)
    args = ap.parse_args()
    analysis = not args.no_analysis

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
    draw_seed = TEMPLATE_SEED[workload] + 1 + rank * 7919   # different packets per rank, one template pool

    t0 = time.time()
    ua, ud, d_arena, desc, d_desc = build_device_batch(torch, n, workload, draw_seed, args.unique)
    log(f"[rank {rank}] batch: {n} packets, {int(desc['caplen'].astype(np.int64).sum()) / 1e9:.2f} GB "
        f"({time.time() - t0:.1f} s to build)")

    if analysis:
        cfg = f"select={CONTRACT};resources={RESOURCES};analysis"
        ctx = mercury_amd.Context(cfg, device=torch.cuda.current_device())
        assert ctx.analysis_enabled
    else:
        cfg = CONTRACT if args.tls_format == 0 else f"select={CONTRACT};format=tls/{args.tls_format}"
        ctx = mercury_amd.Context(cfg, device=torch.cuda.current_device())
    tls_format = mercury_amd.parse_filter(cfg)[1] if not analysis else None

    # size the fp arena from the unique set (exact per replica)
    rec_u, fp_u = ctx.process_host(ua, ud)
    reps = (n + len(ud) - 1) // len(ud)
    cap = int(int(rec_u["fp_len"].astype(np.int64).sum() + 16 * len(ud)) * reps * 1.05) + (2 << 30)
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_fp = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
    d_an = torch.empty(n * 24 if analysis else 1, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap,
                           d_used.data_ptr(), stream.cuda_stream)
        if analysis:
            ctx.analyze_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(),
                               d_an.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    reserved, overflow, used, n_fallback = [int(x) for x in d_used.cpu()]
    if overflow:
        raise RuntimeError("fp arena overflow")

    ctx.profile(True)   # HIP events around every kernel launch, on `stream`
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t_start
    prof = ctx.profile_read()
    ctx.profile(False)
    if dist:
        from mercury_amd import shard
        elapsed = shard.max_over_ranks(elapsed, device="cuda")

    rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
    caplen_bytes = int(desc["caplen"].astype(np.int64).sum())
    fp_bytes = int(rec["fp_len"].astype(np.int64).sum())
    assert fp_bytes == used
    # algorithmic bytes per step: every packet
    # read once, its descriptor, its 32-B record and its fingerprint written;
    # the classifier re-reads the record and the fingerprint of each
    # classified packet and writes a 24-B analysis record per packet
    alg_bytes = caplen_bytes + 16 * n + 32 * n + fp_bytes
    an_info = None
    if analysis:
        an = d_an.cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE)
        valid = (an["flags"] & 1) != 0
        alg_bytes += 32 * n + 24 * n + int(rec["fp_len"][valid].astype(np.int64).sum())
        st = np.bincount(an["status"][valid], minlength=5)
        an_info = {"classified": int(valid.sum()),
                   "status": {mercury_amd.api.STATUS_NAMES[i]: int(st[i]) for i in range(5)},
                   "malware": int(((an["flags"] & 2) != 0).sum())}
    kern_ms = {k: v[1] / args.steps for k, v in prof.items()}
    step_kern_ms = sum(kern_ms.values())
    dominant = max(kern_ms, key=kern_ms.get)
    achieved = alg_bytes / (step_kern_ms * 1e-3) / 1e9

    total_pkts = n * world
    value = total_pkts * args.steps / elapsed / 1e6
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, len(os.sched_getaffinity(0)))
            try:
                cpu = cpu_baseline(workload, draw_seed, 200_000, threads, args.cpu_seconds, analysis)
            except Exception as e:   # baseline is reported, never the target
                log(f"cpu baseline failed: {e}")
        cfg_key = f"{workload}/{n}/{'analysis' if analysis else 'fp'}"
        tr = find_traffic(cfg_key)
        traffic = None
        if tr:
            traffic = tr[1]["hbm_bytes_per_step"]
        n_fp = int((rec["fp_type"] > 0).sum())
        e2e = None
        if world == 1 and args.e2e_packets:
            del d_arena, d_desc, d_fp          # room for the pipeline's staging buffers
            torch.cuda.empty_cache()
            try:
                e2e = end_to_end(torch, ctx, ua, ud, args.e2e_packets, analysis, 3, args.e2e_chunk)
            except Exception as e:   # reported beside the device-resident number, never instead of it
                log(f"end-to-end leg failed: {e}")
        if workload == "mixed":
            wl = ("config 4: 50M mixed TLS/HTTP/SSH/TCP, protocol-ident + fingerprint + --analysis classifier "
                  "(synthetic resource archive)") if analysis else \
                 "config 3: 50M mixed TLS/HTTP/SSH/TCP, protocol-ident + fingerprint"
        else:
            wl = "config 2: 10M TLS ClientHello, fingerprint" + (" + classifier" if analysis else "")
        if n != (50_000_000 if workload == "mixed" else 10_000_000):
            wl += f" (at {n} packets)"
        out = {
            "metric": METRIC,
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
                "workload": wl,
                "packets_per_gpu": n,
                "unique_packets": len(ud),
                "packet_bytes_per_gpu": caplen_bytes,
                "select": CONTRACT,
                "analysis": analysis,
                "resources": os.path.relpath(RESOURCES, ROOT) if analysis else None,
                "tls_format": "archive's (tls/1)" if analysis else tls_format,
                "parallelism": f"shard{world}",
            },
            "gb_per_s": round(caplen_bytes * world * args.steps / elapsed / 1e9, 3),
            "fingerprints_per_step": n_fp,
            "fallback_packets_per_step": n_fallback,
            "analysis": an_info,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": os.path.relpath(tr[0], ROOT) if tr else None,
                "kernel": "step pipeline (every kernel of one step, back to back on one stream)",
                "kernel_ms": round(step_kern_ms, 4),
                "dominant_kernel": dominant,
                "algorithmic_bytes_per_launch": alg_bytes,
            },
            "kernels": {k: {"launches_per_step": prof[k][0] / args.steps, "ms_per_step": round(v, 4)}
                        for k, v in kern_ms.items()},
            "cpu_baseline": cpu,
            "end_to_end": e2e,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
