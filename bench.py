"""bench.py -- device-resident fingerprint + classify throughput of the MI355X path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mixed|tls_ch]
                    [--packets P] [--no-analysis] [--e2e-total T]

A step is one pass of the hot path (libmercury_amd.so) over one batch of P
synthetic packets already resident in HBM:

  default       BASELINE config 4: 50 M mixed TLS/HTTP/SSH/TCP packets,
                protocol identification + fingerprint + the --analysis
                process classifier on a SURVEY-sized synthetic resource
                archive (tests/synth_db.py build_survey: ~20 000
                fingerprints, P ~ Zipf on 1..256, ~100 000 pyasn prefixes,
                encrypted-DNS watchlist, domain mappings; regenerated into
                tests/golden/_gen/ when absent); --resources test: the
                small test archive tests/golden/synth_resources.tgz
  --no-analysis config 3: protocol identification + fingerprint only
  --workload tls_ch --packets 10000000 --no-analysis   config 2

Multi-GPU (one process per GPU).  Under torch.distributed.run the ranks come
from RANK/LOCAL_RANK/WORLD_SIZE; a bare `python bench.py --gpus N` starts the N
rank processes itself (before anything touches the GPU) with the same
arguments.  Packets are independent, so every rank processes its own shard
(weak scaling, no data-path collective; all ranks draw from one template pool
so the classifier's label rate is the same on every shard).  A gloo group
carries the barrier and the max-over-ranks time: nothing goes over RCCL.

Rank 0 prints one JSON line.  `roofline` covers the kernels of one step
(timed with HIP events on the stream they run on, mfp_profile_enable) against
the HBM peak; `kernels` breaks the step down per launch.  `roofline.traffic`
comes from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the same command
(profiles/*traffic*.json, tools/pmc_traffic.py) when one matches this
configuration.  `cpu_baseline` is the reference libmerc compiled from
/root/reference (oracle/_ref, travels with the snapshot) or else the C oracle
port, timed on a bounded sample on the host cores (both entry points:
write_json and get_analysis_context).  `end_to_end` is config 5's
H2D/D2H-inclusive rate: --e2e-total packets per job (split over the ranks)
from page-locked host memory through mfp_process_pipelined, reported beside
`value`, never instead of it.
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
TEST_RESOURCES = os.path.join(ROOT, "tests", "golden", "synth_resources.tgz")
TEMPLATE_SEED = {"mixed": 0x5EED0003, "tls_ch": 0x5EED0001}
N_TEMPLATES = 4096
METRIC = "device-resident Mpkt/s + GB/s, fingerprint+classify, mixed-protocol batch"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_device_batch(torch, n, workload, draw_seed, unique, diverse_tls=0.0):
    """`unique` distinct packets generated on the host, replicated on the device."""
    from tests import synth
    u = min(unique, n)
    ua, ud = synth.batch(u, seed=TEMPLATE_SEED[workload], workload=workload, n_templates=N_TEMPLATES,
                         draw_seed=draw_seed, diverse_tls=diverse_tls)
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


GOLD = os.path.join(ROOT, "tests", "golden")
OUTPUT_TOL = 1e-6   # score / p_malware (the reference's fp32 expf)


def golden_applies(n, unique, workload, analysis, resources_kind, draw_seed):
    """bench_sample.npz / bench_diverse_status.bin.gz hold the reference's
    output for the default config-4 batch of rank 0 (tests/golden/make_golden_bench.py)."""
    m = json.load(open(os.path.join(GOLD, "bench_manifest.json")))
    return (analysis and workload == "mixed" and resources_kind == "survey" and n == m["packets"] and
            unique == m["unique"] and draw_seed == m["draw_seed"])


def check_step_output(torch, ctx, rec, an, d_fp, n, u):
    """The timed step's records at 24 000 seeded positions (one per sampled
    unique packet, in a seeded period of the 50 M) against the reference's:
    emit flag, fingerprint type and bytes, analysis validity, status, process,
    malware flag; score and p_malware within OUTPUT_TOL."""
    g = dict(np.load(os.path.join(GOLD, "bench_sample.npz")))   # (an NpzFile decompresses on every access)
    rows = g["rows"].astype(np.int64)
    reps = n // u
    k = np.random.default_rng(0x5EED0B1D).integers(0, reps, len(rows))
    idx = rows + k * u
    r, a = rec[idx], an[idx]
    # the sampled strings, gathered on the device (the arena is tens of GB)
    lens = r["fp_len"].astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    gidx = np.repeat(r["fp_offset"].astype(np.int64) - starts, lens) + np.arange(int(lens.sum()), dtype=np.int64)
    blob = d_fp[torch.from_numpy(gidx).to(d_fp.device)].cpu().numpy().tobytes() if len(gidx) else b""
    ends = np.concatenate([[0], g["fp_ends"].astype(np.int64)])
    gblob = g["fp_blob"].tobytes()
    names = g["proc_names"].tobytes().decode().split("\n")
    bad = []
    for j in range(len(rows)):
        fi = int(g["fp_idx"][j])
        want_fp = gblob[ends[fi]:ends[fi + 1]]
        got_fp = blob[starts[j]:starts[j] + lens[j]]
        emit = int(r["flags"][j] & 1)
        if (emit, int(r["fp_type"][j]), got_fp) != (int(g["emit"][j]), int(g["fp_type"][j]), want_fp):
            bad.append((int(idx[j]), "fingerprint"))
            continue
        valid = int(a["flags"][j] & 1)
        if valid != int(g["valid"][j]):
            bad.append((int(idx[j]), "valid"))
            continue
        if not valid:
            continue
        name = ctx.process_name(int(a["process"][j]))
        mal = int((a["flags"][j] >> 1) & 1)
        pm = float(a["malware_prob"][j]) if a["flags"][j] & 4 else 0.0
        want_name = names[int(g["proc_idx"][j])]
        if (int(a["status"][j]) != int(g["status"][j]) or name != want_name or mal != int(g["malware"][j]) or
                abs(float(a["score"][j]) - float(g["score"][j])) > OUTPUT_TOL or
                (want_name and abs(pm - float(g["p_malware"][j])) > OUTPUT_TOL)):
            bad.append((int(idx[j]), "analysis"))
    return {"ok": not bad, "records_checked": len(rows), "classified_checked": int(g["valid"].sum()),
            "mismatches": len(bad), "first": bad[:5],
            "against": "tests/golden/bench_sample.npz (reference libmerc, make_golden_bench.py)"}


def check_diverse_statuses(an):
    """The diversity leg's first step: every unknown-TLS sighting's status
    (randomized / unlabeled) in stream order against the reference's 17.5 M
    decisions (tests/golden/bench_diverse_status.bin.gz)."""
    import gzip
    m = json.load(open(os.path.join(GOLD, "bench_manifest.json")))
    with gzip.open(os.path.join(GOLD, "bench_diverse_status.bin.gz"), "rb") as f:
        want = np.unpackbits(np.frombuffer(f.read(), np.uint8))[:m["diverse_sightings"]]
    valid = (an["flags"] & 1) != 0
    st = an["status"]
    sight = valid & ((st == 2) | (st == 3))
    got = (st[sight] == 3).astype(np.uint8)
    ok = len(got) == len(want) and bool(np.array_equal(got, want))
    first = None
    if not ok and len(got) == len(want):
        first = int(np.flatnonzero(got != want)[0])
    return {"ok": ok, "sightings": int(len(got)), "reference_sightings": int(len(want)),
            "unlabeled": int(got.sum()), "first_mismatch": first,
            "against": "tests/golden/bench_diverse_status.bin.gz (reference libmerc, make_golden_bench.py)"}


def diverse_multi_rank(torch, ctx, args, n, step, drain, nstep, merge_s, merge_ph, tdist, world, rank):
    """The realistic-diversity leg on several ranks: each rank's batch carries
    per-packet cipher suites (350 k distinct unknown-TLS fingerprints per rank
    and step, the LRU cycling), every step pipelined -- step k's kernels
    launched, then step k-1's sightings decided across the ranks in shard
    order (shard.ordered_prevalence_merge) while they run; the last step's
    merge inside the timed region.  Reports the job rate and each rank's
    merge time beside its kernel time."""
    from mercury_amd import shard
    steps2 = max(1, min(args.steps, 10))
    nstep[0] = 0          # the main leg's last step was decided by its drain()
    step()
    drain()
    nstep[0] = 0
    torch.cuda.synchronize()
    del merge_s[:]
    del merge_ph[:]
    ctx.profile(True)
    tdist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps2):
        step()
    drain()
    torch.cuda.synchronize()
    el_local = time.perf_counter() - t
    tdist.barrier()
    el = shard.max_over_ranks(el_local)
    prof = ctx.profile_read()
    ctx.profile(False)
    kern = sum(v[1] for v in prof.values()) / steps2
    merges = [round(x * 1e3, 3) for x in merge_s]
    per_rank = [None] * world
    tdist.all_gather_object(per_rank, {"rank": rank, "kernel_ms_per_step": round(kern, 4),
                                       "ms_per_step": round(el_local / steps2 * 1e3, 4),
                                       "merge_ms": merges,
                                       "merge_ms_mean": round(float(np.mean(merge_s)) * 1e3, 3) if merge_s else None,
                                       "merge_phase_ms_mean": {k: round(float(np.mean([p.get(k, 0.0) for p in merge_ph]))
                                                                        * 1e3, 3)
                                                               for k in (merge_ph[0] if merge_ph else {})}})
    return {"value": round(n * world * steps2 / el / 1e6, 3), "unit": "Mpkt/s", "steps": steps2,
            "ms_per_step": round(el / steps2 * 1e3, 4), "n_gpus": world,
            "path": "mfp_analyze_batch_device_deferred_pipelined + shard.ordered_prevalence_merge of step k-1 while "
                    "step k runs (each sighting decided once, on its own rank, from the earlier shards' LRU "
                    "summaries); the last step's merge inside the timed region",
            "diverse_tls_fraction": args.diverse_leg, "per_rank": per_rank,
            "what": "the diversity leg's batch on every rank (its own draw), max over ranks"}


def replicate_npz(torch, path, n):
    """The packets of a committed fixture (tests/golden/*.npz: arena + desc),
    replicated on the device to n packets."""
    z = np.load(path)
    ua, ud = z["arena"], z["desc"]
    u = len(ud)
    span = int((ud["offset"].astype(np.int64) + ud["caplen"]).max())
    stride = (span + 64 + 255) // 256 * 256
    reps = (n + u - 1) // u
    host = np.zeros(stride, dtype=np.uint8)
    host[:span] = ua[:span]
    d_arena = torch.from_numpy(host).cuda().repeat(reps)
    desc = np.tile(ud, reps)[:n].copy()
    desc["offset"] += (np.arange(reps, dtype=np.uint64) * np.uint64(stride)).repeat(u)[:n]
    return d_arena, desc, torch.from_numpy(desc.view(np.uint8)).cuda()


def ref_time(npz_or_batch, cfg, threads, seconds):
    """The reference libmerc (oracle/_ref/merc_ref_drv time, write_json per
    packet, one processor per thread) over a fixture's packets; None without it."""
    from tests import pcaplib
    ref = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")
    if not os.path.exists(ref):
        return None
    if isinstance(npz_or_batch, str):
        z = np.load(npz_or_batch)
        a, d = z["arena"], z["desc"]
    else:
        a, d = npz_or_batch
    with tempfile.NamedTemporaryFile(suffix=".mfpb", delete=False) as t:
        path = t.name
    pcaplib.write_mfpb(path, a, d)
    try:
        out = subprocess.run([ref, "time", path, cfg, "-", str(threads), str(seconds), "json"],
                             capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
        r = json.loads(out.decode().strip().splitlines()[-1])
    finally:
        os.unlink(path)
    return {"value": round(r["pps"] / 1e6, 4), "unit": "Mpkt/s", "cores": threads, "kind": "reference",
            "sample": f"{len(d)} packets looped {seconds:.0f} s, write_json per packet, config {cfg!r}"}


def other_paths(torch, steps):
    """The paths config 4 does not exercise, timed on their own batches: QUIC
    Initials (k_quic: key derivation, header protection, AES-GCM, CRYPTO
    frames, fingerprint), STUN + OpenVPN-over-TCP, and the reassembly path
    (device walk, host flow table in stream order, the rebuilt messages'
    device pass) over the TCP / DTLS / QUIC reassembly streams."""
    import mercury_amd
    gold = os.path.join(ROOT, "tests", "golden")
    out = {}
    for name, npz, sel, n in (("quic_initials", "quic_packets.npz", "quic", 2_000_000),
                              ("stun_openvpn", "stun_ovpn_packets.npz", "stun,openvpn_tcp", 4_000_000)):
        d_arena, desc, d_desc = replicate_npz(torch, os.path.join(gold, npz), n)
        ctx = mercury_amd.Context(sel, device=0)
        cap = ctx.fp_arena_bound(desc)
        d_rec = torch.empty(n * mercury_amd.RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        d_fp = torch.empty(cap, dtype=torch.uint8, device="cuda")
        d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
        stream = torch.cuda.current_stream()

        def step():
            ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap,
                               d_used.data_ptr(), stream.cuda_stream)
        step()
        torch.cuda.synchronize()
        ctx.profile(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        prof = ctx.profile_read()
        ctx.profile(False)
        rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
        phases = None
        if os.environ.get("MFP_REPORT_PHASES"):      # probe builds (MFP_K_PHASES): k_quic's phase clock sums
            import ctypes
            fn = getattr(ctx.lib, "mfp_probe_read_quic", None)
            words = (ctypes.c_uint64 * 8)()
            if fn is not None and fn(words) == 0:
                phases = [int(x) for x in words[:5]]
        ctx.close()
        byts = int(desc["caplen"].astype(np.int64).sum())
        kms = {k: round(v[1] / steps, 4) for k, v in prof.items()}
        out[name] = {"value": round(n * steps / el / 1e6, 3), "unit": "Mpkt/s", "packets": n, "steps": steps,
                     "ms_per_step": round(el / steps * 1e3, 4), "gb_per_s": round(byts * steps / el / 1e9, 3),
                     "fingerprints_per_step": int((rec["fp_type"] > 0).sum()), "kernel_ms": kms,
                     "what": f"{npz} (reference pcaps + synthetic) replicated on the device, {sel}"}
        if phases:
            out[name]["quic_phase_clocks"] = phases
        out[name]["cpu_baseline"] = ref_time(os.path.join(gold, npz), sel, cpu_threads(), 6.0)
        del d_arena, d_desc, d_rec, d_fp
        torch.cuda.empty_cache()
    # the reassembly path: one host batch of the three reassembly streams,
    # repeated (the flows reopen on each repetition)
    parts = []
    for npz in ("reasm_packets.npz", "dtls_reasm_packets.npz", "quic_reasm_packets.npz"):
        z = np.load(os.path.join(gold, npz))
        parts.append((z["arena"], z["desc"]))
    reps = 40
    arena = np.concatenate([a for a, _ in parts])
    base = np.cumsum([0] + [len(a) for a, _ in parts[:-1]])
    one = np.concatenate([d.copy() for _, d in parts])
    off = np.concatenate([np.full(len(d), b, np.uint64) for (_, d), b in zip(parts, base)])
    one["offset"] += off
    desc = np.tile(one, reps)
    ctx = mercury_amd.Context("select=tls,ssh,http,dtls,quic;reassembly", device=0)
    ts = np.full(len(desc), 1700000000 * 10**9, np.uint64)
    # warm-up at the timed size (the context's device buffers grow to it),
    # then a fresh flow table for each timed call (the same stream each time)
    ctx.process_host_reassembly(arena, desc, ts_ns=ts, merged=False)
    els = []
    for _ in range(3):
        ctx.lib.mfp_reassembler_destroy(ctx.reasm)
        ctx.reasm = None
        t0 = time.perf_counter()
        rec, fp, props, _, _ = ctx.process_host_reassembly(arena, desc, ts_ns=ts, merged=False)
        els.append(time.perf_counter() - t0)
    el = float(np.mean(els))
    ctx.close()
    # the reference on one thread over the same streams in order (threads
    # would split the flows)
    reasm_cpu = ref_time((arena, one), "select=tls,ssh,http,dtls,quic;reassembly", 1, 6.0)
    out["reassembly"] = {"value": round(len(desc) / el / 1e6, 3), "unit": "Mpkt/s", "packets": len(desc),
                         "ms": round(el * 1e3, 3), "reassembled": int((props & 1).sum()),
                         "what": "host batch (pageable memory): the TCP, DTLS and QUIC reassembly streams "
                                 f"(tests/golden reasm/dtls_reasm/quic_reasm packets) x {reps}, "
                                 "device walk + host flow table + the rebuilt messages' device pass; mean of 3 "
                                 "calls after a warm-up call of the same size, each with a fresh flow table",
                         "cpu_baseline": reasm_cpu}
    return out


def per_packet_shim(seconds=2.0):
    """The libmerc per-packet API as embedders drive it (tests/c/per_packet_bench:
    T threads, one processor each, one call per packet): write_json and
    get_analysis_context through libmercury_amd.so at 1, 8 and 32 threads
    (concurrent calls are combined into device batches,
    mercury_amd/csrc/mfp_libmerc.cpp submit()), and the reference libmerc
    beside it at 1 and 32 threads when oracle/_ref is present."""
    from tests import pcaplib, synth
    prog = os.path.join(ROOT, "tests", "c", "per_packet_bench")
    if not os.path.exists(prog):
        return None
    a, d = synth.batch(20_000, seed=TEMPLATE_SEED["mixed"], workload="mixed", n_templates=N_TEMPLATES)
    pk = [a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes() for x in d]
    res = os.path.join(ROOT, "tests", "golden", "synth_resources.tgz")
    out = {"what": "20 000 mixed packets (tests/synth.py), one processor per thread, one call per packet, "
                   f"{seconds:.0f} s per point; analysis entry with tests/golden/synth_resources.tgz",
           "points": []}
    with tempfile.NamedTemporaryFile(suffix=".pcap", delete=False) as t:
        path = t.name
    pcaplib.write_pcap(path, pk, linktype=1)
    try:
        libs = [("mercury_amd", os.path.join(ROOT, "mercury_amd", "libmercury_amd.so"), (1, 8, 32))]
        ref = os.path.join(ROOT, "oracle", "_ref", "libmerc_ref.so")
        if os.path.exists(ref):
            libs.append(("reference", ref, (1, 32)))
        for name, lib, ths in libs:
            for entry in ("json", "an"):
                for th in ths:
                    r = subprocess.run([prog, lib, path, CONTRACT, res if entry == "an" else "-", str(th), str(seconds),
                                        entry], capture_output=True, timeout=seconds * 6 + 120,
                                       env=dict(os.environ, MFP_SHIM_STATS="1"))
                    if r.returncode != 0:
                        out["points"].append({"lib": name, "entry": entry, "threads": th,
                                              "error": r.stderr.decode(errors="replace")[-300:]})
                        continue
                    x = json.loads(r.stdout.decode().strip().splitlines()[-1])
                    pt = {"lib": name, "entry": x["entry"], "threads": th, "kpkt_s": round(x["pps"] / 1e3, 2),
                          "lat_us_p50": x["lat_us_p50"], "lat_us_p99": x["lat_us_p99"]}
                    for line in r.stderr.decode(errors="replace").splitlines():
                        if '"shim_stats"' in line:        # the combiner's batches (MFP_SHIM_STATS)
                            pt.update(json.loads(line)["shim_stats"])
                        if '"shim_kernels"' in line:      # [launches, total ms] per kernel
                            pt.setdefault("kernels", {}).update(json.loads(line)["shim_kernels"])
                    out["points"].append(pt)
    finally:
        os.unlink(path)
    return out


def cpu_threads():
    """Host threads for the CPU baseline: one GPU's share of the host's cores
    (nproc / 8 on an 8-GPU node), within the cores this process may use."""
    aff = len(os.sched_getaffinity(0))
    return max(1, min(aff, (os.cpu_count() or aff) // 8))


def cpu_baseline(workload, draw_seed, sample_n, threads, seconds, analysis, resources):
    """Reference libmerc (oracle/_ref) if present, else the C oracle port.
    The reference is timed on both of its entry points: write_json (the CLI's
    path, JSON text included) and get_analysis_context (the embedders' path);
    `value` is the write_json rate."""
    from tests import pcaplib, synth
    a, d = synth.batch(sample_n, seed=TEMPLATE_SEED[workload], workload=workload, n_templates=N_TEMPLATES,
                       draw_seed=draw_seed)
    ref = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")
    host = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    if os.path.exists(ref):
        with tempfile.NamedTemporaryFile(suffix=".mfpb", delete=False) as t:
            path = t.name
        pcaplib.write_mfpb(path, a, d)
        try:
            rates = {}
            for entry in ("json", "an"):
                out = subprocess.run([ref, "time", path, CONTRACT, resources if analysis else "-", str(threads),
                                      str(seconds), entry],
                                     capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
                rates[entry] = json.loads(out.decode().strip().splitlines()[-1])
            # the write_json leg at 1 thread, at the box's OMP_NUM_THREADS share,
            # and on every core this process may use, beside the nproc / 8 point
            points = {str(threads): {"threads": threads, "write_json_mpkt_s": round(rates["json"]["pps"] / 1e6, 4)}}
            env = os.environ.get("OMP_NUM_THREADS")
            omp = int(env) if env and env.isdigit() else None
            for th in sorted({1, omp or 1, len(os.sched_getaffinity(0))} - {threads}):
                out = subprocess.run([ref, "time", path, CONTRACT, resources if analysis else "-", str(th),
                                      str(seconds / 2), "json"],
                                     capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
                pr = json.loads(out.decode().strip().splitlines()[-1])
                points[str(th)] = {"threads": th, "write_json_mpkt_s": round(pr["pps"] / 1e6, 4)}
            # the scaling check: the same leg without --analysis (no prevalence
            # LRU) at 1 thread and on all cores
            plain = {}
            if analysis:
                for th in sorted({1, len(os.sched_getaffinity(0))}):
                    out = subprocess.run([ref, "time", path, CONTRACT, "-", str(th), str(seconds / 4), "json"],
                                         capture_output=True, check=True, timeout=seconds * 4 + 120).stdout
                    pr = json.loads(out.decode().strip().splitlines()[-1])
                    plain[str(th)] = {"threads": th, "write_json_mpkt_s": round(pr["pps"] / 1e6, 4)}
            # the baseline: the better of the two per-GPU shares of the host
            # (nproc / 8 and OMP_NUM_THREADS); the reference's rate falls past
            # about 16 threads (its shared LRU lock, analysis.h:372,390)
            share = [str(threads)] + ([str(omp)] if omp and str(omp) in points else [])
            best = max(share, key=lambda k: points[k]["write_json_mpkt_s"])
            what = "with --analysis (resources loaded)" if analysis else "fingerprint only"
            return {"value": points[best]["write_json_mpkt_s"], "unit": "Mpkt/s", "cores": points[best]["threads"],
                    "kind": "reference", "entry": "write_json",
                    "get_analysis_context_mpkt_s": round(rates["an"]["pps"] / 1e6, 4),
                    "get_analysis_context_threads": threads,
                    "thread_points": points,
                    "thread_points_without_analysis": plain,
                    "host": host,
                    "sample": f"{sample_n} {workload} packets looped >= {seconds:.0f} s per entry point "
                              f"({seconds / 2:.0f} s for the extra thread counts), libmerc {what}, one processor "
                              f"per thread; value = the better per-GPU share of the host ({threads} threads = "
                              f"nproc / 8, or OMP_NUM_THREADS); write_json {rates['json']['packets']} packets in "
                              f"{rates['json']['seconds']:.1f} s at {threads} threads"}
        finally:
            os.unlink(path)
    if analysis:
        return None   # the C oracle port restates the fingerprint path only
    from oracle import oracle
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=1)
    reps = max(1, int(seconds / max(t, 1e-3)))
    t, _ = oracle.time_batch(a, d, oracle.config(), threads=threads, reps=reps)
    return {"value": sample_n * reps / t / 1e6, "unit": "Mpkt/s", "cores": threads, "kind": "port", "host": host,
            "sample": f"{sample_n} {workload} packets x {reps} passes, C oracle, {threads} threads"}


def gpu_local_cpus(torch, dev):
    """(NUMA node, CPUs of this process on it) of the GPU's PCIe attachment, or None."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        if node < 0:
            return None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        cpus &= os.sched_getaffinity(0)
        return (node, cpus) if cpus else None
    except Exception:
        return None


def end_to_end(torch, ctx, ua, ud, n_buf, per_rank, analysis, chunk, dist, world, with_json):
    """Runs _end_to_end with the host threads (and so the page-locked buffers
    they allocate, and the JSON writer's threads) on the GPU's NUMA node
    (MFP_E2E_NUMA=0: anywhere).  Measured: JSON text 39.9 -> 58.2 Mpkt/s on 16
    threads, H2D unchanged (profiles/r04k_e2e_numa/)."""
    loc = gpu_local_cpus(torch, torch.cuda.current_device()) if os.environ.get("MFP_E2E_NUMA", "1") == "1" else None
    old = os.sched_getaffinity(0)
    if loc:
        os.sched_setaffinity(0, loc[1])
    try:
        out = _end_to_end(torch, ctx, ua, ud, n_buf, per_rank, analysis, chunk, dist, world, with_json)
    finally:
        if loc:
            os.sched_setaffinity(0, old)
    if out is not None:
        out["numa"] = {"node": loc[0], "cpus": len(loc[1])} if loc else None
    return out


def _end_to_end(torch, ctx, ua, ud, n_buf, per_rank, analysis, chunk, dist, world, with_json):
    """Config 5's host-resident rate: `per_rank` packets per rank from
    page-locked host memory (a buffer of n_buf packets, looped), records,
    fingerprints (and classifier results) back into page-locked host memory,
    through mfp_process_pipelined (two HIP streams: H2D, kernels, D2H
    overlapped).  Timed between barriers; the job time is the max over ranks."""
    from mercury_amd.api import ANALYSIS_DTYPE, ATTR_DB_TAGS, DESC_DTYPE, RECORD_DTYPE
    u = len(ud)
    n = min(n_buf, per_rank)
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
    h_an = torch.empty(n * ANALYSIS_DTYPE.itemsize if analysis else 8, dtype=torch.uint8, pin_memory=True)
    out = (h_rec.numpy().view(RECORD_DTYPE), h_fp.numpy(), h_an.numpy().view(ANALYSIS_DTYPE) if analysis else None)
    d = h_desc.numpy().view(DESC_DTYPE)
    ctx.process_pipelined(av, d, chunk=chunk, analysis=analysis, out=out)   # warm-up (device buffers)
    passes = [n] * (per_rank // n) + ([per_rank % n] if per_rank % n else [])
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    used_tot = 0
    for m in passes:
        dm = d if m == n else d[:m]
        _, used, _ = ctx.process_pipelined(av, dm, chunk=chunk, analysis=analysis, out=out)
        used_tot += used
    el = time.perf_counter() - t0
    if dist:
        dist.barrier()
        from mercury_amd import shard
        el = shard.max_over_ranks(el)
    in_bytes = (int(desc["caplen"].astype(np.int64).sum()) + 16 * n) * per_rank / n
    out_bytes = 32 * per_rank + used_tot + (ANALYSIS_DTYPE.itemsize * per_rank if analysis else 0)
    total = per_rank * world
    res = {"value": round(total / el / 1e6, 3), "unit": "Mpkt/s", "packets": total, "n_gpus": world,
           "packets_per_gpu": per_rank, "host_buffer_packets": n, "chunk": chunk,
           "seconds": round(el, 4), "h2d_gb_per_s_per_gpu": round(in_bytes / el / 1e9, 3),
           "d2h_gb_per_s_per_gpu": round(out_bytes / el / 1e9, 3), "pinned": True,
           "path": "mfp_process_pipelined: pinned host arena -> 2 HIP streams (H2D | kernels | D2H) -> pinned "
                   "records + fingerprints" + (" + classifier results" if analysis else "")}
    if with_json:
        try:
            m = min(n, 2_000_000)
            ap = None
            if analysis:   # the archive tags' probabilities for the writer (not part of the timed leg above)
                ap = np.zeros(m * ATTR_DB_TAGS, np.float64)
                ctx.process_pipelined(av, d[:m], chunk=chunk, analysis=True, out=(out[0], out[1], out[2]),
                                      attr_prob=ap)
            res["json"] = json_writer_rate(av, d, out[0], out[1], m, 16, ctx if analysis else None, out[2], ap)
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
    from mercury_amd.api import ATTR_DB_TAGS
    rec_a, fp_a, an_a = out_a
    ap_sets = [torch.empty(batch * ATTR_DB_TAGS * 8, dtype=torch.uint8, pin_memory=True).numpy().view(np.float64)
               for _ in range(2)] if analysis else [None, None]
    fp_b = torch.empty(fp_a.nbytes // max(1, n // batch), dtype=torch.uint8, pin_memory=True).numpy()
    rec_b = torch.empty(batch * 32, dtype=torch.uint8, pin_memory=True).numpy().view(RECORD_DTYPE)
    an_b = torch.empty(batch * ANALYSIS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True).numpy().view(ANALYSIS_DTYPE) if analysis else None
    sets = [(rec_a[:batch], fp_a, an_a[:batch] if analysis else None), (rec_b, fp_b, an_b)]
    ts = np.full(batch, 1_700_000_000 * 10**9, np.uint64)
    ends = np.zeros(batch, np.uint64)
    cap = batch * 1024
    jbuf = np.empty(cap, np.uint8)
    skipped = ctypes.c_uint64(0)
    total = [0]

    errors = []

    def write(dk, o, ap):
        try:
            if analysis:
                got = lib.mfp_write_json_batch_analysis(ctx.h, av.ctypes.data, dk.ctypes.data, len(dk),
                                                        o[0].ctypes.data, o[1].ctypes.data, o[2].ctypes.data,
                                                        ap.ctypes.data, ts.ctypes.data, jbuf.ctypes.data, cap,
                                                        ends.ctypes.data, ctypes.byref(skipped), threads)
            else:
                got = lib.mfp_write_json_batch(av.ctypes.data, dk.ctypes.data, len(dk), o[0].ctypes.data,
                                               o[1].ctypes.data, ts.ctypes.data, jbuf.ctypes.data, cap,
                                               ends.ctypes.data, ctypes.byref(skipped), threads)
            if got < 0:
                raise RuntimeError("mfp_write_json_batch failed: " + lib.mfp_last_error().decode())
            if skipped.value:
                raise RuntimeError(f"mfp_write_json_batch skipped {skipped.value} records")
            if got < len(dk) * 16:
                raise RuntimeError(f"implausible JSON size {got} for {len(dk)} packets")
            total[0] += got
        except Exception as e:   # re-raised by the caller after join()
            errors.append(e)

    nb = n // batch
    d0 = np.ascontiguousarray(d[:batch])
    ctx.process_pipelined(av, d0, chunk=chunk, analysis=analysis, out=sets[0], attr_prob=ap_sets[0])
    write(d0, sets[0], ap_sets[0])                       # warm-up (page faults on the text buffer)
    total[0] = 0
    t0 = time.perf_counter()
    prev = None
    for k in range(nb):
        dk = np.ascontiguousarray(d[k * batch:(k + 1) * batch])
        o, ap = sets[k % 2], ap_sets[k % 2]
        th = threading.Thread(target=write, args=prev) if prev else None
        if th:
            th.start()
        ctx.process_pipelined(av, dk, chunk=chunk, analysis=analysis, out=o, attr_prob=ap)
        if th:
            th.join()
        if errors:
            raise errors[0]
        prev = (dk, o, ap)
    write(*prev)
    el = time.perf_counter() - t0
    if errors:
        raise errors[0]
    return {"value": round(nb * batch / el / 1e6, 3), "unit": "Mpkt/s", "packets": nb * batch, "batch": batch,
            "threads": threads, "json_gb_per_s": round(total[0] / el / 1e9, 3),
            "path": "pinned packets -> mfp_process_pipelined (batch k) || mfp_write_json_batch" +
                    ("_analysis" if analysis else "") + " (batch k-1) -> JSON text in host memory" +
                    (" (records with their 'analysis' objects)" if analysis else "")}


def json_writer_rate(arena, desc, rec, fp, n, threads, ctx=None, an=None, ap=None):
    """Host JSON record assembly (mfp_write_json_batch[_analysis], the text of
    stateful_pkt_proc::write_json, with the "analysis" objects under
    --analysis) over the first n results of the end-to-end leg, `threads` host
    threads: Mpkt/s and GB/s of JSON text."""
    import ctypes
    from mercury_amd.api import load_library
    lib = load_library()
    ts = np.full(n, 1_700_000_000 * 10**9, np.uint64)
    ends = np.zeros(n, np.uint64)
    skipped = ctypes.c_uint64(0)
    cap = n * 1024
    buf = np.empty(cap, np.uint8)
    if ctx is not None:
        fn = lib.mfp_write_json_batch_analysis
        args = (ctx.h, arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data, fp.ctypes.data, an.ctypes.data,
                ap.ctypes.data, ts.ctypes.data, buf.ctypes.data, cap, ends.ctypes.data, ctypes.byref(skipped), threads)
    else:
        fn = lib.mfp_write_json_batch
        args = (arena.ctypes.data, desc.ctypes.data, n, rec.ctypes.data, fp.ctypes.data, ts.ctypes.data,
                buf.ctypes.data, cap, ends.ctypes.data, ctypes.byref(skipped), threads)
    got = fn(*args)                                       # warm-up (page faults on buf)
    if got < 0:
        raise RuntimeError("mfp_write_json_batch failed: " + lib.mfp_last_error().decode())
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        got = fn(*args)
    el = (time.perf_counter() - t0) / reps
    return {"value": round(n / el / 1e6, 3), "unit": "Mpkt/s", "packets": n, "threads": threads,
            "json_bytes": int(got), "gb_per_s": round(got / el / 1e9, 3), "records": int((rec["flags"][:n] & 1).sum()),
            "skipped": int(skipped.value),
            "analysis_objects": int(((an["flags"][:n] & 1) != 0).sum()) if an is not None else 0,
            "note": "host threads after D2H; text byte-identical to the reference's write_json" +
                    (" (with its 'analysis' objects)" if ctx is not None else "")}


# protocol bin of a record's message (mfp_kernels.hip msg_bin) and its name
BIN_NAMES = ["tls_ch", "http_req", "tcp_syn", "http_resp", "other", "tls_sh", "ssh", "dtls"]
MSG_BIN = np.array([4, 0, 5, 5, 6, 6, 1, 3, 2, 2, 7, 7, 7] + [4] * 243, np.int64)


def arena_slots(rec, desc):
    """Fingerprint-arena bytes the device path reserves for these packets:
    a 64-byte aligned slot holding each string and its 8-byte hash; a TLS
    ClientHello's slot sized by its bound min(2 * caplen + 64, 8192)."""
    fl = rec["fp_len"].astype(np.int64)
    exact = np.where(fl > 0, ((fl + 7) // 8 * 8 + 8 + 63) // 64 * 64, 0)
    bound = np.minimum(2 * desc["caplen"].astype(np.int64) + 64, 8192)
    by_bound = ((bound + 7) // 8 * 8 + 8 + 63) // 64 * 64
    return int(np.where(rec["msg"] == 1, np.maximum(exact, by_bound), exact).sum())


def kernel_bytes(rec, desc, an, n_fallback=0, an_stats=None, tables=None):
    """Algorithmic HBM bytes per step of each kernel:
    what the kernel must read and write at least, from the packets' own
    sizes.  k_classify: descriptor + the packet's first 128 bytes + the bin id
    and index; a bin kernel: index + descriptor + the whole packet + record +
    the fingerprint (+ its 8-byte hash); the classifier kernels: see below.
    Reads of the archive's tables (the pool copies strings are verified
    against, feature-table slots, priors, update lists) are NOT algorithmic
    bytes: a step re-reads the same few thousand entries millions of times and
    the caches serve them; `tables` (a dict), when given, receives them per
    kernel."""
    tb = tables if tables is not None else {}
    cap = desc["caplen"].astype(np.int64)
    fl = rec["fp_len"].astype(np.int64)
    hashed = np.where((rec["flags"] & 4) != 0, 8, 0)
    b = MSG_BIN[rec["msg"].astype(np.int64)]
    per_pkt = 4 + 16 + cap + 32 + fl + hashed
    out = {"k_classify": int((16 + np.minimum(cap, 128) + 5).sum())}
    sums = np.bincount(b, weights=per_pkt, minlength=8)
    for k, nm in enumerate(BIN_NAMES):
        for kern in ("k_fingerprint/", "k_fp_seg/", "k_fp_tls1/", "k_fp_lds/"):
            out[kern + nm] = int(sums[k])
    # the fallback lane re-walks the packets the bin kernels hand back (count
    # only: their mean per-packet bytes stand in for theirs)
    out["k_fingerprint/fallback"] = int(n_fallback * per_pkt.mean()) if len(per_pkt) else 0
    if an is not None:
        # the classifier's five kernels (mfp_analysis.hip); per-kernel counts
        # come from the device counters (mfp_analysis_counters).  Table bytes
        # are SURVEY 8(d)'s: the pool copy of each verified string, one 32-B
        # slot per feature lookup, 8 B per prior and 12 B per update entry
        st = an_stats or {}
        A = an.dtype.itemsize
        valid = (an["flags"] & 1) != 0
        scored = valid & (an["process"] != 0xFFFFFFFF)
        sn = np.where((rec["sni_len"] == 0xffff) | (rec["msg"] == 15), 0, rec["sni_len"]).astype(np.int64)
        ua = np.where(rec["ua_len"] == 0xffff, 0, rec["ua_len"]).astype(np.int64)
        ngroups = (len(rec) + 63) // 64
        # k_analyze: record in, analysis record out; per classified packet the
        # stored string hash and the fingerprint verified against its pool copy;
        # the 16-B work item of each packet with more to do; the sighting bitmap
        out["k_analyze"] = int(len(rec) * (32 + A) + (valid * (8 + fl)).sum() +
                               16 * st.get("work_items", 0) + 8 * ngroups)
        tb["k_analyze"] = int((valid * fl).sum())
        # k_seen_scan: the bitmap, each sighting's record and hash, one 24-B
        # sighting-slot update per distinct fingerprint per block
        out["k_seen_scan"] = int(8 * ngroups + st.get("pending", 0) * (32 + 8) + 24 * st.get("seen_merges", 0))
        # k_an_features: work item, record, descriptor and the 40-B address
        # window of each work item; server name and user agent with their pool
        # copies (scored packets); one 32-B slot per feature lookup; the 64-B
        # entry written to the lane or wave scorer's list
        out["k_an_features"] = int(st.get("work_items", 0) * (16 + 32 + 16 + 40) + (scored * (sn + ua)).sum() +
                                   64 * (st.get("lane_scored", 0) + st.get("deferred", 0)))
        tb["k_an_features"] = int((scored * (sn + ua)).sum() + 32 * st.get("feature_slots", 0))
        # k_an_score: list entry, fingerprint entry, priors, update entries and
        # the analysis record of each lane-scored packet
        out["k_an_score"] = int(st.get("lane_scored", 0) * (64 + 32 + A))
        tb["k_an_score"] = int(8 * st.get("lane_priors", 0) + 12 * st.get("lane_updates", 0))
        # k_analyze_wave: the same for each wave-scored packet
        out["k_analyze_wave"] = int(st.get("deferred", 0) * (64 + 32 + A))
        tb["k_analyze_wave"] = int(8 * st.get("wave_priors", 0) + 12 * st.get("wave_updates", 0))
        # k_analyze_resolve: one 8-byte sighting bitmap word per 64 packets, and per
        # pending sighting its record, its sighting-table slot (24 B) and its result
        out["k_analyze_resolve"] = int(8 * ngroups + st.get("pending", 0) * (32 + 24 + A))
    return out


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


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes
    (this process never touches the GPU) with the torch.distributed.run
    environment, rank 0's stdout passed through; exit with the worst status."""
    import signal
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    log(f"[spawn] {n} rank processes: {[p.pid for p in procs]}")
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            r = p.poll()
            if r is None:
                continue
            pending.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in pending:   # one rank failed: the others would wait at a barrier forever
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.2)
    return rc


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
    ap.add_argument("--resources", default="survey", choices=["survey", "test"],
                    help="survey: the SURVEY-sized synthetic archive (config 4); test: tests/golden/synth_resources.tgz")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-total", type=int, default=200_000_000,
                    help="config 5: host-resident (H2D/D2H-inclusive) packets per job, split over the ranks; 0 = skip")
    ap.add_argument("--e2e-buffer", type=int, default=10_000_000,
                    help="packets in each rank's page-locked source buffer (looped up to its share)")
    ap.add_argument("--e2e-chunk", type=int, default=1_000_000)
    ap.add_argument("--no-json-leg", action="store_true")
    ap.add_argument("--diverse-leg", type=float, default=1.0,
                    help="fraction of TLS ClientHellos with per-packet cipher suites in the realistic-diversity "
                         "leg (reported beside value; 0 = skip)")
    ap.add_argument("--no-other-paths", action="store_true",
                    help="skip the QUIC / STUN+OpenVPN / reassembly legs")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check without a GPU: ranks start, join the gloo group, report, exit")
    args = ap.parse_args()
    analysis = not args.no_analysis

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import mercury_amd

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[rank {rank}] note: WORLD_SIZE={world} overrides --gpus {args.gpus}")
    tdist = None
    if world > 1:
        import torch.distributed as tdist
        # control only (barrier, max-over-ranks): gloo on the host, no RCCL;
        # single node: the loopback interface (the hostname may not resolve)
        if os.environ.get("MASTER_ADDR") in ("127.0.0.1", "localhost") and os.path.exists("/sys/class/net/lo"):
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        tdist.init_process_group("gloo")
    if args.dry_run:
        info = {"rank": rank, "local_rank": local, "pid": os.getpid()}
        seen = [None] * world
        if tdist:
            tdist.all_gather_object(seen, info)
            tdist.barrier()
        else:
            seen = [info]
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": seen, "backend": "gloo" if tdist else None}),
                  flush=True)
        if tdist:
            tdist.destroy_process_group()
        return
    if os.environ.get("MFP_BENCH_DEVICE0") == "1":
        # rehearsal of the multi-rank path on a one-GPU box: every rank on device 0
        # (never a bench line: the ranks share one GPU)
        local = 0
    torch.cuda.set_device(local)

    workload = args.workload
    n = args.packets or (50_000_000 if workload == "mixed" else 10_000_000)
    draw_seed = TEMPLATE_SEED[workload] + 1 + rank * 7919   # different packets per rank, one template pool

    t0 = time.time()
    ua, ud, d_arena, desc, d_desc = build_device_batch(torch, n, workload, draw_seed, args.unique)
    log(f"[rank {rank}] batch on cuda:{local}: {n} packets, {int(desc['caplen'].astype(np.int64).sum()) / 1e9:.2f} GB "
        f"({time.time() - t0:.1f} s to build)")

    resources, db = None, None
    if analysis:
        if args.resources == "survey":
            from tests import synth_db
            t1 = time.time()
            # rank 0 builds the archive (~30 s of host work), the others wait at
            # a gloo barrier and find the file (build_survey's write is atomic)
            if rank == 0:
                resources = synth_db.build_survey()
            if tdist:
                tdist.barrier()
            resources = synth_db.build_survey()
            log(f"[rank {rank}] survey archive {os.path.getsize(resources) / 1e6:.1f} MB ({time.time() - t1:.1f} s)")
        else:
            resources = TEST_RESOURCES
        cfg = f"select={CONTRACT};resources={resources};analysis"
        t1 = time.time()
        ctx = mercury_amd.Context(cfg, device=local)
        assert ctx.analysis_enabled
        db = dict(mercury_amd.resource_stats(resources))
        db.pop("disabled", None)
        db["archive_bytes"] = os.path.getsize(resources)
        db["device_table_bytes"] = ctx.device_table_bytes()
        db["load_seconds"] = round(time.time() - t1, 2)
    else:
        cfg = CONTRACT if args.tls_format == 0 else f"select={CONTRACT};format=tls/{args.tls_format}"
        ctx = mercury_amd.Context(cfg, device=local)
    tls_format = mercury_amd.parse_filter(cfg)[1] if not analysis else None

    # size the fp arena from the unique set: each string's 64-byte slot, the
    # TLS ClientHellos' slots by their upper bound (k_fp_tls1 reserves before it walks)
    rec_u, fp_u = ctx.process_host(ua, ud)
    distinct_fps = len(set(mercury_amd.fingerprints(rec_u, fp_u)) - {""})
    reps = (n + len(ud) - 1) // len(ud)
    cap = int(arena_slots(rec_u, ud) * reps * 1.02) + (2 << 30)
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_fp = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
    d_an = torch.empty(n * mercury_amd.ANALYSIS_DTYPE.itemsize if analysis else 1, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    prev = None
    if analysis and tdist:
        # the shards of one stream: unknown-TLS statuses decided in shard order
        # (shard.ordered_prevalence_merge), every rank on its own copy of the LRU
        from mercury_amd import shard
        prev = mercury_amd.Prevalence(100000)
        ctx.set_prevalence(prev)
        ctx.defer(True)

    # several ranks: the steps are pipelined -- step k's kernels are launched,
    # then step k-1's sightings are merged across the ranks while they run
    # (mfp_analyze_batch_device_deferred_pipelined; two sets of output buffers)
    sets = [(d_rec, d_fp, d_used, d_an)]
    if prev is not None:
        sets.append((torch.empty_like(d_rec), torch.empty_like(d_fp), torch.zeros_like(d_used),
                     torch.empty_like(d_an)))
    nstep = [0]
    merge_s = []          # host seconds of each ordered cross-rank merge (several ranks)
    merge_ph = []         # ... and its phases (shard.last_merge_phases)

    def timed_merge():
        tm = time.perf_counter()
        shard.ordered_prevalence_merge(ctx, prev, rank * n)
        merge_s.append(time.perf_counter() - tm)
        merge_ph.append(dict(shard.last_merge_phases))

    def step():
        r_, f_, u_, a_ = sets[nstep[0] % len(sets)]
        ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, r_.data_ptr(), f_.data_ptr(), cap,
                           u_.data_ptr(), stream.cuda_stream)
        if analysis and prev is None:
            ctx.analyze_device(d_arena.data_ptr(), d_desc.data_ptr(), n, r_.data_ptr(), f_.data_ptr(),
                               a_.data_ptr(), stream.cuda_stream)
        elif analysis:
            ctx.analyze_device_deferred_pipelined(d_arena.data_ptr(), d_desc.data_ptr(), n, r_.data_ptr(),
                                                  f_.data_ptr(), a_.data_ptr(), stream.cuda_stream)
            if nstep[0]:
                timed_merge()   # step k-1, step k in flight
        nstep[0] += 1

    def drain():
        # the last step's merge (inside the timed region)
        if prev is not None and nstep[0]:
            ctx.analysis_defer_newest()
            timed_merge()

    for _ in range(args.warmup):
        step()
    drain()
    nstep[0] = 0
    torch.cuda.synchronize()
    reserved, overflow, used, n_fallback = [int(x) for x in d_used.cpu()]
    if overflow:
        raise RuntimeError("fp arena overflow")

    ctx.profile(True)   # HIP events around every kernel launch, on `stream`
    if tdist:
        tdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if tdist:
        tdist.barrier()
    elapsed = time.perf_counter() - t_start
    d_rec, d_fp, d_used, d_an = sets[(args.steps - 1) % len(sets)]   # the last step's outputs
    prof = ctx.profile_read()
    ctx.profile(False)
    if tdist:
        from mercury_amd import shard
        elapsed = shard.max_over_ranks(elapsed)

    rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
    caplen_bytes = int(desc["caplen"].astype(np.int64).sum())
    fp_bytes = int(rec["fp_len"].astype(np.int64).sum())
    assert fp_bytes == used
    an_info = None
    if analysis:
        an = d_an.cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE)
        valid = (an["flags"] & 1) != 0
        st = np.bincount(an["status"][valid], minlength=5)
        an_info = {"classified": int(valid.sum()),
                   "status": {mercury_amd.api.STATUS_NAMES[i]: int(st[i]) for i in range(5)},
                   "malware": int(((an["flags"] & 2) != 0).sum())}
    output_check = None
    if rank == 0 and golden_applies(n, args.unique, workload, analysis, args.resources, draw_seed):
        output_check = check_step_output(torch, ctx, rec, an, d_fp, n, len(ud))
        log(f"[rank 0] timed step's output vs the reference: {output_check}")
    kern_ms = {k: v[1] / args.steps for k, v in prof.items()}
    step_kern_ms = sum(kern_ms.values())
    dominant = max(kern_ms, key=kern_ms.get)

    total_pkts = n * world
    value = total_pkts * args.steps / elapsed / 1e6
    an_counters = ctx.analysis_counters() if analysis else None
    if analysis and os.environ.get("MFP_REPORT_PHASES"):   # probe builds (MFP_AN_PHASES): k_analyze_wave clock sums
        import ctypes
        words = (ctypes.c_uint64 * 21)()
        ctx.lib.mfp_analysis_counters(ctx.h, words, 21)
        an_counters["wave_phase_clocks"] = [int(x) for x in words[13:21]]
    if os.environ.get("MFP_REPORT_PHASES"):   # probe builds (MFP_K_PHASES): walker phase clock sums
        import ctypes
        for tu in ("tls", "http"):
            fn = getattr(ctx.lib, f"mfp_probe_read_{tu}", None)
            if fn is not None:
                words = (ctypes.c_uint64 * 8)()
                if fn(words) == 0:
                    (an_counters if an_counters is not None else {})[f"{tu}_phase_clocks"] = [int(x) for x in words[:5]]
    ktables = {}
    kbytes = kernel_bytes(rec, desc, an if analysis else None, n_fallback, an_counters, ktables)
    # the step's algorithmic bytes: the same per-kernel definition summed over
    # the kernels the step launched (so roofline.step and its split agree)
    alg_bytes = sum(kbytes.get(k, 0) or 0 for k in kern_ms)
    achieved = alg_bytes / (step_kern_ms * 1e-3) / 1e9
    diverse = None
    if analysis and args.diverse_leg > 0 and world > 1:
        del d_arena, d_desc
        torch.cuda.empty_cache()
        _, _, d_arena, _, d_desc = build_device_batch(torch, n, workload, draw_seed, args.unique,
                                                      diverse_tls=args.diverse_leg)
        diverse = diverse_multi_rank(torch, ctx, args, n, step, drain, nstep, merge_s, merge_ph, tdist, world, rank)
    if analysis and args.diverse_leg > 0 and world == 1:
        # realistic diversity: the same step over a batch whose TLS ClientHellos
        # carry per-packet cipher suites -- hundreds of thousands of distinct
        # fingerprints per step, unknown to the archive, cycling the 100 000-entry LRU
        del d_arena, d_desc
        torch.cuda.empty_cache()
        ua2, ud2, d_arena, desc2, d_desc = build_device_batch(torch, n, workload, draw_seed, args.unique,
                                                              diverse_tls=args.diverse_leg)
        rec2u, fp2u = ctx.process_host(ua2, ud2)
        distinct2 = len(set(mercury_amd.fingerprints(rec2u, fp2u)) - {""})
        step()
        torch.cuda.synchronize()
        diverse_check = None
        if golden_applies(n, args.unique, workload, analysis, args.resources, draw_seed):
            # the first diversity step follows the main leg's steps: its 17.5 M
            # LRU decisions against the reference's
            diverse_check = check_diverse_statuses(sets[0][3].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE))
            log(f"[rank 0] diversity step's LRU decisions vs the reference: {diverse_check}")
        ctx.profile(True)
        # (as many steps as the main leg, up to 10: the pipelined form's last
        # decision -- mfp_analysis_flush, one step's host decision -- is the
        # one not hidden behind kernels, and it is spread over these steps)
        steps2 = max(1, min(args.steps, 10))
        t2 = time.perf_counter()
        for _ in range(steps2):
            step()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t2
        prof2 = ctx.profile_read()
        ctx.profile(False)
        an2 = d_an.cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE)
        v2 = (an2["flags"] & 1) != 0
        st2 = np.bincount(an2["status"][v2], minlength=5)
        sync_leg = {"value": round(n * steps2 / el2 / 1e6, 3), "ms_per_step": round(el2 / steps2 * 1e3, 4),
                    "classifier_ms": {k: round(v[1] / steps2, 4) for k, v in prof2.items()
                                      if k.startswith(("k_analyze", "k_an_", "k_seen"))},
                    "kernel_ms": round(sum(v[1] for v in prof2.values()) / steps2, 4),
                    "host_ms": round(el2 / steps2 * 1e3 - sum(v[1] for v in prof2.values()) / steps2, 4),
                    "path": "mfp_analyze_batch_device: each step's sightings decided before it returns"}
        # the same steps with the decisions pipelined (mfp_analyze_batch_device_pipelined):
        # step k's kernels run while step k-1's sightings are decided on the host
        # (stream order kept; two sets of output buffers, alternating)
        psets = [(d_rec, d_fp, d_used, d_an),
                (torch.empty_like(d_rec), torch.empty_like(d_fp), torch.zeros_like(d_used), torch.empty_like(d_an))]

        def pstep(k):
            r_, f_, u_, a_ = psets[k % 2]
            ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, r_.data_ptr(), f_.data_ptr(), cap,
                               u_.data_ptr(), stream.cuda_stream)
            ctx.analyze_device_pipelined(d_arena.data_ptr(), d_desc.data_ptr(), n, r_.data_ptr(), f_.data_ptr(),
                                         a_.data_ptr(), stream.cuda_stream)
        pstep(0)
        pstep(1)
        ctx.analysis_flush()
        torch.cuda.synchronize()
        ctx.profile(True)
        t3 = time.perf_counter()
        for k in range(steps2):
            pstep(k)
        ctx.analysis_flush()
        torch.cuda.synchronize()
        el3 = time.perf_counter() - t3
        prof3 = ctx.profile_read()
        ctx.profile(False)
        an3 = psets[(steps2 - 1) % 2][3].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE)
        v3 = (an3["flags"] & 1) != 0
        st3 = np.bincount(an3["status"][v3], minlength=5)
        del psets
        diverse = {"value": round(n * steps2 / el3 / 1e6, 3), "unit": "Mpkt/s", "steps": steps2,
                   "ms_per_step": round(el3 / steps2 * 1e3, 4),
                   "path": "mfp_analyze_batch_device_pipelined: step k's kernels run while step k-1's sightings are "
                           "decided (stream order, the same decisions); mfp_analysis_flush after the last step, "
                           "inside the timed region",
                   "diverse_tls_fraction": args.diverse_leg,
                   "distinct_fingerprints_per_step": distinct2,
                   "classifier_ms": {k: round(v[1] / steps2, 4) for k, v in prof3.items()
                                     if k.startswith(("k_analyze", "k_an_", "k_seen"))},
                   "kernel_ms": round(sum(v[1] for v in prof3.values()) / steps2, 4),
                   "status": {mercury_amd.api.STATUS_NAMES[i]: int(st3[i]) for i in range(5)},
                   "status_sync": {mercury_amd.api.STATUS_NAMES[i]: int(st2[i]) for i in range(5)},
                   "synchronous": sync_leg,
                   "lru_entries": int(ctx.analysis_stats()[3]),
                   "reference_check": diverse_check,
                   "what": "same step, same archive; the unique packets' TLS ClientHellos get random first two "
                           "cipher suites (tests/synth.py diverse_tls), replicated like the main leg"}
    e2e = None
    if args.e2e_total:
        del d_arena, d_desc, d_fp          # room for the pipeline's staging buffers
        torch.cuda.empty_cache()
        try:
            e2e = end_to_end(torch, ctx, ua, ud, args.e2e_buffer, args.e2e_total // world, analysis,
                             args.e2e_chunk, tdist, world, world == 1 and not args.no_json_leg)
        except Exception as e:   # reported beside the device-resident number, never instead of it
            log(f"[rank {rank}] end-to-end leg failed: {e}")
            if tdist:
                raise
    shim = None
    if world == 1 and not args.no_other_paths:
        try:
            shim = per_packet_shim()
        except Exception as e:   # reported beside the headline, never instead of it
            log(f"per-packet shim leg failed: {e}")
    others = None
    if world == 1 and not args.no_other_paths:
        try:
            others = other_paths(torch, max(1, min(args.steps, 5)))
        except Exception as e:   # reported beside the headline, never instead of it
            log(f"other-paths legs failed: {e}")
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(workload, draw_seed, 200_000, cpu_threads(), args.cpu_seconds, analysis, resources)
            except Exception as e:   # baseline is reported, never the target
                log(f"cpu baseline failed: {e}")
        cfg_key = f"{workload}/{n}/" + (f"analysis/{args.resources}" if analysis else "fp")
        tr = find_traffic(cfg_key)
        traffic = None
        if tr:
            # per-launch counter bytes (dispatch order == the order the step's
            # kernels were first profiled in), and the step total
            traffic = {"step": tr[1]["hbm_bytes_per_step"]}
            names = [k for k in kern_ms]
            fams = {k.split("/")[0] for k in names}
            pl = [x for x in tr[1].get("per_launch") or [] if x["kernel"].split("<")[0] in fams]
            if len(pl) == len(names) and all(abs(prof[k][0] / args.steps - 1.0) < 1e-9 for k in names):
                for k, x in zip(names, pl):
                    traffic[k] = x["hbm_bytes"]
        # the step split into the fingerprint kernels and the classifier's (whose
        # table re-reads are mostly cache-resident, so its traffic/bytes ratio
        # reads differently from the walkers')
        def step_part(pred):
            ks = [k for k in kern_ms if pred(k)]
            ms = sum(kern_ms[k] for k in ks)
            ab = sum(kbytes.get(k, 0) or 0 for k in ks)
            tb = (sum(traffic[k] for k in ks) if isinstance(traffic, dict) and ks and all(k in traffic for k in ks)
                  else None)
            ach = ab / (ms * 1e-3) / 1e9 if ms else 0.0
            return {"kernels": len(ks), "kernel_ms": round(ms, 4), "algorithmic_bytes": ab, "achieved": round(ach, 2),
                    "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": tb,
                    "table_read_bytes": sum(ktables.get(k, 0) for k in ks),
                    "traffic_per_algorithmic_byte": round(tb / ab, 3) if tb and ab else None}
        is_clf = lambda k: k.startswith(("k_analyze", "k_an_", "k_seen"))   # noqa: E731
        step_split = {"walkers": step_part(lambda k: not is_clf(k)), "classifier": step_part(is_clf)}
        n_fp = int((rec["fp_type"] > 0).sum())
        if workload == "mixed":
            wl = ("config 4: 50M mixed TLS/HTTP/SSH/TCP, protocol-ident + fingerprint + --analysis classifier "
                  f"({'SURVEY-sized' if args.resources == 'survey' else 'test'} synthetic resource archive)") \
                if analysis else \
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
                "resources": os.path.relpath(resources, ROOT) if analysis else None,
                "resource_db": db,
                "tls_format": "archive's (tls/1)" if analysis else tls_format,
                "parallelism": f"shard{world}",
                "distinct_fingerprints_per_step": distinct_fps,
            },
            "gb_per_s": round(caplen_bytes * world * args.steps / elapsed / 1e9, 3),
            "fingerprints_per_step": n_fp,
            "fallback_packets_per_step": n_fallback,
            "analysis": an_info,
            "output_check": output_check,
            "roofline": {
                "bound": "hbm",
                "achieved": round(kbytes.get(dominant, 0) / (kern_ms[dominant] * 1e-3) / 1e9, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(kbytes.get(dominant, 0) / (kern_ms[dominant] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                "traffic": (traffic or {}).get(dominant) if isinstance(traffic, dict) else None,
                "traffic_source": os.path.relpath(tr[0], ROOT) if tr else None,
                "kernel": dominant,
                "kernel_ms_per_launch": round(kern_ms[dominant] / max(1.0, prof[dominant][0] / args.steps), 4),
                "algorithmic_bytes_per_launch": kbytes.get(dominant, 0),
                "step": {"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "kernel_ms": round(step_kern_ms, 4), "algorithmic_bytes": alg_bytes,
                         "traffic": traffic if not isinstance(traffic, dict) else traffic.get("step"),
                         "what": "every kernel of one step, back to back on one stream; algorithmic bytes = the "
                                 "sum of the kernels' own (kernels[*].algorithmic_bytes: inputs read once, outputs "
                                 "written once; archive-table re-reads excluded, kernels[*].table_read_bytes)",
                         "split": step_split},
            },
            "kernels": {k: {"launches_per_step": prof[k][0] / args.steps, "ms_per_step": round(v, 4),
                            "algorithmic_bytes": kbytes.get(k),
                            "table_read_bytes": ktables.get(k),
                            "hbm_bytes": traffic.get(k) if traffic else None,
                            "achieved_gb_s": round(kbytes[k] / (v * 1e-3) / 1e9, 2) if kbytes.get(k) and v else None}
                        for k, v in kern_ms.items()},
            "cpu_baseline": cpu,
            "diversity": diverse,
            "analysis_counters": an_counters,
            "end_to_end": e2e,
            "other_paths": others,
            "per_packet_shim": shim,
        }
        checks = [c for c in (output_check, (diverse or {}).get("reference_check")) if c]
        if any(not c["ok"] for c in checks):
            # the records the line times differ from the reference's: no line
            log(json.dumps(out))
            log("bench: the timed output differs from the reference (output_check / diversity.reference_check)")
            sys.exit(3)
        print(json.dumps(out), flush=True)
    ctx.close()
    if tdist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
