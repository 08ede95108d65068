"""File -> JSON / filtered-pcap rate of the `mercury-amd` driver
(mercury_amd/csrc/mfp_drv.cpp): every packet of a pcap file through
pkt_proc::apply() into the batch packet processors, as `mercury -r in.pcap
-f out.json` / `-w out.pcap` drive the reference's processors.

    python tools/drv_rate.py [--unique 1000000] [--loops 5] [--out gpurun_out/drv]

Writes a pcap of the bench's mixed unique packets (tests/synth.py, the
config-4 draw of rank 0) to --tmp, runs the driver over it --loops times
(mercury's -l), output to a file under --tmp, and prints one JSON line per run
with the driver's own summary."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unique", type=int, default=1_000_000)
    ap.add_argument("--loops", type=int, default=5)
    ap.add_argument("--tmp", default="/tmp")
    ap.add_argument("--batch", type=int, nargs="*", default=[0])
    ap.add_argument("--analysis", action="store_true")
    args = ap.parse_args()
    from tests import synth
    t0 = time.time()
    a, d = synth.batch(args.unique, seed=0x5EED0003, workload="mixed", n_templates=4096, draw_seed=0x5EED0004)
    src = os.path.join(args.tmp, "drv_in.pcap")
    import numpy as np
    with open(src, "wb") as f:
        f.write(np.array([0xA1B2C3D4], "<u4").tobytes() + np.array([2, 4], "<u2").tobytes() +
                np.array([0, 0, 65535, 1], "<u4").tobytes())
        hdr = np.zeros((len(d), 4), "<u4")
        hdr[:, 0] = 1700000000 + np.arange(len(d)) // 100000
        hdr[:, 2] = d["caplen"]
        hdr[:, 3] = d["caplen"]
        for i in range(len(d)):
            f.write(hdr[i].tobytes())
            o = int(d["offset"][i])
            f.write(a[o:o + int(d["caplen"][i])].tobytes())
    print(f"pcap: {len(d)} packets, {os.path.getsize(src) / 1e9:.2f} GB ({time.time() - t0:.1f} s)", file=sys.stderr,
          flush=True)
    cfg = "tls,dtls,ssh,http,tcp,tcp.syn_ack"   # a bare list ("select=..." needs the key=value form's ';')
    if args.analysis:
        from tests import synth_db
        cfg = f"select={cfg};resources={synth_db.build_survey()};analysis"
    drv = os.path.join(ROOT, "mercury_amd", "mercury-amd")
    runs = []
    for b in args.batch:
        runs += [("-f", os.path.join(args.tmp, "drv_out.json"), b, False), ("-f", "/dev/null", b, False),
                 ("-w", "/dev/null", b, False), ("-f", "/dev/null", b, True)]
    for flag, out, batch, bulk in runs:
        cmd = [drv, "-r", src, flag, out, "-c", cfg, "-l", str(args.loops)] + (["-B"] if bulk else [])
        if batch:
            cmd += ["-b", str(batch)]
        t = time.time()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        wall = time.time() - t
        if r.returncode:
            print(r.stderr, file=sys.stderr)
            sys.exit(r.returncode)
        st = json.loads(r.stderr.strip().splitlines()[-1])
        st.update({"output": ("json" if flag == "-f" else "pcap") + (" -> file" if out != "/dev/null" else " -> /dev/null"),
                   "apply": "apply_batch per file block" if bulk else "apply() per packet",
                   "analysis": args.analysis, "batch_pkts": batch or 131072, "wall_s": round(wall, 3),
                   "input_gb_per_loop": round(os.path.getsize(src) / 1e9, 3)})
        if out != "/dev/null":
            st["output_bytes"] = os.path.getsize(out)
            os.remove(out)
        print(json.dumps(st), flush=True)
    os.remove(src)


if __name__ == "__main__":
    main()
