"""--analysis on SSH client KEXINITs (ssh_init_packet::do_analysis
ssh.h:480-499): the user agent is the protocol string + the comment string in
a data_buffer<512> (empty when there is no comment or when they do not fit).
Fixtures from the REFERENCE (oracle/_ref/merc_ref_drv an); run in the dev
container:

    python tests/golden/make_golden_ssh_an.py

Outputs (committed):
  ssh_an_packets.npz     SSH banners + KEXINITs in one segment (clients and
                         servers): comments absent / empty / long (protocol +
                         comment of 510..514 bytes) / with a NUL, bare "\\n"
                         line ends, banners without a KEXINIT
  ssh_resources.tgz      a resource archive in the reference format with the
                         ssh fingerprints of those packets and user-agent
                         features keyed by protocol + comment
  ssh_an.tsv.gz          reference analysis_context results per packet
"""
import gzip
import io
import json
import os
import subprocess
import sys
import tarfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth, synth_db  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

CFG = "ssh"


def packets(rng):
    out = []
    protos = [b"SSH-2.0-OpenSSH_9.6", b"SSH-2.0-PuTTY_Release_0.80", b"SSH-2.0-libssh_0.10.6", b"SSH-1.99-Cisco-1.25"]
    comments = [None, b"", b"Ubuntu-3ubuntu13", b"FreeBSD-20240701", b"x" * 200]
    for k in range(240):
        proto = protos[k % len(protos)]
        c = comments[(k // len(protos)) % len(comments)]
        nl = b"\r\n" if k % 7 else b"\n"
        banner = proto + (b"" if c is None else b" " + c) + nl
        kex = synth.ssh_kexinit(rng)
        sport, dport = (int(rng.integers(1024, 65535)), 22) if k % 9 else (22, int(rng.integers(1024, 65535)))
        out.append(synth.frame(synth.tcp(banner + kex, sport=sport, dport=dport), 6, v6=(k % 11 == 0)))
    # protocol + comment around the 512-byte buffer, and a NUL inside the comment
    for total in (509, 510, 511, 512, 513, 514, 700):
        proto = b"SSH-2.0-LongAgent"
        c = b"c" * (total - len(proto) - 1)          # minus the '\r' the comment keeps
        out.append(synth.frame(synth.tcp(proto + b" " + c + b"\r\n" + synth.ssh_kexinit(rng), sport=40000 + total,
                                         dport=22), 6))
    out.append(synth.frame(synth.tcp(b"SSH-2.0-Nul Com\x00ment\r\n" + synth.ssh_kexinit(rng), sport=45000, dport=22), 6))
    out.append(synth.frame(synth.tcp(b"SSH-2.0-OnlyBanner Hello\r\n", sport=45001, dport=22), 6))
    return out


def user_agents(pk):
    """protocol + comment of each packet (the archive's user-agent keys)."""
    uas = []
    for p in pk:
        d = p[14 + (40 if p[12:14] == b"\x86\xdd" else 20) + 20:]
        line = d.split(b"\n", 1)[0] + b"\n"
        sp = line.find(b" ")
        if 0 <= sp < line.find(b"\n"):
            uas.append((line[:sp] + line[sp + 1:-1]).decode("latin-1"))
    return uas


def archive(fps, uas, rng):
    lines = []
    for fp in fps:
        procs = []
        for k in range(int(rng.integers(1, 5))):
            e = synth_db._proc_entry(rng, str(rng.choice(synth_db.PROC_NAMES)), int(rng.integers(1, 500)), [], [],
                                     uas, rng.random() < 0.2, {a: rng.random() < 0.2 for a in synth_db.ATTRS}, False)
            e["classes_port_port"] = {"22": e["count"]}
            procs.append(e)
        lines.append(json.dumps({"str_repr": fp, "fp_type": "ssh", "total_count": sum(p["count"] for p in procs),
                                 "process_info": procs}))
    files = {"VERSION": "2026.01.01; 2.0.dual\n", "fingerprint_db.json": "\n".join(lines) + "\n",
             "fp_prevalence_tls.txt": "", "pyasn.db": "\n".join(synth_db.ASN_LINES) + "\n"}
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode("latin-1")
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()


def main():
    rng = np.random.default_rng(0x5EED0010)
    pk = packets(rng)
    arena, desc = pcaplib.make_batch([(1, p) for p in pk])
    np.savez_compressed(os.path.join(HERE, "ssh_an_packets.npz"), arena=arena, desc=desc)
    tmp = "/tmp/ssh_an.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    out = subprocess.run([REF, "fp", tmp, CFG, "-"], capture_output=True, check=True).stdout.decode("latin-1")
    fps = sorted({l.split("\t")[4] for l in out.splitlines() if l.split("\t")[2] == "5"})
    chosen = [fp for fp in fps if rng.random() < 0.8]
    uas = sorted(set(user_agents(pk)))
    apath = os.path.join(HERE, "ssh_resources.tgz")
    with open(apath, "wb") as f:
        f.write(archive(chosen, uas, rng))
    an = subprocess.run([REF, "an", tmp, CFG, apath], capture_output=True, check=True).stdout
    with gzip.open(os.path.join(HERE, "ssh_an.tsv.gz"), "wb") as f:
        f.write(an)
    rows = [l.split(b"\t") for l in an.splitlines()]
    print(json.dumps({"packets": len(pk), "ssh_fps": len(fps), "archive": len(chosen),
                      "valid": sum(r[1] == b"1" for r in rows), "labeled": sum(r[3] == b"1" for r in rows)}))
    os.unlink(tmp)


if __name__ == "__main__":
    main()
