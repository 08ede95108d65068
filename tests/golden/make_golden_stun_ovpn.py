"""STUN and OpenVPN-over-TCP fixtures from the REFERENCE (libmerc 2.18.0 built
by oracle/Makefile.ref, driven by oracle/_ref/merc_ref_drv); run in the dev
container:

    python tests/golden/make_golden_stun_ovpn.py

Outputs (committed):
  stun_ovpn_packets.npz    packets: every packet of the reference's stun.pcap,
                           stun_classic.pcap, openvpn_tcp_single.pcap and
                           openvpn_tcp_multi.pcap; the packets of emix.pcap and
                           surfshark.pcap for which the reference writes a
                           record under config "so"; the synthetic scenarios of
                           tests/stun_ovpn_synth.py and 3000 mutations of them
  stun_ovpn_fp_<cfg>.tsv.gz reference output per packet (write_json path):
                           idx, emit, fp_type, truncated, fingerprint
  stun_ovpn_json_<cfg>.txt.gz the write_json text per packet (so, mix)
  stun_ovpn_an.tsv.gz      reference analysis_context path with
                           stun_resources.tgz (a synthetic archive in the
                           reference format with stun/1 entries)
  stun_resources.tgz       that archive
  stun_ovpn_manifest.json  configurations, sources, counts
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
from tests import pcaplib, stun_ovpn_synth, synth  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

ESCAPED = []   # filled in main(): utf8_safe() of the fixture's SOFTWARE values

PCAPS_ALL = ["stun.pcap", "stun_classic.pcap", "openvpn_tcp_single.pcap", "openvpn_tcp_multi.pcap"]
PCAPS_EMIT = ["emix.pcap", "surfshark.pcap"]
CONFIGS = {
    "so": "stun,openvpn_tcp",
    "mix": "select=tls,dtls,ssh,http,tcp,tcp.syn_ack,stun,openvpn_tcp;format=tls/1",
    "stun": "stun",
}


def ref(mode, path, cfg, res="-"):
    return subprocess.run([REF, mode, path, cfg, res], capture_output=True, check=True).stdout


def utf8_safe(b):
    """The text utf8_safe_string<512> gives the classifier for SOFTWARE value b
    (utf8.hpp:200-340, 1059-1088; stun.h:1024), "" when null: test
    infrastructure only, to key the archive's user agents; checked below
    against the reference's own JSON text for the same values."""
    out = []
    try:
        t = b.decode("utf-8", errors="strict")
    except UnicodeDecodeError:
        return ""
    for ch in t:
        c = ord(ch)
        if 0xd800 <= c <= 0xdfff or 0xe000 <= c <= 0xf8ff or 0xf0000 <= c <= 0xffffd or 0x100000 <= c <= 0x10fffd:
            return ""
        if c < 0x20 or c == 0x7f or c >= 0x80:
            if c > 0xffff:
                c -= 0x10000
                out.append("\\u%04x\\u%04x" % ((c >> 10) + 0xd800, (c & 0x3ff) + 0xdc00))
            else:
                out.append("\\u%04x" % c)
        elif ch in '"\\':
            out.append("\\" + ch)
        else:
            out.append(ch)
    # fit: 511 bytes, a \uXXXX's hex digits only below offset 507 (append_memcpy's strict bound)
    k = 0
    for piece in out:
        if piece.startswith("\\u"):
            for j in range(0, len(piece), 6):
                if k + 2 > 511 or k + 2 >= 507:
                    return ""
                k += 6
        else:
            if k + len(piece) > 511:
                return ""
            k += len(piece)
    return "".join(out)


def make_archive(fps):
    """A resource archive in the reference format (analysis.h:854-931, the
    process entries of tests/synth_db.py): the STUN request fingerprints
    chosen from the fixture, 1..5 processes each, user-agent features keyed
    by SOFTWARE values of the fixture."""
    from tests import synth_db
    rng = np.random.default_rng(0x5EED000C)
    lines = []
    for fp, uas in fps:
        procs = []
        for k in range(int(rng.integers(1, 6))):
            e = synth_db._proc_entry(rng, str(rng.choice(synth_db.PROC_NAMES)), int(rng.integers(1, 500)), [], [],
                                     uas, rng.random() < 0.2, {a: rng.random() < 0.2 for a in synth_db.ATTRS}, False)
            e["classes_port_port"] = {"3478": e["count"], "19302": max(1, e["count"] // 4)}
            # every escaped SOFTWARE value of the fixture is a user agent of every process
            for u in ESCAPED:
                e["classes_user_agent"][u] = int(rng.integers(1, e["count"] + 1))
            e["classes_ip_ip"] = {"3.132.228.249": int(rng.integers(1, e["count"] + 1)),
                                  "13.89.178.27": int(rng.integers(1, e["count"] + 1))}
            procs.append(e)
        lines.append(json.dumps({"str_repr": fp, "fp_type": "stun", "total_count": sum(p["count"] for p in procs),
                                 "process_info": procs}))
    files = {
        "VERSION": "2026.01.01; 2.0.dual\n",
        "fingerprint_db.json": "\n".join(lines) + "\n",
        "fp_prevalence_tls.txt": "",
        "pyasn.db": "\n".join(synth_db.ASN_LINES + ["3.128.0.0/13\t16509", "3.132.0.0/14\t16510"]) + "\n",
    }
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()


def main():
    ESCAPED[:] = sorted({utf8_safe(b) for b in stun_ovpn_synth.SOFTWARE_ESCAPES} - {""})
    keep, sources = [], []
    for name in PCAPS_ALL:
        for i, p in enumerate(pcaplib.read_pcap(os.path.join("/root/reference/unit_tests/pcaps", name))):
            keep.append(p)
            sources.append(f"{name}:{i}")
    for name in PCAPS_EMIT:
        fn = os.path.join("/root/reference/unit_tests/pcaps", name)
        pkts = pcaplib.read_pcap(fn)
        out = ref("fp", fn, CONFIGS["so"]).decode("latin-1").splitlines()
        for i, l in enumerate(out):
            if l.split("\t")[1] == "1":
                keep.append(pkts[i])
                sources.append(f"{name}:{i}")
    scen = stun_ovpn_synth.scenarios()
    for label, p in scen:
        keep.append((1, p))
        sources.append(f"synth:{label}")
    for k, p in enumerate(synth.fuzz([(1, p) for _, p in scen], 3000, seed=0x5EED000D)):
        keep.append(p)
        sources.append(f"fuzz:{k}")
    arena, desc = pcaplib.make_batch(keep)
    np.savez_compressed(os.path.join(HERE, "stun_ovpn_packets.npz"), arena=arena, desc=desc,
                        sources=np.array(sources, dtype="U64"))
    tmp = "/tmp/stun_ovpn_golden.mfpb"
    pcaplib.write_mfpb(tmp, arena, desc)
    counts = {}
    stun_fps = {}
    for key, cfg in CONFIGS.items():
        out = ref("fp", tmp, cfg)
        with gzip.open(os.path.join(HERE, f"stun_ovpn_fp_{key}.tsv.gz"), "wb") as f:
            f.write(out)
        if key in ("so", "mix"):                      # the write_json text
            js = ref("json", tmp, cfg).decode("latin-1").split("\n")[:len(desc)]
            with gzip.open(os.path.join(HERE, f"stun_ovpn_json_{key}.txt.gz"), "wt", encoding="latin-1") as f:
                f.write("\n".join(js) + "\n")
        rows = [l.split(b"\t") for l in out.splitlines()]
        counts[key] = {"emit": sum(int(r[1]) for r in rows), "stun_fp": sum(r[2] == b"16" for r in rows),
                       "openvpn_fp": sum(r[2] == b"14" for r in rows), "truncated": sum(int(r[3]) for r in rows)}
        if key == "stun":
            for i, r in enumerate(rows):
                if r[2] == b"16":
                    stun_fps.setdefault(r[4].decode("latin-1"), i)
    # the escaped SOFTWARE values against the reference's JSON "stun" text
    # (the same utf8_string::write), for the values it accepts
    js_stun = ref("json", tmp, "stun").decode("latin-1")
    for b in stun_ovpn_synth.SOFTWARE_ESCAPES:
        e = utf8_safe(b)
        assert not e or ('"' + e + '"') in js_stun, b
    # archive: about 60 % of the distinct STUN fingerprints, and those of the
    # SOFTWARE scenarios
    rng = np.random.default_rng(0x5EED000E)
    sw_fps = set()
    rows_stun = [l.split(b"\t") for l in ref("fp", tmp, "stun").splitlines()]
    for i, src in enumerate(sources):
        if src.startswith("synth:software") and rows_stun[i][2] == b"16":
            sw_fps.add(rows_stun[i][4].decode("latin-1"))
    chosen = [fp for fp in sorted(stun_fps) if rng.random() < 0.6 or fp in sw_fps]
    uas = ["libjingle", "WebRTC", "first", "second", "Coturn-4.5.2 'dan Eider'", "v6 agent", "x" * 37]
    arch = make_archive([(fp, uas) for fp in chosen])
    apath = os.path.join(HERE, "stun_resources.tgz")
    with open(apath, "wb") as f:
        f.write(arch)
    an = ref("an", tmp, "select=stun;analysis", apath)
    with gzip.open(os.path.join(HERE, "stun_ovpn_an.tsv.gz"), "wb") as f:
        f.write(an)
    arows = [l.split(b"\t") for l in an.splitlines()]
    counts["an"] = {"valid": sum(r[1] == b"1" for r in arows), "labeled": sum(r[3] == b"1" for r in arows),
                    "archive_fps": len(chosen)}
    os.unlink(tmp)
    manifest = {"reference": "cisco/mercury 2.18.0 (/root/reference), libmerc built by oracle/Makefile.ref",
                "driver": "oracle/_ref/merc_ref_drv fp|an <batch> <config> [resources]", "configs": CONFIGS,
                "analysis_config": "select=stun;analysis + stun_resources.tgz",
                "packets": len(keep), "pcaps": PCAPS_ALL + PCAPS_EMIT,
                "synthetic": "tests/stun_ovpn_synth.py scenarios(seed=0x5EED000B) + synth.fuzz(3000, 0x5EED000D)",
                "counts": counts}
    with open(os.path.join(HERE, "stun_ovpn_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(counts))


if __name__ == "__main__":
    main()
