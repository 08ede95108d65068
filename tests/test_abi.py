"""The drop-in boundary on the CPU: libmercury_amd.so loads, exports every
symbol include/*.h declares, parses the reference's packet_filter_cfg syntax
(global_config.h:143-153,246-275) and refuses to run without a HIP device
(there is no CPU fallback).  No compute calls are made here."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

import mercury_amd
from oracle import oracle

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"#define[^\n]*", "", src)
        for m in re.finditer(r"MFP_EXPORT[^;{(]*?\b(\w+)\s*\(", src):
            names.add(m.group(1))
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", mercury_amd.library_path()], capture_output=True,
                         check=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads():
    lib = mercury_amd.load_library()
    assert lib.mfp_reference_version() == (2 << 16) | (18 << 8)


def test_every_declared_symbol_is_exported():
    decl = declared_symbols()
    assert {"mfp_init", "mfp_process_batch_device", "mfp_process_batch_host", "mfp_parse_filter"} <= decl
    missing = decl - exported_symbols()
    assert not missing, missing


def test_only_declared_symbols_are_exported():
    extra = {s for s in exported_symbols() - declared_symbols() if not s.startswith("_")}
    assert not extra, extra


@pytest.mark.parametrize("cfg,sel,fmt", [
    ("tls", oracle.SEL["tls"], 0),
    ("tls,dtls,ssh,http,tcp,tcp.syn_ack", oracle.SEL_ALL, 0),
    ("select=tls,http;format=tls/1", oracle.SEL["tls"] | oracle.SEL["http"], 1),
    ("select=tls.client_hello;format=tls/2", oracle.SEL["tls.client_hello"], 2),
    ("select=ssh.client;", oracle.SEL["ssh.client"], 0),
    ("format=tls/1;", 0, 1),          # key=value form without select= selects nothing
    ("tls,none", 0, 0),              # proto_identify.h:623-627
])
def test_parse_filter(cfg, sel, fmt):
    assert mercury_amd.parse_filter(cfg) == (sel, fmt)


# what the reference only logs (set_protocols / set_fingerprint_format return
# false, and mercury_init goes on, global_config.h:55-121, 246-276): an unknown
# protocol name ends the list, an unknown format keeps the default
@pytest.mark.parametrize("cfg,sel,fmt", [
    ("select=tls", 0, 0),                                  # a bare list: "select=tls" is one unknown name
    ("tls,bogus,http", oracle.SEL["tls"], 0),              # the list ends at the unknown name
    ("tls, http", oracle.SEL["tls"], 0),                   # the last token keeps its space
    ("select=tls;format=tls/9", oracle.SEL["tls"], 0),
    ("select=tls;format=tls/1, quic/1", oracle.SEL["tls"], 1),   # " quic/1" keeps its space
    ("tls,,http", oracle.SEL["tls"], 0),
])
def test_parse_filter_logged(cfg, sel, fmt):
    assert mercury_amd.parse_filter(cfg) == (sel, fmt)
    assert mercury_amd.api.parse_filter_ex(cfg)[2]        # the reference logs it


# "all" (also the empty and the missing selection, global_config.h:248) and
# lists naming protocols outside the path: this path's protocols run, the
# others write no record; those whose matchers or ports come first are
# recorded in the "other" bits (mfp_device.hpp BLK_*); in the ';' form a key no
# option recognises is a protocol list (config_generator.cc:156-160)
BLK_ALL = (1 << 27) - 1
SEL_EVERY = (1 << 16) - 1


@pytest.mark.parametrize("cfg,sel,other", [
    ("all", SEL_EVERY, BLK_ALL), ("", SEL_EVERY, BLK_ALL), (None, SEL_EVERY, BLK_ALL),
    ("select=all;format=tls/1", SEL_EVERY, BLK_ALL), ("tls,all", SEL_EVERY, BLK_ALL),
    ("all;format=tls/1;reassembly", SEL_EVERY, BLK_ALL), ("select=;format=tls/1", SEL_EVERY, BLK_ALL),
    ("tls,dns", oracle.SEL["tls"], (1 << 1) | (1 << 2)), ("quic,mdns", 1 << 10, 1 << 2),
    ("tls,arp,icmp,tofsee", oracle.SEL["tls"], 0), ("http,rdp,telnet", oracle.SEL["http"], (1 << 13) | (1 << 19)),
    ("all,none", 0, 0), ("tls;metadata=0;none", 0, 0), ("format=tls/1", 0, 0),
])
def test_parse_filter_other_protocols(cfg, sel, other):
    assert mercury_amd.api.parse_filter_ex(cfg)[:2] == (sel, other)


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(mercury_amd.MercuryAmdError, match="no HIP device"):
        mercury_amd.Context("tls")


def test_record_layout_matches_header():
    hdr = open(os.path.join(ROOT, "include", "mfp.h")).read()
    assert "uint64_t offset;" in hdr and mercury_amd.DESC_DTYPE.itemsize == 16
    assert mercury_amd.RECORD_DTYPE.itemsize == 32
    assert ctypes.sizeof(ctypes.c_void_p) == 8


def libmerc_h_symbols():
    """Every function /root/reference/src/libmerc/libmerc.h declares
    (tests/golden/libmerc_h_symbols.txt, made by make_libmerc_symbols.py)."""
    with open(os.path.join(ROOT, "tests", "golden", "libmerc_h_symbols.txt")) as f:
        return [s.strip() for s in f if s.strip()]


def test_every_libmerc_h_function_is_exported():
    names = libmerc_h_symbols()
    assert len(names) == 31 and "mercury_print_git_commit" in names and "get_stats_aggregator_num_entries" in names
    missing = set(names) - exported_symbols()
    assert not missing, missing
    # and each is declared in the drop-in header
    assert not set(names) - declared_symbols()


def test_libmerc_link_program(tmp_path):
    """A C program calling every libmerc.h function compiles against
    include/mercury_amd_libmerc.h and links against libmercury_amd.so alone;
    on the CPU the packet calls fail softly (0 / NULL, logged) and the rest
    answer as the reference's do (libmerc.cc:59-90, 242-253, 377-396, 477-484)."""
    exe = str(tmp_path / "libmerc_link")
    lib_dir = os.path.dirname(mercury_amd.library_path())
    subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "libmerc_link.c"), "-L" + lib_dir, "-l:libmercury_amd.so",
                    "-Wl,-rpath," + lib_dir, "-o", exe], check=True)
    src = open(os.path.join(ROOT, "tests", "c", "libmerc_link.c")).read()
    called = {n for n in libmerc_h_symbols() if re.search(r"\b" + n + r"\s*\(", src)}
    assert called == set(libmerc_h_symbols())
    out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=120).stdout
    kv = dict(line.split(" ", 1) for line in out.strip().splitlines())
    assert kv["version_string"] == "2.18.0" and kv["print_version"] == "2.18.0"
    assert kv["version_number"] == str((2 << 16) | (18 << 8))
    assert kv["init_with_stats"] == "0" and kv["init"] == "1"          # do_stats refused at init
    assert kv["write_stats"] == "0" and kv["stats_entries"] == "0"
    assert kv["fdc"] == "-4" and kv["finalize"] == "0" and kv["logged"] == "1"
    assert kv["accessors"] == "0 0 0 0 0 0 0 0 0"
