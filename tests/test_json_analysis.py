"""--analysis JSON records and the analysis-context accessors against the
REFERENCE (libmerc with do_analysis and a resource archive), committed by
tests/golden/make_golden_json_analysis.py:

* the "analysis" object (analysis_result::write_json, src/libmerc/result.h:207-252)
  placed as pkt_proc.cc:1211-1213 places it: process, score, malware,
  p_malware, os_info (report_os), status, attributes with their probability
  scores -- archive tags (analysis.h:268-277,335-341), encrypted_channel,
  encrypted_dns and domain_faking (analysis.h:555-570), faketls
  (tls.h:1977-1996);
* the libmerc accessors (mercury_packet_processor_get_attributes,
  analysis_context_get_os_info, analysis_context_get_alpns) through the
  per-packet shims.

Bar: every line byte-identical to the reference (floats as its "%f"), on
crafted packets (every attribute branch), a synthetic mixed batch and the
packets of the reference's own test pcaps (faketls_potatovpn,
ipv6-domain-faking, malware_tls among them) with its resources-test.tgz.
"""
import ctypes
import gzip
import os

import numpy as np
import pytest

import mercury_amd
from mercury_amd.api import ATTR_DB_FIRST, AN_VALID
from tests import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"
TS = 1700000000 * 10**9
SYNTH_RES = os.path.join(GOLD, "synth_resources.tgz")
TEST_RES = os.path.join(GOLD, "resources-test.tgz")


def _lines(name):
    with gzip.open(os.path.join(GOLD, name), "rb") as f:
        return f.read().split(b"\n")[:-1]


def _crafted():
    z = np.load(os.path.join(GOLD, "json_an_crafted.npz"))
    blob = z["json"].tobytes()
    ends = [0] + [int(e) for e in z["json_end"]]
    js = [blob[ends[i]:ends[i + 1]] for i in range(len(ends) - 1)]
    attr = z["attr"].tobytes().split(b"\n")[:-1]
    return z["arena"], z["desc"], js, attr


def _check(lines, gold, skipped):
    assert len(lines) == len(gold)
    for i, (got, want) in enumerate(zip(lines, gold)):
        exp = want + b"\n" if want else b""
        assert got == exp, (i, got[:400], exp[:400])
    assert skipped == 0


def _json_device(arena, desc, resources, threads=1, report_os_in_cfg=False):
    """report_os through mfp_analysis_report_os, or through the config
    string's report_os option (config_generator.cc:35)"""
    extra = ";report_os" if report_os_in_cfg else ""
    ctx = mercury_amd.Context(f"select={CONTRACT};resources={resources};analysis{extra}", device=0)
    assert ctx.analysis_enabled
    if not report_os_in_cfg:
        ctx.report_os(True)
    rec, fp, an, ap = ctx.process_host_analysis(arena, desc, attr_prob=True)
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64),
                                            threads=threads, ctx=ctx, analysis=an, attr_prob=ap)
    return ctx, lines, skipped, an


@pytest.mark.gpu
def test_json_analysis_crafted_device():
    arena, desc, gold, _ = _crafted()
    ctx, lines, skipped, an = _json_device(arena, desc, SYNTH_RES, report_os_in_cfg=True)
    _check(lines, gold, skipped)
    # every attribute branch is exercised by the crafted set
    names = {ctx.attribute_name(b) for a in an for b in range(16) if (int(a["attr"]) >> b) & 1}
    assert {"encrypted_dns", "domain_faking", "faketls", "encrypted_channel"} <= names
    ctx.close()


@pytest.mark.gpu
def test_json_analysis_synthetic_device():
    arena, desc = synth.batch(4000, seed=0x5EED0003)
    ctx, lines, skipped, an = _json_device(arena, desc, SYNTH_RES, threads=4)
    _check(lines, _lines("json_an_synth.txt.gz"), skipped)
    with_an = sum(1 for l in lines if b'"analysis":' in l)
    tagged = int(((an["attr"] >> ATTR_DB_FIRST) != 0).sum())
    assert with_an > 1500 and tagged > 100
    ctx.close()


@pytest.mark.gpu
def test_json_analysis_reference_pcaps_device():
    with np.load(os.path.join(GOLD, "ref_packets.npz")) as z:
        arena, desc = z["arena"], z["desc"]
    ctx, lines, skipped, an = _json_device(arena, desc, TEST_RES, threads=4)
    _check(lines, _lines("json_an_ref.txt.gz"), skipped)
    assert int((an["flags"] & AN_VALID).astype(bool).sum()) > 100
    ctx.close()


# ---- the per-packet libmerc shims ----
class LibmercConfig(ctypes.Structure):
    """struct libmerc_config (include/mercury_amd_libmerc.h, libmerc.h:109-154)."""
    _fields_ = [("dns_json_output", ctypes.c_bool), ("certs_json_output", ctypes.c_bool),
                ("metadata_output", ctypes.c_bool), ("do_analysis", ctypes.c_bool), ("do_stats", ctypes.c_bool),
                ("report_os", ctypes.c_bool), ("output_tcp_initial_data", ctypes.c_bool),
                ("output_udp_initial_data", ctypes.c_bool), ("resources", ctypes.c_char_p),
                ("enc_key", ctypes.c_void_p), ("key_type", ctypes.c_int), ("packet_filter_cfg", ctypes.c_char_p),
                ("fp_proc_threshold", ctypes.c_float), ("proc_dst_threshold", ctypes.c_float),
                ("max_stats_entries", ctypes.c_size_t)]


class Timespec(ctypes.Structure):
    _fields_ = [("tv_sec", ctypes.c_long), ("tv_nsec", ctypes.c_long)]


class AttributeContext(ctypes.Structure):
    _fields_ = [("tag_names", ctypes.POINTER(ctypes.c_char_p)), ("prob_scores", ctypes.POINTER(ctypes.c_longdouble)),
                ("attributes_len", ctypes.c_size_t)]


class OsInformation(ctypes.Structure):
    _fields_ = [("os_name", ctypes.c_char_p), ("os_prevalence", ctypes.c_uint64)]


def _libmerc():
    lib = mercury_amd.load_library()
    vp = ctypes.c_void_p
    lib.mercury_init.restype = vp
    lib.mercury_init.argtypes = [ctypes.POINTER(LibmercConfig), ctypes.c_int]
    lib.mercury_packet_processor_construct.restype = vp
    lib.mercury_packet_processor_construct.argtypes = [vp]
    lib.mercury_packet_processor_destruct.argtypes = [vp]
    lib.mercury_finalize.argtypes = [vp]
    lib.mercury_packet_processor_write_json_linktype.restype = ctypes.c_size_t
    lib.mercury_packet_processor_write_json_linktype.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t,
                                                                 ctypes.POINTER(Timespec), ctypes.c_uint16]
    lib.mercury_packet_processor_get_analysis_context_linktype.restype = vp
    lib.mercury_packet_processor_get_analysis_context_linktype.argtypes = [vp, vp, ctypes.c_size_t,
                                                                           ctypes.POINTER(Timespec), ctypes.c_uint16]
    lib.mercury_packet_processor_get_attributes.restype = ctypes.POINTER(AttributeContext)
    lib.mercury_packet_processor_get_attributes.argtypes = [vp]
    lib.analysis_context_get_fingerprint_status.restype = ctypes.c_int
    lib.analysis_context_get_fingerprint_status.argtypes = [vp]
    lib.analysis_context_get_os_info.restype = ctypes.c_bool
    lib.analysis_context_get_os_info.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(OsInformation)),
                                                 ctypes.POINTER(ctypes.c_size_t)]
    lib.analysis_context_get_alpns.restype = ctypes.c_bool
    lib.analysis_context_get_alpns.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                               ctypes.POINTER(ctypes.c_size_t)]
    lib.mercury_get_classifier.restype = vp
    lib.mercury_get_classifier.argtypes = [vp]
    lib.mercury_get_resource_version.restype = ctypes.c_char_p
    lib.mercury_get_resource_version.argtypes = [vp]
    return lib


def _attr_line(lib, p, ac, i):
    """merc_ref_drv "attr" line of one packet (oracle/ref_driver.cc)."""
    attrs = b""
    at = lib.mercury_packet_processor_get_attributes(p)
    if at:
        a = at.contents
        for k in range(a.attributes_len):
            v = a.prob_scores[k]
            if v == 0:
                continue
            attrs += a.tag_names[k] + b"=" + (b"%.17g" % v) + b";"
    os_, alpn = b"", b""
    if ac:
        oi, ol = ctypes.POINTER(OsInformation)(), ctypes.c_size_t(0)
        if lib.analysis_context_get_os_info(ac, ctypes.byref(oi), ctypes.byref(ol)):
            for k in range(ol.value):
                os_ += oi[k].os_name + b"=%d;" % oi[k].os_prevalence
        ad, al = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_size_t(0)
        if lib.analysis_context_get_alpns(ac, ctypes.byref(ad), ctypes.byref(al)):
            alpn = bytes(ad[k] for k in range(min(al.value, 128))).hex().encode() + b":%d" % al.value
    st = lib.analysis_context_get_fingerprint_status(ac) if ac else 0
    return b"%d\t%d\t%d\t%s\t%s\t%s" % (i, 1 if ac else 0, st, attrs, os_, alpn)


def _run_shims(arena, desc, resources, report_os=True):
    lib = _libmerc()
    cfg = LibmercConfig()
    cfg.packet_filter_cfg = CONTRACT.encode()
    cfg.do_analysis = True
    cfg.report_os = report_os
    cfg.resources = resources.encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc
    p = lib.mercury_packet_processor_construct(mc)
    out = []
    for i in range(len(desc)):
        off, ln = int(desc[i]["offset"]), int(desc[i]["caplen"])
        pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
        ts = Timespec(1700000000, 0)
        ac = lib.mercury_packet_processor_get_analysis_context_linktype(p, pkt, ln, ctypes.byref(ts),
                                                                        int(desc[i]["linktype"]))
        out.append(_attr_line(lib, p, ac, i))
    assert lib.mercury_get_classifier(mc)
    assert lib.mercury_get_resource_version(mc)
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)
    return out


@pytest.mark.gpu
def test_libmerc_accessors_crafted_device():
    """get_attributes / get_os_info / get_alpns per packet (the libmerc
    fixture's check_attr and counter paths, unit_tests/libmerc_fixture.cc:172-314)."""
    arena, desc, _, gold = _crafted()
    got = _run_shims(arena, desc, SYNTH_RES)
    assert got == gold


@pytest.mark.gpu
def test_libmerc_accessors_synthetic_device():
    # the first 1500 packets of the golden's 4000-packet batch (a stream prefix)
    gold = _lines("an_attr_synth.tsv.gz")[:1500]
    a4, d4 = synth.batch(4000, seed=0x5EED0003)
    got = _run_shims(a4, d4[:1500], SYNTH_RES)
    assert got == gold


@pytest.mark.gpu
def test_libmerc_write_json_analysis_device():
    """mercury_packet_processor_write_json_linktype under do_analysis: the
    record text with its "analysis" object, one packet at a time."""
    lib = _libmerc()
    cfg = LibmercConfig()
    cfg.packet_filter_cfg = CONTRACT.encode()
    cfg.do_analysis = True
    cfg.report_os = True
    cfg.resources = SYNTH_RES.encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    p = lib.mercury_packet_processor_construct(mc)
    arena, desc, gold, _ = _crafted()
    buf = ctypes.create_string_buffer(1 << 16)
    for i in range(len(desc)):
        off, ln = int(desc[i]["offset"]), int(desc[i]["caplen"])
        pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
        ts = Timespec(1700000000, 0)
        n = lib.mercury_packet_processor_write_json_linktype(p, buf, len(buf), pkt, ln, ctypes.byref(ts), 1)
        want = gold[i] + b"\n" if gold[i] else b""
        assert buf.raw[:n] == want, (i, buf.raw[:n][:300], want[:300])
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)


def test_golden_json_analysis_shapes():
    """CPU: the committed goldens hold every branch the writer has to match."""
    _, _, js, attr = _crafted()
    text = b"".join(js)
    for k in (b'"status":"randomized_fingerprint"', b'"status":"unlabeled_fingerprint"', b'"os_info":',
              b'"name":"encrypted_dns"', b'"name":"domain_faking"', b'"name":"faketls"',
              b'"name":"encrypted_channel"'):
        assert k in text, k
    syn = b"".join(_lines("json_an_synth.txt.gz"))
    for k in (b'"process":', b'"malware":', b'"p_malware":', b'"name":"malware"', b'"status":"unknown"'):
        assert k in syn, k
    ref = b"".join(_lines("json_an_ref.txt.gz"))
    for k in (b'"name":"faketls"', b'"name":"domain_faking"', b'"name":"encrypted_channel"', b'"name":"malware"'):
        assert k in ref, k
    assert len(attr) == len(js)
