"""The libmerc counters of the reference's own unit tests
(unit_tests/libmerc_fixture.cc, cases of libmerc_dbmultiprotocol_test.cc) run
by a plain C program over the public libmerc API (tests/c/libmerc_fixture.c,
built by __graft_entry__.build()).  The program dlopen()s the library under
test:

* CPU: the reference's own libmerc (oracle/_ref/libmerc_ref.so, dev host
  only) -- pins every expected count (with the in-scope filters that replace
  "all") to the reference itself;
* GPU: libmercury_amd.so -- the same counts through the MI355X path.

The pcaps are the reference's test pcaps, written back from
tests/golden/ref_packets.npz (packet bytes, link types and file order kept;
of the large captures ref_packets keeps every packet that emits a record
under the contract selection, a superset of what each case counts, plus every
tenth packet).
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from tests import pcaplib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
PROG = os.path.join(ROOT, "tests", "c", "libmerc_fixture")
RESOURCES = os.path.join(GOLD, "resources-test.tgz")
PCAPS = ["capture2.pcap", "multi_packet_http_request.pcap", "http_rawip.pcap", "sll2_tls.pcap", "sll_tls.pcap",
         "tls_sgt.pcap", "dtls_fragmented_client_hello.pcap", "dtls_fragmented_client_hello_partial.pcap",
         "malware_tls.pcap", "ipv6-domain-faking.pcap", "faketls_potatovpn.pcap"]


def write_pcaps(d):
    with np.load(os.path.join(GOLD, "ref_packets.npz")) as z:
        arena, desc, src = z["arena"], z["desc"], z["sources"]
    base = np.array([x.rsplit(":", 1)[0] for x in src])
    for name in PCAPS:
        idx = np.nonzero(base == name)[0]
        assert len(idx), name
        pkts = [arena[int(desc[i]["offset"]):int(desc[i]["offset"]) + int(desc[i]["caplen"])].tobytes() for i in idx]
        pcaplib.write_pcap(os.path.join(d, name), pkts, linktype=int(desc[idx[0]]["linktype"]))


def run(lib):
    assert os.path.exists(PROG), "tests/c/libmerc_fixture is built by __graft_entry__.build()"
    with tempfile.TemporaryDirectory() as d:
        write_pcaps(d)
        r = subprocess.run([PROG, lib, d, RESOURCES], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    return r


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libmerc_ref.so")),
                    reason="the reference libmerc is built only where /root/reference exists")
def test_fixture_counts_reference_libmerc():
    r = run(os.path.join(ROOT, "oracle", "_ref", "libmerc_ref.so"))
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_fixture_counts_mercury_amd():
    r = run(os.path.join(ROOT, "mercury_amd", "libmercury_amd.so"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 case(s) failed" in r.stdout
