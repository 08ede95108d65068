"""--analysis on SSH client KEXINITs: the classifier's user agent is the
protocol string + the comment string (ssh_init_packet::do_analysis
ssh.h:480-499, a data_buffer<512> that is empty without a comment or when the
two do not fit), built by k_analyze_wave from the record's span.  Expected
values: the reference (tests/golden/make_golden_ssh_an.py) on banners with
and without comments, comments around the 512-byte buffer, a NUL in the
comment, bare "\\n" line ends, servers, IPv6, and the libmerc accessor.
"""
import os

import numpy as np
import pytest

import mercury_amd
from tests import test_analysis

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def test_ssh_fixture_shape():
    ref = test_analysis.load_ref_an("ssh_an.tsv.gz")
    z = np.load(os.path.join(GOLD, "ssh_an_packets.npz"))
    assert len(ref) == len(z["desc"]) and sum(r["valid"] for r in ref) > 200
    assert len({round(r["score"], 6) for r in ref if r["valid"]}) > 3   # the user agent moves the score


@pytest.mark.gpu
def test_ssh_analysis_vs_reference():
    z = np.load(os.path.join(GOLD, "ssh_an_packets.npz"))
    cfg = f"select=ssh;resources={os.path.join(GOLD, 'ssh_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        rec, fp, an = ctx.process_host_analysis(z["arena"], z["desc"])
        names = [ctx.process_name(int(p)) for p in an["process"]]
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("ssh_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
