"""Subnet lookups of the --analysis classifier against the REFERENCE
(tests/golden/lpm_*, made by tests/golden/make_golden_lpm.py from the
reference's subnet_data built out of /root/reference).

subnet_data answers get_asn_info and is_domain_faking (addr.cc:172-208,
707-792) with level-compressed tries (lctrie/lctrie.hpp:347-386) that are not a
clean longest-prefix match on nested prefixes: an IPv6 /32 holding exactly one
/48 counts as "full" (subnet_prefix lctrie_ip.hpp:541-569 caps sizes of 64 or
more host bits at UINT64_MAX), so an address in the /32 outside the /48 has no
ASN.  The build constructs the same tries (mfp_classifier.cpp l_build) and
looks them up with the reference's lct_find (mfp_lctrie.hpp), host and device.

CPU: the host copy of the tries against every query of the golden.
GPU: ClientHellos to a sample of the query addresses through the analysis
path (the ASN moves the naive-Bayes score; domain_faking is an attribute).
"""
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ARCH = os.path.join(GOLD, "lpm_resources.tgz")


def load_ref():
    with gzip.open(os.path.join(GOLD, "lpm_ref.tsv.gz"), "rt", encoding="latin-1") as f:
        return [line.rstrip("\n").split("\t") for line in f]


def test_lpm_golden_shape():
    ref = load_ref()
    m = json.load(open(os.path.join(GOLD, "lpm_manifest.json")))
    assert len(ref) == m["queries"] > 20000
    by = {(r[0], r[1]): (int(r[2]), int(r[3])) for r in ref}
    # the reference's quirk the golden must hold: 2607:f8b0::/32 (15169) holds
    # one /48 (15170); the /32 outside the /48 has no ASN
    assert by[("2607:f8b0::5", "")][0] == 15170
    assert by[("2607:f8b0:1::5", "")][0] == 0
    assert by[("13.89.1.1", "")][0] if ("13.89.1.1", "") in by else True


def test_lpm_host_tries_vs_reference():
    ref = load_ref()
    got = mercury_amd.lpm_query(ARCH, [(r[0], r[1]) for r in ref])
    bad = [(r[0], r[1], (int(r[2]), int(r[3])), g) for r, g in zip(ref, got) if (int(r[2]), int(r[3])) != g]
    assert len(got) == len(ref)
    assert not bad, f"{len(bad)} of {len(ref)} lookups differ from the reference, first {bad[:5]}"


def test_lpm_clean_match_would_differ():
    """The golden distinguishes the reference's tries from a clean longest-prefix
    match: count the queries whose clean answer differs (the /32 gap and its kin)."""
    import ipaddress
    lines = []
    import tarfile
    with tarfile.open(ARCH) as tf:
        for ln in tf.extractfile("pyasn.db").read().decode().splitlines():
            lines.append(ln)
    pref = {}
    for ln in lines:
        if "\t" not in ln or "/" not in ln:
            continue
        net, asn = ln.split("\t", 1)
        try:
            n = ipaddress.ip_network(net, strict=False)
            if n.prefixlen == 0 or not asn.isdigit():
                continue
        except ValueError:
            continue
        pref.setdefault((n.version, int(n.network_address), n.prefixlen), int(asn))
    v6 = sorted(((a, ln), asn) for (v, a, ln), asn in pref.items() if v == 6)
    ref = [r for r in load_ref() if ":" in r[0]][:3000]
    differ = 0
    for r in ref:
        x = int(ipaddress.IPv6Address(r[0]))
        best = (-1, 0)
        for (a, ln), asn in v6:
            if ln > best[0] and (x >> (128 - ln)) == (a >> (128 - ln)):
                best = (ln, asn)
        differ += best[1] != int(r[2])
    assert differ > 0


@pytest.mark.gpu
def test_lpm_device_analysis_vs_reference():
    from tests import test_analysis, test_quic
    z = np.load(os.path.join(GOLD, "lpm_packets.npz"))
    arena, desc = z["arena"], z["desc"]
    ctx = mercury_amd.Context(f"select=tls;resources={ARCH};analysis", device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        rec, fp, an, ap = ctx.process_host_analysis(arena, desc, attr_prob=True)
        names = [ctx.process_name(int(p)) for p in an["process"]]
        tag_names = {b: ctx.attribute_name(b) for b in range(16)}
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("lpm_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert sum(r["status"] == 1 for r in ref) == len(ref)
    assert len({r["score"] for r in ref}) > 50          # the ASN moves the score
    want = test_quic.load_attr_file("lpm_attr.tsv.gz")
    bad = []
    n_fake = 0
    for i, (valid, status, w) in enumerate(want):
        got = {tag_names[b] for b in range(16) if (int(an["attr"][i]) >> b) & 1 and tag_names[b] == "domain_faking"}
        wf = {k for k in w if k == "domain_faking"}
        n_fake += bool(wf)
        if got != wf:
            bad.append((i, got, wf))
    assert not bad, f"{len(bad)} domain_faking mismatches, first {bad[:3]}"
    assert 100 < n_fake < len(want) - 100
