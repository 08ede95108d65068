"""Synthetic tunnelled packets for the decapsulation fixtures
(pkt_proc.cc:959-1049: GRE, VXLAN, Geneve, IP-in-IP), test infrastructure run
by tests/golden/make_golden_tunnel.py in the dev container.

Inner messages: TLS ClientHellos, HTTP requests, TCP SYNs and QUIC Initials.
Tunnel variants: GRE over IP (with and without the checksum word, with the
key bit the reference does not skip, non-IP protocol types), GRE over UDP
4754, VXLAN (I flag set / clear, inner VLAN, inner ARP), Geneve (Ethernet,
IP, BSD-loopback and unknown payload types, option words), stacks of up to
six levels (the reference walks four), IPv6 outer headers and headers cut
short at every byte.
"""
import struct

import numpy as np

from tests import quic_synth, synth


def gre(payload, proto=0x0800, csum=False, key=None):
    flags = (0x8000 if csum else 0) | (0x2000 if key is not None else 0)
    h = struct.pack(">HH", flags, proto)
    if csum:
        h += b"\x00\x00\x00\x00"
    if key is not None:
        h += struct.pack(">I", key)
    return h + payload


def vxlan(inner_frame, flags=0x08, vni=0x1234):
    return struct.pack(">B3s3sB", flags, b"\0\0\0", vni.to_bytes(3, "big"), 0) + inner_frame


def geneve(payload, proto=0x6558, opt_words=0, vni=0x42):
    return struct.pack(">BBH3sB", opt_words & 0x3f, 0, proto, vni.to_bytes(3, "big"), 0) + bytes(4 * opt_words) + payload


def ip4(payload, proto, src=0x14000001, dst=0x14000002):
    return synth.ipv4(payload, proto, src=src, dst=dst)


def ip6(payload, nh):
    return synth.ipv6(payload, nh)


def eth_inner(ip_pkt, v6=False, vlan=None):
    return synth.eth(ip_pkt, 0x86dd if v6 else 0x0800, vlan=vlan)


def scenarios(seed=0x5EED000A):
    rng = np.random.default_rng(seed)
    names = ["tunnel.example.com", "inner.test", "vxlan.example.org"]
    out = []

    def tls_ip(v6=False):
        ch = synth.client_hello(rng, ["chrome", "firefox", "safari", "openssl"][int(rng.integers(4))],
                                names[int(rng.integers(len(names)))])
        l4 = synth.tcp(ch, sport=int(rng.integers(1024, 65535)))
        return ip6(l4, 6) if v6 else ip4(l4, 6, src=0x0a000105, dst=0x5db8d822)

    def http_ip():
        return ip4(synth.tcp(synth.http_request(rng, "inner.test"), dport=80), 6)

    def syn_ip():
        return ip4(synth.tcp(b"", flags=0x02, opts=synth.syn_opts(rng, 1)), 6)

    def quic_ip():
        c = quic_synth.quic_client_hello(rng, "chrome", "quic.inner.test")
        q = quic_synth.initial(1, bytes(8), bytes(4), b"", 0, 1, quic_synth.f_crypto(0, c))
        return ip4(synth.udp(q, 50000, 443), 17)

    inners = [("tls", tls_ip), ("http", http_ip), ("syn", syn_ip), ("quic", quic_ip)]
    for name, fn in inners:
        out.append((f"gre-{name}", synth.eth(ip4(gre(fn()), 47))))
        out.append((f"gre-csum-{name}", synth.eth(ip4(gre(fn(), csum=True), 47))))
        out.append((f"gre-key-{name}", synth.eth(ip4(gre(fn(), key=7), 47))))
        out.append((f"gre-udp-{name}", synth.eth(ip4(synth.udp(gre(fn()), 40000, 4754), 17))))
        out.append((f"vxlan-{name}", synth.eth(ip4(synth.udp(vxlan(eth_inner(fn())), 40000, 4789), 17))))
        out.append((f"vxlan-vlan-{name}", synth.eth(ip4(synth.udp(vxlan(eth_inner(fn(), vlan=7)), 40000, 4789), 17))))
        out.append((f"vxlan-noflag-{name}", synth.eth(ip4(synth.udp(vxlan(eth_inner(fn()), flags=0), 40000, 4789), 17))))
        out.append((f"geneve-eth-{name}", synth.eth(ip4(synth.udp(geneve(eth_inner(fn())), 40000, 6081), 17))))
        out.append((f"geneve-ip-{name}", synth.eth(ip4(synth.udp(geneve(fn(), proto=0x0800, opt_words=2), 40000, 6081), 17))))
        out.append((f"geneve-lo-{name}", synth.eth(ip4(synth.udp(geneve(b"\x02\x00\x00\x00" + fn(), proto=0), 40000, 6081), 17))))
        out.append((f"ipip-gre-{name}", synth.eth(ip4(ip4(gre(fn()), 47), 4))))
        out.append((f"v6-gre-{name}", synth.eth(ip6(gre(fn(), proto=0x0800), 47), 0x86dd)))
    out.append(("gre-v6-inner", synth.eth(ip4(gre(tls_ip(v6=True), proto=0x86dd), 47))))
    out.append(("gre-teb", synth.eth(ip4(gre(eth_inner(tls_ip()), proto=0x6558), 47))))
    out.append(("vxlan-arp", synth.eth(ip4(synth.udp(vxlan(synth.eth(bytes(28), 0x0806)), 40000, 4789), 17))))
    out.append(("geneve-unknown", synth.eth(ip4(synth.udp(geneve(tls_ip(), proto=0x1234), 40000, 6081), 17))))
    out.append(("geneve-lo-osi", synth.eth(ip4(synth.udp(geneve(b"\x07\x00\x00\x00" + tls_ip(), proto=0), 40000, 6081), 17))))
    out.append(("vxlan-wrong-port", synth.eth(ip4(synth.udp(vxlan(eth_inner(tls_ip())), 40000, 4790), 17))))
    # stacks: GRE in VXLAN in Geneve in IP-in-IP ... (the reference stops after four)
    for depth in range(2, 7):
        p = tls_ip()
        for k in range(depth):
            kind = k % 4
            if kind == 0:
                p = ip4(gre(p), 47)
            elif kind == 1:
                p = ip4(synth.udp(vxlan(eth_inner(p)), 40000, 4789), 17)
            elif kind == 2:
                p = ip4(synth.udp(geneve(p, proto=0x0800), 40000, 6081), 17)
            else:
                p = ip4(p, 4)
        out.append((f"stack-{depth}", synth.eth(p)))
    # tunnel headers cut short at every byte
    full = synth.eth(ip4(synth.udp(vxlan(eth_inner(tls_ip())), 40000, 4789), 17))
    for cut in range(34 + 8, 34 + 8 + 8 + 14 + 2):
        out.append((f"vxlan-cut-{cut}", full[:cut]))
    full = synth.eth(ip4(gre(tls_ip(), csum=True), 47))
    for cut in range(34, 34 + 8 + 2):
        out.append((f"gre-cut-{cut}", full[:cut]))
    full = synth.eth(ip4(synth.udp(geneve(eth_inner(tls_ip()), opt_words=3), 40000, 6081), 17))
    for cut in range(42, 42 + 8 + 12 + 14 + 2):
        out.append((f"geneve-cut-{cut}", full[:cut]))
    return out
