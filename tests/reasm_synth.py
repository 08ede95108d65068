"""Synthetic TCP streams for the reassembly fixtures
(tests/golden/make_golden_reasm.py; test infrastructure, the expected values
come from the reference libmerc with "reassembly" configured).

Scenarios (process_tcp_data pkt_proc.cc:773-893, reassembly.hpp:140-520):
ClientHellos split into 2..6 segments in order, reordered, duplicated,
with partial / subset / superset overlaps, a missing middle segment, more than
20 segments, sequence numbers wrapping 2^32, continuing segments with
sequence number 0, several flows interleaved, IPv6 flows, a ClientHello
longer than the 8192-byte buffer, an oversized segment, a complete message in
the middle of a flow in reassembly; SSH banners followed by their KEXINIT in
later segments (indefinite SSH reassembly), split standalone KEXINITs;
TLS ServerHello + Certificate split; HTTP requests split (no reassembly).
"""
import struct

import numpy as np

from tests import synth


class Flow:
    def __init__(self, sport, dport=443, v6=False, seq=1000, src=0x0a000001, dst=0x0d59b21b):
        self.sport, self.dport, self.v6, self.seq0, self.src, self.dst = sport, dport, v6, seq, src, dst

    def pkt(self, data, off, seq=None, flags=0x18):
        s = (self.seq0 + off) & 0xffffffff if seq is None else seq
        l4 = synth.tcp(data, sport=self.sport, dport=self.dport, seq=s, flags=flags)
        if self.v6:
            return synth.eth(synth.ipv6(l4, 6), 0x86dd)
        return synth.eth(synth.ipv4(l4, 6, src=self.src, dst=self.dst))


def cuts(n, k, rng):
    c = sorted(set(int(x) for x in rng.integers(1, n, k - 1)))
    return [0] + c + [n]


def ssh_banner(comment=True):
    return b"SSH-2.0-OpenSSH_9.6" + (b" Ubuntu-3ubuntu13\r\n" if comment else b"\r\n")


def scenarios(seed=0x5EED000F):
    rng = np.random.default_rng(seed)
    out = []   # (label, frame)
    port = [40000]

    def flow(**kw):
        port[0] += 1
        return Flow(port[0], **kw)

    def ch(name="reasm.example.com", big=False):
        prof = ["chrome", "firefox", "safari", "openssl"][int(rng.integers(4))]
        return synth.client_hello(rng, prof, ("x" * 300 + ".") * 20 + "example.com" if big else name)

    def emit(label, f, parts, order=None, seqs=None):
        order = range(len(parts)) if order is None else order
        for j in order:
            data, off = parts[j]
            out.append((f"{label}.{j}", f.pkt(data, off, None if seqs is None else seqs[j])))

    def split(data, c):
        return [(data[c[k]:c[k + 1]], c[k]) for k in range(len(c) - 1)]

    # in order, 2..6 segments
    for k in range(2, 7):
        d = ch(big=False)
        emit(f"inorder{k}", flow(), split(d, cuts(len(d), k, rng)))
    # post-quantum sized hello (about 1.8 kB) over 2 MTU-sized segments
    d = synth.client_hello(rng, "chrome", "pq.example.com") + b""
    emit("pq", flow(), split(d, [0, min(1400, len(d) - 1), len(d)]))
    # reordered: later segments before the second
    d = ch(); c = cuts(len(d), 4, rng)
    emit("reorder", flow(), split(d, c), order=[0, 2, 1, 3])
    d = ch(); c = cuts(len(d), 3, rng)
    emit("first_late", flow(), split(d, c), order=[1, 0, 2])
    # duplicates and overlaps
    d = ch(); c = cuts(len(d), 3, rng); p = split(d, c)
    emit("dup", flow(), [p[0], p[1], p[1], p[2]])
    d = ch(); n = len(d)
    f = flow()
    emit("back_partial", f, [(d[:n // 2], 0), (d[n // 3:], n // 3)])
    d = ch(); n = len(d); f = flow()
    emit("back_subset", f, [(d[:n // 2], 0), (d[n // 4:n // 3], n // 4), (d[n // 2:], n // 2)])
    d = ch(); n = len(d); f = flow()
    emit("front_superset", f, [(d[:n // 4], 0), (d[n // 2:3 * n // 4], n // 2), (d[3 * n // 4:], 3 * n // 4),
                               (d[n // 4:n], n // 4)])
    d = ch(); n = len(d); f = flow()
    emit("front_partial", f, [(d[:n // 4], 0), (d[n // 2:], n // 2), (d[n // 4:n // 2 + 10], n // 4)])
    # a missing middle segment: never completes
    d = ch(); c = cuts(len(d), 4, rng); p = split(d, c)
    emit("missing", flow(), [p[0], p[2], p[3]])
    # more than 20 segments
    d = ch(); c = list(range(0, len(d), max(1, len(d) // 25))) + [len(d)]
    emit("maxseg", flow(), split(d, sorted(set(c))))
    # sequence numbers wrapping 2^32
    d = ch(); c = cuts(len(d), 3, rng)
    emit("wrap", flow(seq=0xffffff00), split(d, c))
    # continuing segments with sequence number 0 (in-order placement)
    d = ch(); c = cuts(len(d), 3, rng); p = split(d, c)
    f = flow()
    emit("seq0", f, p, seqs=[None, 0, 0])
    # interleaved flows
    fs = [flow() for _ in range(4)]
    ps = []
    for f in fs:
        d = ch(); ps.append(split(d, cuts(len(d), int(rng.integers(2, 5)), rng)))
    idx = [0] * 4
    while any(idx[k] < len(ps[k]) for k in range(4)):
        k = int(rng.integers(4))
        if idx[k] < len(ps[k]):
            data, off = ps[k][idx[k]]
            out.append((f"interleave{k}.{idx[k]}", fs[k].pkt(data, off)))
            idx[k] += 1
    # IPv6
    d = ch(); emit("v6", flow(v6=True), split(d, cuts(len(d), 3, rng)))
    # longer than the buffer: more > 8192 -> a truncated record, no reassembly
    d = ch(big=True); emit("big", flow(), split(d, [0, 1200, len(d)]))
    # a hello of about 7 kB (a padding extension), over five segments
    d = synth.client_hello(rng, "chrome", "y" * 200 + ".example.com")
    hs = bytearray(d[9:])                          # ClientHello body (after record + handshake headers)
    p = 2 + 32
    p += 1 + hs[p]                                 # session id
    p += 2 + struct.unpack(">H", hs[p:p + 2])[0]   # cipher suites
    p += 1 + hs[p]                                 # compression methods
    ext = struct.pack(">HH", 0x0015, 6000) + bytes(6000)
    el = struct.unpack(">H", hs[p:p + 2])[0]
    hs[p:p + 2] = struct.pack(">H", el + len(ext))
    hs += ext
    rec = b"\x16\x03\x01" + struct.pack(">H", len(hs) + 4) + b"\x01" + len(hs).to_bytes(3, "big") + bytes(hs)
    emit("padded6k", flow(), split(rec, [0, 1400, 2800, 4200, 5600, len(rec)]))
    # a complete hello in the middle of a flow in reassembly (on the same flow)
    d = ch(); c = cuts(len(d), 3, rng); p = split(d, c)
    f = flow()
    whole = ch("whole.example.com")
    out.append(("midwhole.0", f.pkt(p[0][0], 0)))
    out.append(("midwhole.x", f.pkt(whole, 5000)))
    out.append(("midwhole.1", f.pkt(p[1][0], p[1][1])))
    out.append(("midwhole.2", f.pkt(p[2][0], p[2][1])))
    # non-matching data on a flow not in reassembly, and ACKs with no data
    f = flow(); out.append(("junk", f.pkt(b"hello world, not a protocol", 0)))
    out.append(("ack", f.pkt(b"", 0, flags=0x10)))
    # SSH: banner, then KEXINIT in the next segment(s) (indefinite reassembly)
    for k, comment in enumerate((True, False)):
        f = flow(dport=22)
        kex = synth.ssh_kexinit(rng)
        out.append((f"ssh{k}.banner", f.pkt(ssh_banner(comment), 0)))
        bl = len(ssh_banner(comment))
        c = [0, len(kex) // 3, len(kex)]
        out.append((f"ssh{k}.kex0", f.pkt(kex[c[0]:c[1]], bl)))
        out.append((f"ssh{k}.kex1", f.pkt(kex[c[1]:], bl + c[1])))
    f = flow(dport=22)
    kex = synth.ssh_kexinit(rng)
    out.append(("sshkex.0", f.pkt(kex[:40], 0)))
    out.append(("sshkex.1", f.pkt(kex[40:], 40)))
    f = flow(dport=22)                                              # banner + partial KEXINIT together
    kex = synth.ssh_kexinit(rng)
    b = ssh_banner()
    out.append(("sshpart.0", f.pkt(b + kex[:50], 0)))
    out.append(("sshpart.1", f.pkt(kex[50:], len(b) + 50)))
    # TLS ServerHello + Certificate split over segments
    f = Flow(443, dport=port[0] + 1)
    port[0] += 1
    sh = synth.server_hello(rng, cert_bytes=3000)
    out.append(("sh.0", f.pkt(sh[:1000], 0)))
    out.append(("sh.1", f.pkt(sh[1000:2200], 1000)))
    out.append(("sh.2", f.pkt(sh[2200:], 2200)))
    # HTTP request split: the reference does not reassemble HTTP
    f = flow(dport=80)
    req = synth.http_request(rng, "split.example.org")
    out.append(("http.0", f.pkt(req[:40], 0)))
    out.append(("http.1", f.pkt(req[40:], 40)))
    # random streams: splits, drops, duplicates and reorderings
    for r in range(120):
        f = flow(seq=int(rng.integers(0, 1 << 32)), v6=bool(rng.random() < 0.2))
        d = ch()
        p = split(d, cuts(len(d), int(rng.integers(2, 6)), rng))
        order = list(range(len(p)))
        if rng.random() < 0.3:
            j = int(rng.integers(0, len(p) - 1)); order[j], order[j + 1] = order[j + 1], order[j]
        if rng.random() < 0.15:
            order.insert(int(rng.integers(0, len(order) + 1)), int(rng.integers(0, len(p))))
        if rng.random() < 0.1 and len(order) > 2:
            del order[int(rng.integers(1, len(order)))]
        for j in order:
            data, off = p[j]
            out.append((f"rand{r}.{j}", f.pkt(data, off)))
    return out


def timed_scenarios(seed=0x5EED0010, t0=1700000000):
    """A second stream with per-packet capture times (seconds), run by its own
    processor: flows that stall past the 15 s reassembly timeout
    (reassembly_flow_context::is_expired reassembly.hpp:307) and are reaped or
    continued, a time going backwards (the unsigned difference wraps), SYN /
    RST / FIN segments carrying data in the middle of a flow (skipped by the
    analysis_context path, pkt_proc.cc:1631-1633, fed to the flow by
    write_json), and non-TCP packets between segments
    (flow_state_pkts_needed keeps its value).  At most three flows are in
    reassembly at a time.  Returns [(label, frame, seconds)]."""
    rng = np.random.default_rng(seed)
    out = []
    port = [41000]
    t = [t0]

    def flow(**kw):
        port[0] += 1
        return Flow(port[0], **kw)

    def ch(name="timed.example.com"):
        prof = ["chrome", "firefox", "safari", "openssl"][int(rng.integers(4))]
        return synth.client_hello(rng, prof, name)

    def add(label, frame, dt=1):
        t[0] += dt
        out.append((label, frame, t[0]))

    def split(d, k):
        c = cuts(len(d), k, rng)
        return [(d[c[j]:c[j + 1]], c[j]) for j in range(len(c) - 1)]

    udp_pkt = synth.eth(synth.ipv4(synth.udp(b"\x12\x34" + bytes(30), 5353, 5353), 17))
    arp = bytes(12) + b"\x08\x06" + bytes(28)
    for r in range(6):
        # in time
        f = flow(); p = split(ch(), 3)
        for j, (d, o) in enumerate(p):
            add(f"ok{r}.{j}", f.pkt(d, o), dt=int(rng.integers(0, 7)))
        # a stall past the timeout before the last segment
        f = flow(); p = split(ch(), 3)
        add(f"stall{r}.0", f.pkt(*p[0]))
        add(f"stall{r}.1", f.pkt(*p[1]), dt=3)
        add(f"stall{r}.2", f.pkt(*p[2]), dt=15 + int(rng.integers(0, 5)))
        # exactly at / just under the timeout
        f = flow(); p = split(ch(), 2)
        add(f"edge{r}.0", f.pkt(*p[0]))
        add(f"edge{r}.1", f.pkt(*p[1]), dt=14 + (r & 1))
        # other traffic between segments (the analysis path's flag is sticky)
        f = flow(); p = split(ch(), 3)
        add(f"mix{r}.0", f.pkt(*p[0]))
        add(f"mix{r}.udp", udp_pkt)
        add(f"mix{r}.arp", arp)
        add(f"mix{r}.1", f.pkt(*p[1]))
        add(f"mix{r}.ack", f.pkt(b"", 0, flags=0x10))
        add(f"mix{r}.2", f.pkt(*p[2]))
        # control flags on data segments
        f = flow(); p = split(ch(), 4)
        add(f"ctl{r}.0", f.pkt(*p[0]))
        add(f"ctl{r}.rst", f.pkt(*p[1], flags=0x14 if r & 1 else 0x04))
        add(f"ctl{r}.2", f.pkt(*p[2]))
        add(f"ctl{r}.fin", f.pkt(*p[3], flags=0x19))
        f = flow(); p = split(ch(), 2)
        add(f"syn{r}.0", f.pkt(*p[0], flags=0x02 if r & 1 else 0x12))
        add(f"syn{r}.1", f.pkt(*p[1]))
        # an abandoned flow, then a new one on another port much later
        f = flow(); p = split(ch(), 3)
        add(f"abandon{r}.0", f.pkt(*p[0]))
        g = flow(); q = split(ch(), 2)
        add(f"later{r}.0", g.pkt(*q[0]), dt=30)
        add(f"later{r}.1", g.pkt(*q[1]))
        # the time going backwards inside a flow
        f = flow(); p = split(ch(), 2)
        add(f"back{r}.0", f.pkt(*p[0]))
        add(f"back{r}.1", f.pkt(*p[1]), dt=-5)
        t[0] += 10
    return out


def tunnel_scenarios(seed=0x5EED0011):
    """ClientHellos split over two or three TCP segments inside tunnels (IP-in-IP
    over IPv4 / IPv6, GRE, GRE over UDP, VXLAN, Geneve, two levels): the
    reassembled record keeps the completing packet's "encapsulations"
    (pkt_proc.cc:1231-1233).  Returns [(label, frame)]."""
    from tests import tunnel_synth as T
    rng = np.random.default_rng(seed)
    out = []

    def wrap(kind, inner_ip, v6_inner):
        eth_in = T.eth_inner(inner_ip, v6=v6_inner)
        if kind == "ipip4":
            return synth.eth(T.ip4(inner_ip, 41 if v6_inner else 4))
        if kind == "ipip6":
            return synth.eth(T.ip6(inner_ip, 41 if v6_inner else 4), 0x86dd)
        if kind == "gre":
            return synth.eth(T.ip4(T.gre(inner_ip, 0x86dd if v6_inner else 0x0800), 47))
        if kind == "gre_csum":
            return synth.eth(T.ip4(T.gre(inner_ip, 0x86dd if v6_inner else 0x0800, csum=True), 47))
        if kind == "gre_udp":
            return synth.eth(T.ip4(synth.udp(T.gre(inner_ip, 0x86dd if v6_inner else 0x0800), 50000, 4754), 17))
        if kind == "vxlan":
            return synth.eth(T.ip4(synth.udp(T.vxlan(eth_in), 50001, 4789), 17))
        if kind == "geneve":
            return synth.eth(T.ip4(synth.udp(T.geneve(eth_in), 50002, 6081), 17))
        if kind == "vxlan6":
            return synth.eth(T.ip6(synth.udp(T.vxlan(eth_in), 50001, 4789), 17), 0x86dd)
        if kind == "gre_in_ipip":
            return synth.eth(T.ip4(T.ip4(T.gre(inner_ip, 0x86dd if v6_inner else 0x0800), 47), 4))
        raise ValueError(kind)

    kinds = ["ipip4", "ipip6", "gre", "gre_csum", "gre_udp", "vxlan", "geneve", "vxlan6", "gre_in_ipip"]
    sport = 42000
    for r in range(2):
        for kind in kinds:
            sport += 1
            v6_inner = bool(r & 1)
            prof = ["chrome", "firefox", "safari", "openssl"][int(rng.integers(4))]
            d = synth.client_hello(rng, prof, f"{kind}.tunnel.example.com")
            c = cuts(len(d), 2 + (sport & 1), rng)
            for j in range(len(c) - 1):
                l4 = synth.tcp(d[c[j]:c[j + 1]], sport=sport, dport=443, seq=5000 + c[j])
                inner_ip = T.ip6(l4, 6) if v6_inner else T.ip4(l4, 6, src=0x0a000105, dst=0x5db8d822)
                out.append((f"tun_{kind}{r}.{j}", wrap(kind, inner_ip, v6_inner)))
    return out


def reap_scenarios(seed=0x5EED0018, t0=1700000000, n_active=10150, n_stall=64, n_new=8):
    """(phase, frame, capture time in seconds) for the reaping-order fixture
    (tests/golden/make_golden_reap.py): the flow table filled past its 10 000
    entries with ClientHellos whose first segment says more bytes follow
    (active_reap drops two flows per new one), their second segments (the
    survivors complete, active reaping goes on), then flows stalled past the
    15 s timeout reaped by passive_reap while new flows arrive, and the
    stalled flows' second segments."""
    rng = np.random.default_rng(seed)
    hello = synth.client_hello(rng, "openssl", "reap.example.com")
    cut = 60
    out = []

    def flow(k, sport_base):
        # distinct source addresses and ports: the flow keys spread over the buckets
        return Flow(sport_base + k % 20000, src=0x0a000000 + (k * 2654435761 & 0xffffff), dst=0x0d59b21b)

    flows = [flow(k, 20000) for k in range(n_active)]
    for f in flows:                                   # phase A: first segments
        out.append(("fill", f.pkt(hello[:cut], 0), t0))
    for f in flows:                                   # phase B: second segments
        out.append(("finish", f.pkt(hello[cut:], cut), t0 + 1))
    t1 = t0 + 100
    stalled = [flow(k + 500000, 30000) for k in range(n_stall)]
    cut2 = len(hello) - 8                             # a timed-out buffer still holds a ClientHello
    for f in stalled:                                 # phase C: flows that stall
        out.append(("stall", f.pkt(hello[:cut2], 0), t1))
    fresh = [flow(k + 900000, 40000) for k in range(n_new)]
    for f in fresh:                                   # phase D: new flows after the timeout (passive reaping)
        out.append(("new", f.pkt(hello[:cut], 0), t1 + 20))
    order = list(rng.permutation(n_stall))
    for j in order:                                   # phase E: the stalled flows' second segments
        out.append(("late", stalled[j].pkt(hello[cut2:], cut2), t1 + 21))
    for f in fresh:                                   # phase F: the new flows complete
        out.append(("done", f.pkt(hello[cut:], cut), t1 + 22))
    return out
