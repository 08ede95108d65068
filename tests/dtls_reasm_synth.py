"""Synthetic DTLS ClientHello fragment streams for the UDP offset-reassembly
fixtures (tests/golden/make_golden_dtls_reasm.py; test infrastructure, the
expected values come from the reference libmerc with "reassembly" configured).

Scenarios (process_udp_offset_reassembly reassembly.hpp:1036-1100 over the
tcp_reassembler's flow table): ClientHellos whose handshake message is split
into 2..6 fragments (one per datagram) in order, reordered, duplicated,
overlapping, with a missing middle fragment, a later fragment arriving first,
several flows interleaved, a second message_seq on a 5-tuple in reassembly
(the connection-id mismatch), IPv6, a long ClientHello, messages larger than
the 8192-byte buffer, whole ClientHellos in between, and a timed stream whose
flows stall past the 15 s timeout.
"""
import struct

import numpy as np

from tests import synth


def hello_body(rng, name):
    """A DTLS ClientHello's handshake body (synth.dtls_client_hello without headers)."""
    rec = synth.dtls_client_hello(rng, name)
    return rec[13 + 12:]


def fragment(body, off, ln, mseq=0, total=None, rseq=0):
    """One datagram payload: a DTLS record holding the handshake fragment body[off:off+ln]."""
    total = len(body) if total is None else total
    piece = body[off:off + ln]
    hs = (b"\x01" + struct.pack(">I", total)[1:] + struct.pack(">H", mseq) + struct.pack(">I", off)[1:] +
          struct.pack(">I", len(piece))[1:] + piece)
    return struct.pack(">BHH", 0x16, 0xfefd, 0) + struct.pack(">Q", rseq)[2:] + struct.pack(">H", len(hs)) + hs


class Flow:
    def __init__(self, sport, dport=443, v6=False, src=0x0a000001, dst=0x0d59b21b):
        self.sport, self.dport, self.v6, self.src, self.dst = sport, dport, v6, src, dst

    def pkt(self, payload):
        l4 = synth.udp(payload, sport=self.sport, dport=self.dport)
        if self.v6:
            return synth.eth(synth.ipv6(l4, 17), 0x86dd)
        return synth.eth(synth.ipv4(l4, 17, src=self.src, dst=self.dst))


def cuts(n, k, rng):
    c = sorted(set(int(x) for x in rng.integers(1, n, k - 1)))
    return [0] + c + [n]


def scenarios(seed=0x5EED0014):
    rng = np.random.default_rng(seed)
    out = []   # (label, frame)
    port = [45000]

    def flow(**kw):
        port[0] += 1
        return Flow(port[0], **kw)

    def parts(body, k):
        c = cuts(len(body), k, rng)
        return [(c[j], c[j + 1] - c[j]) for j in range(len(c) - 1)]

    def emit(label, f, body, ps, order=None, mseq=0):
        order = range(len(ps)) if order is None else order
        for j in order:
            off, ln = ps[j]
            out.append((f"{label}.{j}", f.pkt(fragment(body, off, ln, mseq=mseq, rseq=j))))

    names = ["dtls.example.com", "webrtc.example.org", "a.b.example.net", "voip.example.com"]
    for rep in range(6):
        for k in (2, 3, 4, 6):
            body = hello_body(rng, names[(rep + k) % len(names)])
            f = flow()
            ps = parts(body, k)
            emit(f"inorder{k}.{rep}", f, body, ps)
            body = hello_body(rng, names[rep % len(names)])
            f = flow()
            ps = parts(body, k)
            order = list(rng.permutation(len(ps)))
            if order[0] != 0 and rep % 2 == 0:               # keep some with the first fragment first
                order.remove(0)
                order.insert(0, 0)
            emit(f"perm{k}.{rep}", f, body, ps, order=order)
    for rep in range(4):
        body = hello_body(rng, names[rep])
        f = flow()
        ps = parts(body, 3)
        emit(f"dup.{rep}", f, body, ps, order=[0, 1, 1, 2])
        body = hello_body(rng, names[rep])
        f = flow()
        n = len(body)
        ov = [(0, n // 2), (n // 3, n // 2), (n // 2 + 5, n - n // 2 - 5)]
        emit(f"overlap.{rep}", f, body, ov)
        body = hello_body(rng, names[rep])
        f = flow()
        ps = parts(body, 4)
        emit(f"missing.{rep}", f, body, ps, order=[0, 1, 3])   # never completes
        body = hello_body(rng, names[rep])
        f = flow()
        ps = parts(body, 3)
        emit(f"later_first.{rep}", f, body, ps, order=[2, 0, 1])
    # interleaved flows
    fl = [flow() for _ in range(3)]
    bodies = [hello_body(rng, names[j]) for j in range(3)]
    pss = [parts(b, 3) for b in bodies]
    for j in range(3):
        for q in range(3):
            off, ln = pss[q][j]
            out.append((f"interleave{q}.{j}", fl[q].pkt(fragment(bodies[q], off, ln, rseq=j))))
    # a second message_seq while the first is in reassembly, then the rest of both
    f = flow()
    b0, b1 = hello_body(rng, names[0]), hello_body(rng, names[1])
    p0, p1 = parts(b0, 2), parts(b1, 2)
    out.append(("cid.0", f.pkt(fragment(b0, *p0[0], mseq=0))))
    out.append(("cid.1", f.pkt(fragment(b1, *p1[0], mseq=1))))
    out.append(("cid.2", f.pkt(fragment(b1, *p1[1], mseq=1))))
    out.append(("cid.3", f.pkt(fragment(b0, *p0[1], mseq=0))))
    # IPv6
    for rep in range(3):
        body = hello_body(rng, names[rep])
        emit(f"v6.{rep}", flow(v6=True), body, parts(body, 3))
    # a long ClientHello (long server name) in 4..6 fragments
    for rep in range(3):
        body = hello_body(rng, ("y" * 60 + ".") * 30 + "example.com")
        emit(f"long.{rep}", flow(), body, parts(body, 4 + rep))
    # whole ClientHellos between fragments of a flow in reassembly
    f, g = flow(), flow()
    body = hello_body(rng, names[2])
    ps = parts(body, 2)
    out.append(("mid.0", f.pkt(fragment(body, *ps[0]))))
    whole = hello_body(rng, names[3])
    out.append(("mid.whole", g.pkt(fragment(whole, 0, len(whole)))))
    out.append(("mid.1", f.pkt(fragment(body, *ps[1]))))
    # beyond the buffer: a message length over 8192, and a fragment + rest over 8192
    body = hello_body(rng, names[0])
    out.append(("big.total", flow().pkt(fragment(body, 0, 300, total=9000))))
    f = flow()
    out.append(("big.rest", f.pkt(fragment(body, 0, 300, total=8100))))
    out.append(("big.rest2", f.pkt(fragment(body, 300, 200, total=8100))))
    # fragment_length beyond the datagram (the body does not parse)
    f = flow()
    fr = bytearray(fragment(body, 0, 200))
    fr[13 + 9:13 + 12] = struct.pack(">I", 5000)[1:]
    out.append(("badlen.0", f.pkt(bytes(fr))))
    return out


def timed_scenarios(seed=0x5EED0015, t0=1700000000):
    """(label, frame, capture time in seconds): flows that stall past the timeout."""
    rng = np.random.default_rng(seed)
    out = []
    port = [47000]
    t = [t0]

    def add(label, frame, dt=1):
        t[0] += dt
        out.append((label, frame, t[0]))

    for rep in range(4):
        port[0] += 1
        f = Flow(port[0])
        body = hello_body(rng, "timed.example.com")
        c = [0, len(body) // 3, 2 * len(body) // 3, len(body)]
        add(f"stall.{rep}.0", f.pkt(fragment(body, c[0], c[1] - c[0])))
        add(f"stall.{rep}.1", f.pkt(fragment(body, c[1], c[2] - c[1])), dt=16 if rep % 2 == 0 else 3)
        add(f"stall.{rep}.2", f.pkt(fragment(body, c[2], c[3] - c[2])))
    return out
