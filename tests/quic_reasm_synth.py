"""Synthetic QUIC Initial streams whose ClientHello spans several datagrams,
for the QUIC CRYPTO-frame reassembly fixtures
(tests/golden/make_golden_quic_reasm.py; test infrastructure, the expected
values come from the reference libmerc with "reassembly" configured).

Scenarios (process_quic_reassembly reassembly.hpp:895-1033 over the
tcp_reassembler's flow table): ClientHellos of 2-7 KB (post-quantum sized key
shares) sent as 2..6 Initials of one connection, in order, reordered, with the
first datagram last; each datagram's part in one CRYPTO frame or several
(shuffled, with PING / PADDING / ACK between), with a gap inside a datagram
(the missing-frames path, a first frame shorter than 10 bytes), duplicated
datagrams, overlapping parts, a lost datagram, two connections (DCIDs) on one
5-tuple, interleaved 5-tuples, IPv6, QUIC v2, draft versions, unprotected
("already decrypted") Initials, ClientHellos beyond the 8 KiB buffer, a whole
Initial on a 5-tuple in reassembly, and a timed stream whose connections stall
past the 15 s timeout.
"""
import numpy as np

from tests import quic_synth as qs
from tests import synth

NAMES = ["pq.example.com", "video.example.net", "a.b.example.org", "h3.service.test"]


class Conn:
    """One client connection: a 5-tuple, a version and a DCID/SCID."""

    def __init__(self, rng, sport, version=1, v6=False, dcid_len=8, scid_len=5):
        self.sport, self.version, self.v6 = sport, version, v6
        self.dcid = bytes(rng.integers(0, 256, dcid_len, dtype=np.uint8))
        self.scid = bytes(rng.integers(0, 256, scid_len, dtype=np.uint8))
        self.pn = 0

    def datagram(self, frames, protect=True, min_size=1200, dcid=None):
        self.pn += 1
        first = 0xd0 if qs.VERSIONS.get(self.version, ("v1", False))[1] else 0xc0
        q = qs.initial(self.version, self.dcid if dcid is None else dcid, self.scid, b"", self.pn, 2, frames,
                       first=first, protect=protect, min_size=min_size)
        return synth.frame(synth.udp(q, self.sport, 443), 17, self.v6)


def big_hello(rng, size, name=None, profile="chrome"):
    """A QUIC ClientHello (handshake header + body) of about `size` bytes."""
    base = qs.quic_client_hello(rng, profile, name or NAMES[int(rng.integers(len(NAMES)))])
    pad = max(0, size - len(base) - 4)
    return qs.quic_client_hello(rng, profile, name or NAMES[int(rng.integers(len(NAMES)))], pad=pad)


def parts(n, k, rng, cap=1050):
    """k contiguous (offset, length) parts covering [0, n): an even split with
    jittered cuts, each part at most cap bytes."""
    k = max(k, -(-n // cap))
    step = n / k
    j = int(min(100, step / 4))
    cuts = [int(round(step * x)) + (int(rng.integers(-j, j + 1)) if j else 0) for x in range(1, k)]
    bounds = [0] + cuts + [n]
    ps = [(bounds[x], bounds[x + 1] - bounds[x]) for x in range(k)]
    assert all(0 < ln for _, ln in ps)
    return ps


def crypto(ch, off, ln):
    return qs.f_crypto(off, ch[off:off + ln])


def scenarios(seed=0x5EED0016):
    rng = np.random.default_rng(seed)
    out = []
    port = [52000]

    def conn(**kw):
        port[0] += 1
        return Conn(rng, port[0], **kw)

    def emit(label, c, frames_list, order=None, **kw):
        order = range(len(frames_list)) if order is None else order
        for j in order:
            out.append((f"{label}.{j}", c.datagram(frames_list[j], **kw)))

    for rep in range(4):
        for k in (2, 3, 4):
            ch = big_hello(rng, 900 * k + int(rng.integers(0, 400)))
            c = conn()
            emit(f"inorder{k}.{rep}", c, [crypto(ch, o, l) for o, l in parts(len(ch), k, rng)])
            ch = big_hello(rng, 900 * k + int(rng.integers(0, 400)))
            c = conn()
            fl = [crypto(ch, o, l) for o, l in parts(len(ch), k, rng)]
            order = list(rng.permutation(k))
            emit(f"perm{k}.{rep}", c, fl, order=order)
        # the first datagram last
        ch = big_hello(rng, 2400)
        c = conn()
        fl = [crypto(ch, o, l) for o, l in parts(len(ch), 3, rng)]
        emit(f"first_last.{rep}", c, fl, order=[1, 2, 0])
        # several CRYPTO frames per datagram, shuffled, with other frames between
        ch = big_hello(rng, 3000)
        c = conn()
        fl = []
        for o, l in parts(len(ch), 3, rng):
            sub = parts(l, 3, rng, cap=l)
            pieces = [crypto(ch, o + so, sl) for so, sl in sub]
            rng.shuffle(pieces)
            fr = b""
            for k2, p in enumerate(pieces):
                fr += p + [qs.f_ping(), qs.f_padding(2), qs.f_ack(), b""][(k2 + rep) % 4]
            fl.append(fr)
        emit(f"multi.{rep}", c, fl)
        # a gap inside the first datagram (missing frames), filled by the second
        ch = big_hello(rng, 2000)
        c = conn()
        a, b = 300 + 20 * rep, 700 + 30 * rep
        emit(f"gap.{rep}", c, [crypto(ch, 0, a) + crypto(ch, b, 1000 - b),
                               crypto(ch, a, b - a) + crypto(ch, 1000, len(ch) - 1000)])
        # a first frame shorter than 10 bytes (min_crypto_data)
        ch = big_hello(rng, 2000)
        c = conn()
        s0 = 4 + rep
        emit(f"short_first.{rep}", c, [crypto(ch, 0, s0) + crypto(ch, 40, 900),
                                       crypto(ch, s0, 40 - s0) + crypto(ch, 940, len(ch) - 940)])
        # the missing-frames path without the first frame in the first datagram
        ch = big_hello(rng, 2000)
        c = conn()
        emit(f"gap_nofirst.{rep}", c, [crypto(ch, 500, 300) + crypto(ch, 900, 200),
                                       crypto(ch, 0, 500) + crypto(ch, 800, 100) + crypto(ch, 1100, len(ch) - 1100)])
        # a duplicated datagram
        ch = big_hello(rng, 2600)
        c = conn()
        fl = [crypto(ch, o, l) for o, l in parts(len(ch), 3, rng)]
        emit(f"dup.{rep}", c, fl, order=[0, 1, 1, 2])
        # overlapping parts
        ch = big_hello(rng, 2200)
        c = conn()
        n = len(ch)
        emit(f"overlap.{rep}", c, [crypto(ch, 0, 1000), crypto(ch, 800, 900), crypto(ch, 1600, n - 1600)])
        # a lost datagram: never completes
        ch = big_hello(rng, 2600)
        c = conn()
        fl = [crypto(ch, o, l) for o, l in parts(len(ch), 3, rng)]
        emit(f"lost.{rep}", c, fl, order=[0, 2])
    # two connections on one 5-tuple: the second DCID while the first is in reassembly
    c = conn()
    ch0, ch1 = big_hello(rng, 2000), big_hello(rng, 2000)
    p0, p1 = parts(len(ch0), 2, rng), parts(len(ch1), 2, rng)
    other = bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    out.append(("cid.0", c.datagram(crypto(ch0, *p0[0]))))
    out.append(("cid.1", c.datagram(crypto(ch1, *p1[0]), dcid=other)))
    out.append(("cid.2", c.datagram(crypto(ch1, *p1[1]), dcid=other)))
    out.append(("cid.3", c.datagram(crypto(ch0, *p0[1]))))
    # interleaved 5-tuples
    cs = [conn() for _ in range(3)]
    chs = [big_hello(rng, 2500) for _ in range(3)]
    pss = [parts(len(x), 3, rng) for x in chs]
    for j in range(3):
        for q in range(3):
            out.append((f"interleave{q}.{j}", cs[q].datagram(crypto(chs[q], *pss[q][j]))))
    # IPv6, QUIC v2, drafts, empty DCID
    for lab, kw in (("v6", {"v6": True}), ("v2", {"version": 0x6b3343cf}), ("d29", {"version": 0xff00001d}),
                    ("mvfst", {"version": 0xfaceb002}), ("nodcid", {"dcid_len": 0})):
        ch = big_hello(rng, 2300)
        c = conn(**kw)
        emit(f"{lab}", c, [crypto(ch, o, l) for o, l in parts(len(ch), 3, rng)])
    # unprotected ("already decrypted") Initials
    for rep in range(2):
        ch = big_hello(rng, 2000)
        c = conn()
        emit(f"plain.{rep}", c, [crypto(ch, o, l) for o, l in parts(len(ch), 2, rng)], protect=False)
    # a whole Initial on the 5-tuple while it is in reassembly (same connection)
    c = conn()
    ch = big_hello(rng, 2000)
    p = parts(len(ch), 2, rng)
    small = qs.quic_client_hello(rng, "firefox", NAMES[0])
    out.append(("whole_mid.0", c.datagram(crypto(ch, *p[0]))))
    out.append(("whole_mid.w", c.datagram(qs.f_crypto(0, small))))
    out.append(("whole_mid.1", c.datagram(crypto(ch, *p[1]))))
    # beyond the buffer: a ClientHello over 8192 bytes, and one whose first
    # datagram plus the rest exceed it
    for lab, size in (("huge", 9500), ("edge", 8150)):
        ch = big_hello(rng, size)
        c = conn()
        ps = parts(len(ch), len(ch) // 900 + 1, rng)
        emit(lab, c, [crypto(ch, o, l) for o, l in ps])
    return out


def _vli(b, p):
    if p >= len(b):
        return None, p
    n = 1 << (b[p] >> 6)
    if p + n > len(b):
        return None, p
    v = b[p] & 0x3f
    for k in range(1, n):
        v = v * 256 + b[p + k]
    return v, p + n


def _strict_crypto_writes(raw):
    """quic_init_decry::parse (quic.h:1369-1390) over raw bytes: the CRYPTO
    frames it writes into the buffer (extend: within 8 KiB) before it fails,
    and whether it failed."""
    p, writes = 0, []
    while p < len(raw):
        t = raw[p]
        p += 1
        data = None
        if t == 0x06:
            off, p = _vli(raw, p)
            ln, p = _vli(raw, p) if off is not None else (None, p)
            if ln is None or p + ln > len(raw):
                return writes, True
            data, p = (off, raw[p:p + ln]), p + ln
        elif t == 0x1c:
            for _ in range(2):
                v, p = _vli(raw, p)
                if v is None:
                    return writes, True
            rl, p = _vli(raw, p)
            if rl is None or p + rl > len(raw):
                return writes, True
            p += rl
        elif t in (0x02, 0x03):
            return writes, True           # (an ACK in ciphertext: skipped by the search)
        elif t not in (0x00, 0x01):
            return writes, True
        if data and data[1] and data[0] <= 8192 and data[0] + len(data[1]) <= 8192:
            writes.append(data)
    return writes, False


def stale_scenarios(seed=0x5EED0C0C, n=3, gap=(60, 70)):
    """Initials whose crypto buffer shows the bytes of the failed
    already-decrypted parse (quic.h:1513-1528: crypto_buffer.reset() keeps
    the bytes): the protected first byte's reserved bits are zero, the
    ciphertext read as frames writes a CRYPTO frame over [gap), the decrypted
    frames cover [0, 970) but that gap, overlapping so the frame check sees
    no missing frame (total == span, quic.h:1267-1272); a second datagram
    completes the ClientHello.  Found by searching DCIDs."""
    rng = np.random.default_rng(seed)
    out = []
    found = 0
    while found < n:
        ch = big_hello(rng, 2000)
        a, b = gap
        f1 = crypto(ch, 0, a - 20) + crypto(ch, a - 30, 30) + crypto(ch, b, 970 - b)
        for _ in range(400000):
            c = Conn(rng, 57000 + found)
            c.pn = int(rng.integers(0, 1000))
            q = qs.initial(c.version, c.dcid, c.scid, b"", c.pn + 1, 2, f1)
            if q[0] & 0x0c:
                continue
            hl = 1 + 4 + 1 + len(c.dcid) + 1 + len(c.scid) + 1 + 2
            raw = q[hl + (q[0] & 3) + 1:]
            writes, failed = _strict_crypto_writes(raw)
            if failed and any(o < b and o + len(d) > a for o, d in writes):
                break
        else:
            raise RuntimeError("no stale-byte Initial found")
        out.append((f"stale.{found}.0", c.datagram(f1)))
        out.append((f"stale.{found}.1", c.datagram(crypto(ch, 970, len(ch) - 970))))
        found += 1
    return out


def timed_scenarios(seed=0x5EED0017, t0=1700000000):
    """(label, frame, capture time in seconds): connections that stall past the timeout."""
    rng = np.random.default_rng(seed)
    out = []
    t = [t0]
    for rep in range(4):
        c = Conn(rng, 56000 + rep)
        ch = big_hello(rng, 2600)
        ps = parts(len(ch), 3, rng)
        for j, (o, l) in enumerate(ps):
            t[0] += (16 if rep % 2 == 0 else 3) if j == 1 else 1
            out.append((f"stall.{rep}.{j}", c.datagram(crypto(ch, o, l)), t[0]))
    return out
