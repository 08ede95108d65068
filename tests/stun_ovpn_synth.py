"""Synthetic STUN messages and OpenVPN-over-TCP segments for the fixtures of
tests/golden/make_golden_stun_ovpn.py (test infrastructure; the expected
values come from the reference libmerc run over these packets).

STUN (stun.h:323-1013): modern (magic cookie) and classic headers, every
message class, the fingerprinted attribute types (type only / type + length
+ value), SOFTWARE values, padding, truncated attributes, length fields that
do and do not match the UDP payload, classic messages with zero-heavy
transaction ids, unknown methods.

OpenVPN (openvpn.h:116-500): P_CONTROL_V1 records carrying a TLS ClientHello
in one record or split over several, with and without an HMAC (tls-auth) of
16..64 bytes, net_time, packet-id arrays, acks, hard resets, data opcodes,
unknown opcodes, ClientHellos over the 800-byte reassembly buffer, truncated
records.
"""
import struct

import numpy as np

from tests import synth

COOKIE = b"\x21\x12\xa4\x42"


def stun_attr(t, v, pad=True):
    b = struct.pack(">HH", t, len(v)) + v
    if pad:
        b += b"\0" * ((4 - len(v) % 4) % 4)
    return b


def stun_msg(mtype, attrs, tid=None, cookie=True, length=None):
    body = b"".join(attrs)
    if tid is None:
        tid = bytes(range(1, 13))
    hdr = struct.pack(">HH", mtype, len(body) if length is None else length) + (COOKIE if cookie else b"\x01\x02\x03\x04") + tid
    return hdr + body


def udp_frame(payload, sport=52380, dport=3478, v6=False):
    return synth.frame(synth.udp(payload, sport=sport, dport=dport), 17, v6=v6)


def ovpn_record(opcode, key=0, session=0x1122334455667788, hmac=b"", replay=1, net_time=None, ids=(),
                remote=0x8877665544332211, msg_id=None, data=b"", length=None):
    body = struct.pack(">B", (opcode << 3) | key) + struct.pack(">Q", session) + hmac + struct.pack(">I", replay)
    if net_time is not None:
        body += struct.pack(">I", net_time)
    body += struct.pack(">B", len(ids)) + b"".join(struct.pack(">I", x) for x in ids)
    if ids:
        body += struct.pack(">Q", remote)
    if msg_id is not None:
        body += struct.pack(">I", msg_id)
    body += data
    return struct.pack(">H", len(body) if length is None else length) + body


def tcp_frame(payload, sport=51089, dport=1194, v6=False):
    return synth.frame(synth.tcp(payload, sport=sport, dport=dport), 6, v6=v6)


SOFTWARE_ESCAPES = [b'quote " backslash \\ slash /', b"tab\tnewline\n ctl\x01 del\x7f", "ünïcode ✓ 😀".encode(),
                    b"\xff\xfe invalid", b"\xc0\x80 overlong", b"\xed\xa0\x80 surrogate", "\ue000 private".encode(),
                    b"x" * 505 + "é".encode(), b"x" * 504 + "é".encode(), b"x" * 511, b"x" * 512, b"nul\x00inside",
                    "😀".encode() * 42, "😀".encode() * 43, b"\xe2\x82", "€uro".encode()]


def stun_scenarios(rng):
    out = []
    sw = [b"libjingle", b"Coturn-4.5.2 'dan Eider'", b"WebRTC", b"x" * 37, "ünïcode".encode()]
    # SOFTWARE values the classifier sees through utf8_safe_string<512>
    # (stun.h:1024): JSON escapes, non-ASCII, invalid UTF-8 (null: empty user
    # agent), and the 511-byte bound around a \uXXXX escape
    sw += SOFTWARE_ESCAPES
    fp_types = [0x0006, 0x0008, 0x0020, 0x8007, 0x8008, 0x8022, 0x8028, 0xc003, 0xc057, 0xdaba]
    other = [0x0001, 0x0003, 0x0024, 0x0025, 0x8029, 0x802a, 0x000c, 0x000d, 0x0019, 0x0013, 0xc001]
    for cls in (0x0000, 0x0010, 0x0100, 0x0110):
        for method in (0x001, 0x003, 0x00a, 0x080, 0x0fff):
            mt = cls | (method & 0x0f) | ((method & 0x70) << 1) | ((method & 0xf80) << 2)
            out.append((f"cls{cls:x}.m{method:x}", udp_frame(stun_msg(mt, [stun_attr(0x0003, b"\0" * 4)]))))
    for t in fp_types + other + [0x8037, 0x8070]:
        v = bytes(rng.integers(0, 256, int(rng.integers(0, 13)), dtype=np.uint8))
        out.append((f"attr{t:04x}", udp_frame(stun_msg(0x0001, [stun_attr(t, v), stun_attr(0x8028, b"\x12\x34\x56\x78")]))))
    for i, s in enumerate(sw):
        out.append((f"software{i}", udp_frame(stun_msg(0x0001, [stun_attr(0x0006, b"user:pass"), stun_attr(0x8022, s),
                                                              stun_attr(0x8070, b"\0\0\0\x02"), stun_attr(0x8037, b"\x01\x02\x03\x04\x05")]))))
    # two SOFTWARE attributes: the last one is the classifier's
    out.append(("software2x", udp_frame(stun_msg(0x0001, [stun_attr(0x8022, b"first"), stun_attr(0x8022, b"second")]))))
    # responses: records, no fingerprint
    out.append(("resp.software", udp_frame(stun_msg(0x0101, [stun_attr(0x8022, b"server 1.0"), stun_attr(0x0020, b"\0\x01\xae\x8e\x21\x12\xa4\x43")]))))
    # classic STUN: zero-heavy transaction ids, empty bodies, unknown types
    for tid, name in ((bytes(16), "tid0"), (b"\x01" + bytes(15), "tid1"), (bytes(range(1, 17)), "tidok"),
                      (b"\0" + bytes(range(1, 16)), "tid_onezero")):
        for mt in (0x0001, 0x0101, 0x0002, 0x1401):
            out.append((f"classic.{name}.{mt:04x}.empty", udp_frame(struct.pack(">HH", mt, 0) + tid)))
            out.append((f"classic.{name}.{mt:04x}.attr", udp_frame(struct.pack(">HH", mt, 8) + tid + stun_attr(0x0001, b"\0\x01\x7f\x01"))))
    # malformed: body length not a multiple of 4, unpadded / truncated attributes
    out.append(("unpadded", udp_frame(stun_msg(0x0001, [stun_attr(0x8022, b"abc", pad=False)]))))
    out.append(("trunc.attr", udp_frame(stun_msg(0x0001, [stun_attr(0x0006, b"user"), struct.pack(">HH", 0x8022, 40) + b"short"]))))
    out.append(("len.mismatch", udp_frame(stun_msg(0x0001, [stun_attr(0x0006, b"user")], length=12))))
    out.append(("len.over", udp_frame(stun_msg(0x0001, [stun_attr(0x0006, b"user")], length=400))))
    out.append(("nocookie.unknown", udp_frame(stun_msg(0x0003, [stun_attr(0x0006, b"user")], cookie=False))))
    out.append(("ipv6", udp_frame(stun_msg(0x0001, [stun_attr(0x8022, b"v6 agent")]), v6=True)))
    out.append(("short15", udp_frame(b"\0\x01\0\0" + bytes(11))))
    # many attributes (long fingerprint)
    many = [stun_attr(0x8070, bytes(rng.integers(0, 256, 60, dtype=np.uint8))) for _ in range(60)]
    out.append(("many", udp_frame(stun_msg(0x0001, many))))
    # random requests
    for k in range(300):
        attrs = []
        for _ in range(int(rng.integers(0, 7))):
            t = int(rng.choice(fp_types + other + [0x8037, 0x8070]))
            attrs.append(stun_attr(t, bytes(rng.integers(0, 256, int(rng.integers(0, 24)), dtype=np.uint8))))
        mt = int(rng.choice([0x0001, 0x0011, 0x0003, 0x0101, 0x0111, 0x0009]))
        out.append((f"rand{k}", udp_frame(stun_msg(mt, attrs, tid=bytes(rng.integers(0, 256, 12, dtype=np.uint8)),
                                                   cookie=bool(rng.random() < 0.85)), sport=int(rng.integers(1024, 65535)),
                                          dport=int(rng.choice([3478, 19302, 443, 5349])))))
    return out


def ovpn_scenarios(rng):
    out = []
    ch = synth.client_hello(rng, "openssl", "vpn.example.com")
    ch2 = synth.client_hello(rng, "firefox", "")
    hm = {16: bytes(rng.integers(1, 256, 16, dtype=np.uint8)), 20: bytes(rng.integers(1, 256, 20, dtype=np.uint8)),
          32: bytes(rng.integers(1, 256, 32, dtype=np.uint8)), 64: bytes(rng.integers(1, 256, 64, dtype=np.uint8))}
    # the handshake of openvpn_tcp_single.pcap, then variants
    out.append(("reset.client", tcp_frame(ovpn_record(7, msg_id=0, session=0))))
    out.append(("reset.server", tcp_frame(ovpn_record(8, ids=(0,), msg_id=0, session=0), sport=1194, dport=51089)))
    out.append(("ack", tcp_frame(ovpn_record(5, ids=(0,), session=0))))
    out.append(("ctrl.ch", tcp_frame(ovpn_record(4, msg_id=1, data=ch, session=0))))
    for n, h in hm.items():
        out.append((f"ctrl.ch.hmac{n}", tcp_frame(ovpn_record(4, msg_id=1, data=ch, hmac=h, replay=1, net_time=0x5f000000))))
        out.append((f"ack.hmac{n}", tcp_frame(ovpn_record(5, ids=(3, 4), hmac=h, replay=2, net_time=0x5f000001))))
    out.append(("ctrl.ch.key3", tcp_frame(ovpn_record(4, key=3, msg_id=1, data=ch, session=0))))
    out.append(("ctrl.ch.ids", tcp_frame(ovpn_record(4, msg_id=1, ids=(7,), data=ch, session=0))))
    out.append(("ctrl.ch.nettime", tcp_frame(ovpn_record(4, msg_id=1, net_time=0x01020304, data=ch, session=0))))
    # ClientHello split over 2 and 3 records, with acks between
    for parts in (2, 3):
        cut = [len(ch) * k // parts for k in range(parts + 1)]
        recs = [ovpn_record(4, msg_id=1 + k, replay=3 + k, data=ch[cut[k]:cut[k + 1]], session=0) for k in range(parts)]
        out.append((f"split{parts}", tcp_frame(b"".join(recs))))
        out.append((f"split{parts}.ack", tcp_frame(recs[0] + ovpn_record(5, ids=(1,), session=0) + b"".join(recs[1:]))))
    # the hello past the 800-byte buffer (one record, and split)
    big = synth.client_hello(rng, "chrome", "a" * 200 + ".example.com")
    big = big + b""
    out.append(("big.one", tcp_frame(ovpn_record(4, msg_id=1, data=big + bytes(900 - len(big)) if len(big) < 900 else big, session=0))))
    out.append(("second.hello", tcp_frame(ovpn_record(4, msg_id=1, data=ch2, session=0))))
    # non-ClientHello data, data opcodes, unknown opcodes, truncation, wrong port
    out.append(("ctrl.junk", tcp_frame(ovpn_record(4, msg_id=1, data=b"\x17\x03\x03\x00\x10" + bytes(16), session=0))))
    out.append(("data.v2", tcp_frame(ovpn_record(9, session=0) + bytes(20))))
    out.append(("opcode.unknown", tcp_frame(ovpn_record(12, msg_id=1, session=0))))
    out.append(("opcode0", tcp_frame(ovpn_record(0, session=0))))
    rec = ovpn_record(4, msg_id=1, data=ch, session=0)
    for cut in (1, 2, 3, 10, 14, 18, 20, 40, len(rec) - 1):
        out.append((f"trunc{cut}", tcp_frame(rec[:cut])))
    out.append(("len.short", tcp_frame(ovpn_record(4, msg_id=1, data=ch, session=0, length=10))))
    out.append(("len.long", tcp_frame(ovpn_record(4, msg_id=1, data=ch, session=0, length=len(ch) + 400))))
    out.append(("port443", tcp_frame(ovpn_record(4, msg_id=1, data=ch, session=0), dport=443)))
    out.append(("ipv6", tcp_frame(ovpn_record(4, msg_id=1, data=ch, session=0), v6=True)))
    # random record streams
    for k in range(200):
        recs = []
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.choice([4, 5, 7, 8, 4, 9, 3]))
            h = hm[int(rng.choice([16, 20, 32, 64]))] if rng.random() < 0.4 else b""
            ids = tuple(int(x) for x in rng.integers(0, 9, int(rng.integers(0, 3))))
            d = ch[:int(rng.integers(0, len(ch) + 1))] if op == 4 else b""
            recs.append(ovpn_record(op, key=int(rng.integers(0, 8)) if rng.random() < 0.2 else 0, hmac=h,
                                    replay=int(rng.integers(0, 1 << 16)),
                                    net_time=int(rng.integers(1, 1 << 31)) if rng.random() < 0.4 else None, ids=ids,
                                    msg_id=int(rng.integers(0, 9)) if op not in (5, 9) else None, data=d,
                                    session=int(rng.integers(0, 1 << 62))))
        out.append((f"rand{k}", tcp_frame(b"".join(recs), sport=int(rng.integers(1024, 65535)))))
    return out


def scenarios(seed=0x5EED000B):
    rng = np.random.default_rng(seed)
    return stun_scenarios(rng) + ovpn_scenarios(rng)
