"""Synthetic QUIC Initial packets for the QUIC parity fixtures (test
infrastructure; run in the dev container by tests/golden/make_golden_quic.py,
never on the GPU box).

Packets are protected as a QUIC client protects its Initial (RFC 9001 §5):
HKDF from the version's salt and the DCID (hashlib/hmac), AES-128-GCM and the
AES-ECB header-protection mask from the system libcrypto (ctypes).  The
scenarios cover what quic.h does with them: every version family of
quic_parameters (v1, v2, drafts, mvfst), DCID/SCID/token lengths, 1-4 byte
packet numbers, CRYPTO frames split and reordered with PADDING / PING / ACK /
ACK_ECN / CONNECTION_CLOSE in between, missing CRYPTO ranges (the first-frame
and first-10-bytes paths), offsets past the 8 KiB buffer, unknown frame types,
bad tags, reserved bits, non-Initial long headers, unprotected ("already
decrypted") Initials, short packets and ClientHellos larger than a packet.
"""
import ctypes
import hashlib
import hmac
import struct

import numpy as np

from tests import synth

_lib = ctypes.CDLL("libcrypto.so.3")
_lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_lib.EVP_aes_128_gcm.restype = ctypes.c_void_p
_lib.EVP_aes_128_ecb.restype = ctypes.c_void_p
for _f in ("EVP_EncryptInit_ex", "EVP_EncryptUpdate", "EVP_EncryptFinal_ex", "EVP_CIPHER_CTX_ctrl",
           "EVP_CIPHER_CTX_set_padding"):
    getattr(_lib, _f).restype = ctypes.c_int
_lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
_lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                   ctypes.c_int]
_lib.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
_lib.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
_lib.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
EVP_CTRL_GCM_GET_TAG = 0x10


def aes_ecb(key, block):
    c = _lib.EVP_CIPHER_CTX_new()
    out = ctypes.create_string_buffer(32)
    n = ctypes.c_int(0)
    _lib.EVP_EncryptInit_ex(c, _lib.EVP_aes_128_ecb(), None, key, None)
    _lib.EVP_CIPHER_CTX_set_padding(c, 0)
    _lib.EVP_EncryptUpdate(c, out, ctypes.byref(n), block, 16)
    _lib.EVP_CIPHER_CTX_free(c)
    return out.raw[:16]


def aes_gcm_seal(key, iv, aad, pt):
    c = _lib.EVP_CIPHER_CTX_new()
    out = ctypes.create_string_buffer(len(pt) + 32)
    tag = ctypes.create_string_buffer(16)
    n = ctypes.c_int(0)
    _lib.EVP_EncryptInit_ex(c, _lib.EVP_aes_128_gcm(), None, None, None)
    _lib.EVP_EncryptInit_ex(c, None, None, key, iv)
    _lib.EVP_EncryptUpdate(c, None, ctypes.byref(n), aad, len(aad))
    _lib.EVP_EncryptUpdate(c, out, ctypes.byref(n), pt, len(pt))
    k = n.value
    _lib.EVP_EncryptFinal_ex(c, ctypes.cast(ctypes.addressof(out) + k, ctypes.c_char_p), ctypes.byref(n))
    _lib.EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag)
    _lib.EVP_CIPHER_CTX_free(c)
    return out.raw[:len(pt)] + tag.raw


SALTS = {
    "d22": "7fbcdb0e7c66bbe9193a96cd21519ebd7a02644a", "d23": "c3eef712c72ebb5a11a7d2432bb46365bef9f502",
    "d29": "afbfec289993d24c9e9786f19c6111e04390a899", "v1": "38762cf7f55934b34d179ae6a4c80cadccbb7f0a",
    "v2d": "a707c203a59b47184a1d62ca570406ea7ae3e5d3", "v2": "0dede3def700a6db819381be6e269dcbf9bd2ed9",
}
VERSIONS = {   # version -> (salt, v2 labels / packet type bits)   quic.h:695-721
    0x00000001: ("v1", False), 0x6b3343cf: ("v2", True), 0x709a50c4: ("v2d", True), 0xff00001d: ("d29", False),
    0xff000020: ("d29", False), 0xff00001b: ("d23", False), 0xff000016: ("d22", False), 0xfaceb001: ("d22", False),
    0xfaceb002: ("d23", False), 0xfacefeed: ("v1", False), 0xff000022: ("v1", False), 0xd4000400: ("v1", False),
}


def hkdf_label(secret, label, length):
    info = struct.pack(">HB", length, len(label)) + label + b"\x00"
    return hmac.new(secret, info + b"\x01", hashlib.sha256).digest()[:length]


def initial_keys(version, dcid):
    salt, v2 = VERSIONS.get(version, ("v1", False))
    init = hmac.new(bytes.fromhex(SALTS[salt]), dcid, hashlib.sha256).digest()
    cs = hkdf_label(init, b"tls13 client in", 32)
    p = b"tls13 quicv2 " if v2 else b"tls13 quic "
    return hkdf_label(cs, p + b"key", 16), hkdf_label(cs, p + b"iv", 12), hkdf_label(cs, p + b"hp", 16)


def vli(v):
    if v < 0x40:
        return bytes([v])
    if v < 0x4000:
        return struct.pack(">H", 0x4000 | v)
    if v < 0x40000000:
        return struct.pack(">I", 0x80000000 | v)
    return struct.pack(">Q", 0xc000000000000000 | v)


# ---- frames
def f_crypto(off, data):
    return b"\x06" + vli(off) + vli(len(data)) + data


def f_padding(n):
    return b"\x00" * n


def f_ping():
    return b"\x01"


def f_ack(largest=3, delay=25, ranges=((1, 2),), first=1, ecn=None):
    b = (b"\x03" if ecn else b"\x02") + vli(largest) + vli(delay) + vli(len(ranges)) + vli(first)
    for g, l in ranges:
        b += vli(g) + vli(l)
    if ecn:
        b += b"".join(vli(x) for x in ecn)
    return b


def f_close(code=0x0a, ftype=0x06, reason=b"bad"):
    return b"\x1c" + vli(code) + vli(ftype) + vli(len(reason)) + reason


# ---- ClientHellos as QUIC clients send them (no record layer)
def tp_ext(params, draft=False):
    body = b"".join(vli(i) + vli(len(v)) + v for i, v in params)
    return synth.ext(0xffa5 if draft else 0x39, body)


def quic_client_hello(rng, profile, sni, ua=None, draft_tp=False, pad=0):
    g = [int(x) for x in rng.choice(synth.GREASE, 3, replace=False)]
    params = [(0x01, vli(30000)), (0x03, vli(1472)), (0x04, vli(15728640)), (0x05, vli(6291456)),
              (0x06, vli(6291456)), (0x07, vli(6291456)), (0x08, vli(100)), (0x09, vli(103)),
              (0x0f, bytes(rng.integers(0, 256, 8, dtype=np.uint8)))]
    if profile == "chrome":
        params += [(31 * int(rng.integers(1, 1000)) + 27, b""), (0x20, vli(65536)), (0x6ab2, b"\x00\x00\x00\x01"),
                   (0x4752, b"")]
    if ua is not None:
        params.append((0x3129, ua.encode()))
    rng.shuffle(params)
    ciphers = ([g[0]] if profile == "chrome" else []) + [0x1301, 0x1302, 0x1303]
    exts = [synth.sni_ext(sni), synth.alpn_ext(("h3",) if profile != "draft" else ("h3-29",)),
            synth.groups_ext(([g[1]] if profile == "chrome" else []) + [0x001d, 0x0017, 0x0018]),
            synth.sigalgs_ext(synth.SIGALGS), synth.keyshare_ext([(0x001d, 32)]), synth.ext(45, b"\x01\x01"),
            synth.versions_ext([0x0304]), tp_ext(params, draft_tp)]
    if profile == "chrome":
        exts += [synth.ext(27, b"\x02\x00\x02"), synth.ext(17513, b"\x00\x03\x02h3"), synth.ext(g[2], b""),
                 synth.ext(65037, bytes(rng.integers(0, 256, 186, dtype=np.uint8)))]
        rng.shuffle(exts)
    if pad:
        exts.append(synth.ext(21, bytes(pad)))
    be = b"".join(exts)
    cs = b"".join(struct.pack(">H", c) for c in ciphers)
    body = struct.pack(">H", 0x0303) + bytes(rng.integers(0, 256, 32, dtype=np.uint8)) + b"\x00"
    body += struct.pack(">H", len(cs)) + cs + b"\x01\x00" + struct.pack(">H", len(be)) + be
    return b"\x01" + struct.pack(">I", len(body))[1:] + body


def initial(version, dcid, scid, token, pn, pnl, frames, first=0xc0, protect=True, min_size=1200, tag_flip=False,
            reserved=0, length_delta=0):
    """A client Initial: header + frames padded to min_size, protected unless
    protect=False.  first: the unprotected first byte's type bits (0xc0: v1
    Initial; v2 Initials are 0xd0)."""
    hdr = bytes([first | (reserved << 2) | (pnl - 1)]) + struct.pack(">I", version)
    hdr += bytes([len(dcid)]) + dcid + bytes([len(scid)]) + scid + vli(len(token)) + token
    payload = frames
    need = min_size - (len(hdr) + 2 + pnl + len(payload) + 16)
    if need > 0:
        payload += f_padding(need)
    length = pnl + len(payload) + 16 + length_delta
    hdr += struct.pack(">H", 0x4000 | length)
    pnb = pn.to_bytes(pnl, "big")
    if not protect:
        return hdr + pnb + payload + bytes(16)
    key, iv, hp = initial_keys(version, dcid)
    nonce = (int.from_bytes(iv, "big") ^ pn).to_bytes(12, "big")
    ct = aes_gcm_seal(key, nonce, hdr + pnb, payload)
    if tag_flip:
        ct = ct[:-1] + bytes([ct[-1] ^ 1])
    sample = ct[4 - pnl:20 - pnl]
    mask = aes_ecb(hp, sample)
    b0 = hdr[0] ^ (mask[0] & 0x0f)
    pn_prot = bytes(a ^ b for a, b in zip(pnb, mask[1:1 + pnl]))
    return bytes([b0]) + hdr[1:] + pn_prot + ct


def wrap(quic, rng, v6=False, sport=None, dport=443):
    sport = int(rng.integers(1024, 65535)) if sport is None else sport
    return synth.frame(synth.udp(quic, sport, dport), 17, v6)


def scenarios(seed=0x5EED0009, n_random=600):
    """(label, frame bytes) of every hand-built case plus n_random randomized
    Initials."""
    rng = np.random.default_rng(seed)
    out = []
    names = ["www.example.com", "cdn.video.example.net", "api.service.test", "quic.tech", "a.b.c.d.e.example.org"]

    def ch(profile="chrome", **kw):
        return quic_client_hello(rng, profile, names[int(rng.integers(len(names)))], **kw)

    def dc(n=8):
        return bytes(rng.integers(0, 256, n, dtype=np.uint8))

    # every version family, one plain CRYPTO frame
    for v in VERSIONS:
        first = 0xd0 if VERSIONS[v][1] else 0xc0
        out.append((f"version-{v:08x}", initial(v, dc(), dc(5), b"", 1, 1, f_crypto(0, ch()), first=first)))
    out.append(("unknown-version", initial(0x1a2a3a4a, dc(), dc(5), b"", 1, 1, f_crypto(0, ch()))))
    out.append(("gquic-q050", initial(0x51303530, dc(), dc(5), b"", 1, 1, f_crypto(0, ch()), protect=False)))
    # header fields
    for n in (0, 1, 4, 16, 20):
        out.append((f"dcid-{n}", initial(1, dc(n), dc(3), b"", 0, 1, f_crypto(0, ch()))))
    out.append(("dcid-21", initial(1, dc(21), b"", b"", 0, 1, f_crypto(0, ch()))))
    out.append(("scid-21", initial(1, dc(8), dc(21), b"", 0, 1, f_crypto(0, ch()))))
    for n in (0, 20, 300):
        out.append((f"token-{n}", initial(1, dc(), dc(), dc(n), 7, 2, f_crypto(0, ch()))))
    out.append(("token-aad-over-1k", initial(1, dc(), dc(), dc(1000), 7, 2, f_crypto(0, ch()), min_size=1400)))
    for pnl in (1, 2, 3, 4):
        out.append((f"pnlen-{pnl}", initial(1, dc(), dc(), b"", 0x1234567 & ((1 << (8 * pnl)) - 1), pnl,
                                            f_crypto(0, ch()))))
    # frame layouts
    c = ch()
    h = len(c) // 2
    out.append(("split-2-in-order", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c[:h]) + f_crypto(h, c[h:]))))
    out.append(("split-2-reversed", initial(1, dc(), dc(), b"", 0, 1, f_crypto(h, c[h:]) + f_crypto(0, c[:h]))))
    cuts = sorted(int(x) for x in rng.choice(np.arange(1, len(c)), 5, replace=False))
    pieces = [(a, c[a:b]) for a, b in zip([0] + cuts, cuts + [len(c)])]
    rng.shuffle(pieces)
    mixed = b""
    for k, (o, d) in enumerate(pieces):
        mixed += f_crypto(o, d) + [f_ping(), f_padding(3), f_ack(), f_ack(ecn=(1, 2, 3)), b""][k % 5]
    out.append(("chaos-6-pieces", initial(1, dc(), dc(), b"", 0, 1, mixed)))
    out.append(("ack-close-then-crypto", initial(1, dc(), dc(), b"", 0, 1, f_ack() + f_close() + f_crypto(0, ch()))))
    out.append(("overlap", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c[:h + 20]) + f_crypto(h, c[h:]))))
    out.append(("gap-missing", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c[:h]) + f_crypto(h + 10, c[h + 10:]))))
    out.append(("no-first-frame", initial(1, dc(), dc(), b"", 0, 1, f_crypto(40, c[40:h]) + f_crypto(h + 5, c[h + 5:]))))
    out.append(("first-frame-short", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c[:6]) + f_crypto(50, c[50:]))))
    out.append(("offset-past-8k", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c) + f_crypto(8190, b"abcdef"))))
    out.append(("offset-big", initial(1, dc(), dc(), b"", 0, 1, f_crypto(9000, b"x" * 10) + f_crypto(0, c))))
    out.append(("unknown-frame-mid", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c[:h]) + b"\x1e" + f_crypto(h, c[h:]))))
    out.append(("ack-range-count-big", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c) + b"\x02\x01\x01\x44\x00\x01")))
    out.append(("crypto-len-overrun", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, c) + b"\x06\x00\x44\x00abc")))
    out.append(("bad-tag", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), tag_flip=True)))
    out.append(("reserved-bits", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), reserved=2)))
    out.append(("handshake-type", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), first=0xe0)))
    out.append(("v2-with-v1-type", initial(0x6b3343cf, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), first=0xc0)))
    out.append(("short-1100", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), min_size=1100)))
    out.append(("length-too-long", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), length_delta=40)))
    out.append(("length-short", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), length_delta=-100)))
    out.append(("plaintext-initial", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), protect=False)))
    out.append(("plaintext-split", initial(1, dc(), dc(), b"", 0, 1, f_crypto(h, c[h:]) + f_ping() + f_crypto(0, c[:h]),
                                           protect=False)))
    out.append(("plaintext-bad-frame", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()) + b"\x30", protect=False)))
    out.append(("ua-param", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch(ua="Chrome/120.0.6099.71 Windows NT 10.0")))))
    out.append(("ua-draft-tp", initial(0xff00001d, dc(), dc(), b"", 0, 1,
                                       f_crypto(0, ch("draft", ua="quic-go/0.42", draft_tp=True)))))
    big = ch(pad=1600)
    out.append(("ch-over-one-packet", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, big[:1100]))))
    out.append(("ch-second-packet", initial(1, dc(), dc(), b"", 1, 1, f_crypto(1100, big[1100:]))))
    out.append(("pmtu-1350", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), min_size=1350)))
    out.append(("payload-over-2k", initial(1, dc(), dc(), b"", 0, 1, f_crypto(0, ch()), min_size=2300)))
    out.append(("not-quic-first-bit", synth.frame(synth.udp(b"\x40" + bytes(1300), 5000, 443), 17)))
    # randomized Initials
    profiles = ["chrome", "chrome", "firefox", "draft"]
    vers = list(VERSIONS)
    for k in range(n_random):
        v = vers[int(rng.integers(len(vers)))]
        prof = profiles[int(rng.integers(len(profiles)))]
        c = ch(prof, ua="agent/%d" % k if rng.random() < 0.3 else None, draft_tp=rng.random() < 0.2)
        nf = int(rng.integers(1, 5))
        cuts = sorted(int(x) for x in rng.choice(np.arange(1, len(c)), nf - 1, replace=False)) if nf > 1 else []
        pieces = [(a, c[a:b]) for a, b in zip([0] + cuts, cuts + [len(c)])]
        if rng.random() < 0.5:
            rng.shuffle(pieces)
        fr = b""
        for o, d in pieces:
            fr += f_crypto(o, d)
            if rng.random() < 0.3:
                fr += [f_ping(), f_padding(int(rng.integers(1, 9))), f_ack()][int(rng.integers(3))]
        pnl = int(rng.integers(1, 5))
        out.append((f"random-{k}", initial(v, dc(int(rng.integers(0, 21))), dc(int(rng.integers(0, 21))),
                                           dc(int(rng.integers(0, 60))) if rng.random() < 0.3 else b"",
                                           int(rng.integers(0, 1 << (8 * pnl))), pnl, fr,
                                           first=0xd0 if VERSIONS[v][1] else 0xc0,
                                           min_size=int(rng.choice([1200, 1250, 1350, 1452])))))
    return [(lab, wrap(q, rng, v6=bool(rng.random() < 0.2)) if not lab.startswith("not-quic") else q)
            for lab, q in out]
