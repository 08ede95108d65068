"""Deterministic synthetic packet batches for parity tests and bench.py.

Workloads follow BASELINE.json / SURVEY.md section 8(d):
  * "tls_ch":  TLS ClientHello frames (seed 0x5EED0001), Eth/IPv4 (90 %) or
    IPv6 (10 %), TCP ACK|PSH, ephemeral src port -> 443, ClientHellos modelled
    on real client profiles (cipher lists, extension sets and orders, GREASE,
    key-share sizes, SNI from a Zipf-distributed name list, ALPN)
  * "mixed":   35 % TLS CH, 5 % TLS SH(+cert), 2 % DTLS CH, 20 % HTTP request,
    5 % HTTP response, 5 % SSH (init / init+KEXINIT / KEXINIT, both
    directions), 15 % TCP SYN, 3 % SYN-ACK, 10 % no-output packets (pure ACK,
    unknown TCP payload, DNS over UDP)  (seed 0x5EED0003)
A batch is built from a pool of templates; per packet the IP addresses, ports
and TLS client random are re-drawn with vectorised numpy writes.
"""
import struct

import numpy as np

from tests.pcaplib import DESC_DTYPE

# ---------------------------------------------------------------------------
# framing
# ---------------------------------------------------------------------------


def eth(payload, ethertype=0x0800, vlan=None):
    h = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb"
    if vlan is not None:
        h += struct.pack(">HH", 0x8100, vlan)
    return h + struct.pack(">H", ethertype) + payload


def ipv4(payload, proto, src=0x0a000001, dst=0x0d59b21b, ttl=64, ident=0x1234):
    tl = 20 + len(payload)
    return struct.pack(">BBHHHBBHII", 0x45, 0, tl, ident, 0x4000, ttl, proto, 0, src, dst) + payload


def ipv6(payload, nh, src=b"\x20\x01\x0d\xb8" + b"\x00" * 11 + b"\x01", dst=b"\x26\x07\xf8\xb0" + b"\x00" * 11 + b"\x02",
         hlim=64, flow=0):
    return struct.pack(">IHBB", (6 << 28) | flow, len(payload), nh, hlim) + src + dst + payload


def tcp(payload, sport=50000, dport=443, flags=0x18, seq=1000, ack=2000, win=0xfaf0, opts=b""):
    assert len(opts) % 4 == 0
    off = (20 + len(opts)) // 4
    return struct.pack(">HHIIBBHHH", sport, dport, seq, ack, off << 4, flags, win, 0, 0) + opts + payload


def udp(payload, sport=50000, dport=443):
    return struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload


def frame(l4, proto, v6=False):
    if v6:
        return eth(ipv6(l4, proto), 0x86dd)
    return eth(ipv4(l4, proto))


# ---------------------------------------------------------------------------
# TLS ClientHello profiles
# ---------------------------------------------------------------------------
GREASE = [0x0a0a + 0x1010 * i for i in range(16)]


def ext(t, body):
    return struct.pack(">HH", t, len(body)) + body


def sni_ext(name):
    n = name.encode()
    return ext(0, struct.pack(">HBH", len(n) + 3, 0, len(n)) + n)


def alpn_ext(protos):
    b = b"".join(bytes([len(p)]) + p.encode() for p in protos)
    return ext(16, struct.pack(">H", len(b)) + b)


def groups_ext(groups):
    return ext(10, struct.pack(">H", 2 * len(groups)) + b"".join(struct.pack(">H", g) for g in groups))


def versions_ext(vers):
    return ext(43, bytes([2 * len(vers)]) + b"".join(struct.pack(">H", v) for v in vers))


def sigalgs_ext(algs):
    return ext(13, struct.pack(">H", 2 * len(algs)) + b"".join(struct.pack(">H", a) for a in algs))


def keyshare_ext(shares):
    b = b"".join(struct.pack(">HH", g, n) + bytes(range(n % 256)) * (n // 256) + bytes(range(n % 256)) for g, n in shares)
    return ext(51, struct.pack(">H", len(b)) + b)


CHROME_CIPHERS = [0x1301, 0x1302, 0x1303, 0xc02b, 0xc02f, 0xc02c, 0xc030, 0xcca9, 0xcca8, 0xc013, 0xc014, 0x009c,
                  0x009d, 0x002f, 0x0035]
FIREFOX_CIPHERS = [0x1301, 0x1303, 0x1302, 0xc02b, 0xc02f, 0xcca9, 0xcca8, 0xc02c, 0xc030, 0xc00a, 0xc009, 0xc013,
                   0xc014, 0x009c, 0x009d, 0x002f, 0x0035]
SAFARI_CIPHERS = [0x1301, 0x1302, 0x1303, 0xc02c, 0xc02b, 0xcca9, 0xc030, 0xc02f, 0xcca8, 0xc00a, 0xc009, 0xc014,
                  0xc013, 0x009d, 0x009c, 0x0035, 0x002f, 0xc008, 0xc012, 0x000a]
OPENSSL_CIPHERS = [0x1302, 0x1303, 0x1301, 0xc02c, 0xc030, 0x009f, 0xcca9, 0xcca8, 0xccaa, 0xc02b, 0xc02f, 0x009e,
                   0xc024, 0xc028, 0x006b, 0xc023, 0xc027, 0x0067, 0xc00a, 0xc014, 0x0039, 0xc009, 0xc013, 0x0033,
                   0x009d, 0x009c, 0x003d, 0x003c, 0x0035, 0x002f, 0x00ff]
LEGACY_CIPHERS = [0xc014, 0xc013, 0x0035, 0x002f, 0x000a, 0x0005, 0x0004]
JAVA_CIPHERS = [0xc02c, 0xc02b, 0xc030, 0x009d, 0xc02e, 0xc032, 0x009f, 0x00a3, 0xc02f, 0x009c, 0xc02d, 0xc031,
                0x009e, 0x00a2, 0xc024, 0xc028, 0x003d, 0xc026, 0xc02a, 0x006b, 0x006a, 0xc00a, 0xc014, 0x0035,
                0xc005, 0xc00f, 0x0039, 0x0038, 0xc023, 0xc027, 0x003c, 0xc025, 0xc029, 0x0067, 0x0040, 0xc009,
                0xc013, 0x002f, 0xc004, 0xc00e, 0x0033, 0x0032, 0x00ff]
SIGALGS = [0x0403, 0x0804, 0x0401, 0x0503, 0x0805, 0x0501, 0x0806, 0x0601]
SIGALGS_LONG = SIGALGS + [0x0203, 0x0201, 0x0402, 0x0502, 0x0602, 0x0303, 0x0301, 0x0302]


def client_hello(rng, profile, sni, alpn=("h2", "http/1.1"), session_id=True, record_version=0x0301):
    grease = profile in ("chrome", "chrome_pq", "edge")
    g = [int(x) for x in rng.choice(GREASE, 4, replace=False)]
    if profile in ("chrome", "edge", "chrome_pq"):
        ciphers = ([g[0]] if grease else []) + CHROME_CIPHERS
        groups = ([g[1]] if grease else []) + ([0x11ec] if profile == "chrome_pq" else []) + [0x001d, 0x0017, 0x0018]
        shares = ([(g[1], 1)] if grease else []) + ([(0x11ec, 1216)] if profile == "chrome_pq" else []) + [(0x001d, 32)]
        exts = [sni_ext(sni), ext(23, b""), ext(65281, b"\x00"), groups_ext(groups), ext(11, b"\x01\x00"),
                ext(35, b""), alpn_ext(alpn), ext(5, b"\x01\x00\x00\x00\x00"), sigalgs_ext(SIGALGS),
                ext(18, b""), keyshare_ext(shares), ext(45, b"\x01\x01"),
                versions_ext(([g[2]] if grease else []) + [0x0304, 0x0303]), ext(27, b"\x02\x00\x02"),
                ext(17513, b"\x00\x03\x02h2"), ext(65037, bytes(rng.integers(0, 256, 218, dtype=np.uint8)))]
        rng.shuffle(exts)   # chrome permutes its extensions
        if grease:
            exts = [ext(g[3], b"")] + exts + [ext(g[0] ^ 0x1010 if (g[0] ^ 0x1010) in GREASE else g[0], b"\x00")]
    elif profile == "firefox":
        ciphers = FIREFOX_CIPHERS
        exts = [sni_ext(sni), ext(23, b""), ext(65281, b"\x00"), groups_ext([0x001d, 0x0017, 0x0018, 0x0019, 0x0100, 0x0101]),
                ext(11, b"\x01\x00"), ext(35, b""), alpn_ext(alpn), ext(5, b"\x01\x00\x00\x00\x00"),
                ext(34, b"\x00\x08\x04\x03\x05\x03\x06\x03\x02\x03"),
                keyshare_ext([(0x001d, 32), (0x0017, 65)]), versions_ext([0x0304, 0x0303]),
                sigalgs_ext(SIGALGS + [0x0203, 0x0201]), ext(45, b"\x01\x01"), ext(28, b"\x40\x01"),
                ext(65037, bytes(rng.integers(0, 256, 186, dtype=np.uint8)))]
    elif profile == "safari":
        ciphers = SAFARI_CIPHERS
        exts = [ext(g[0] if grease else 0x0a0a, b""), sni_ext(sni), ext(23, b""), ext(65281, b"\x00"),
                groups_ext([0x0a0a, 0x001d, 0x0017, 0x0018, 0x0019]), ext(11, b"\x01\x00"), alpn_ext(alpn),
                ext(5, b"\x01\x00\x00\x00\x00"), sigalgs_ext(SIGALGS_LONG[:12]), ext(18, b""),
                keyshare_ext([(0x0a0a, 1), (0x001d, 32)]), ext(45, b"\x01\x01"),
                versions_ext([0x0a0a, 0x0304, 0x0303, 0x0302, 0x0301]), ext(27, b"\x02\x00\x01"),
                ext(0x1a1a, b"\x00")]
    elif profile == "openssl":
        ciphers = OPENSSL_CIPHERS
        exts = [sni_ext(sni), ext(11, b"\x03\x00\x01\x02"), groups_ext([0x001d, 0x0017, 0x001e, 0x0019, 0x0018]),
                ext(35, b""), ext(22, b""), ext(23, b""), sigalgs_ext(SIGALGS_LONG), versions_ext([0x0304, 0x0303]),
                ext(45, b"\x01\x01"), keyshare_ext([(0x001d, 32)])]
        if alpn:
            exts.insert(4, alpn_ext(alpn))
    elif profile == "java":
        ciphers = JAVA_CIPHERS
        exts = [sni_ext(sni), ext(5, b"\x01\x00\x00\x00\x00"), groups_ext([0x0017, 0x0018, 0x0019, 0x0009, 0x000a]),
                ext(11, b"\x01\x00"), sigalgs_ext(SIGALGS_LONG), ext(50, struct.pack(">H", 16) + bytes(16)),
                ext(17, b"\x00\x0e\x02\x00\x04\x00\x00\x00\x00\x01\x00\x04\x00\x00\x00\x00"), ext(23, b""),
                ext(65281, b"\x00")]
    else:  # legacy
        ciphers = LEGACY_CIPHERS
        exts = [sni_ext(sni), ext(10, b"\x00\x04\x00\x17\x00\x18"), ext(11, b"\x01\x00"), ext(65281, b"\x00")]
    if profile in ("chrome", "firefox", "edge") and rng.random() < 0.3:
        # padding to a fixed size (extension 21)
        exts.append(ext(21, bytes(int(rng.integers(8, 200)))))
    body_exts = b"".join(exts)
    sid = bytes(32) if session_id else b""
    ver = 0x0303 if profile != "legacy" else 0x0301
    cs = b"".join(struct.pack(">H", c) for c in ciphers)
    body = struct.pack(">H", ver) + bytes(32) + bytes([len(sid)]) + sid + struct.pack(">H", len(cs)) + cs + b"\x01\x00"
    body += struct.pack(">H", len(body_exts)) + body_exts
    hs = b"\x01" + struct.pack(">I", len(body))[1:] + body
    return struct.pack(">BHH", 0x16, record_version, len(hs)) + hs


def server_hello(rng, cipher=0x1301, tls13=True, cert_bytes=0):
    exts = b""
    if tls13:
        exts = ext(43, b"\x03\x04") + ext(51, struct.pack(">HH", 0x001d, 32) + bytes(32))
    else:
        exts = ext(65281, b"\x00") + ext(11, b"\x01\x00") + ext(23, b"")
    body = struct.pack(">H", 0x0303) + bytes(32) + b"\x20" + bytes(32) + struct.pack(">HB", cipher, 0)
    body += struct.pack(">H", len(exts)) + exts
    hs = b"\x02" + struct.pack(">I", len(body))[1:] + body
    if cert_bytes:
        cl = cert_bytes
        cert = b"\x0b" + struct.pack(">I", cl + 3)[1:] + struct.pack(">I", cl)[1:] + bytes(min(cl, 400))
        hs += cert
    return struct.pack(">BHH", 0x16, 0x0303, len(hs)) + hs


def dtls_client_hello(rng, sni):
    ch = client_hello(rng, "openssl", sni, alpn=())
    body = ch[9:]     # strip record(5) + handshake header(4)
    # DTLS CH body: version fefd, random, sid, cookie(len 0), ciphers...
    b = bytearray(body)
    b[0:2] = b"\xfe\xfd"
    sidlen = b[34]
    b = bytes(b[:35 + sidlen]) + b"\x00" + bytes(b[35 + sidlen:])
    hs = b"\x01" + struct.pack(">I", len(b))[1:] + struct.pack(">H", 0) + b"\x00\x00\x00" + struct.pack(">I", len(b))[1:] + b
    return struct.pack(">BHHIHH", 0x16, 0xfefd, 0, 0, 0, len(hs)) + hs


UA = ["Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/120.0.0.0 Safari/537.36",
      "Mozilla/5.0 (X11; Linux x86_64; rv:121.0) Gecko/20100101 Firefox/121.0",
      "curl/8.4.0", "python-requests/2.31.0", "Wget/1.21.2", "Microsoft-CryptoAPI/10.0",
      "Mozilla/5.0 (Macintosh; Intel Mac OS X 10_15_7) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.1 Safari/605.1.15"]
HDR_POOL = [("Accept", "*/*"), ("Accept-Encoding", "gzip, deflate, br"), ("Accept-Language", "en-US,en;q=0.9"),
            ("Connection", "keep-alive"), ("Cache-Control", "no-cache"), ("Upgrade-Insecure-Requests", "1"),
            ("DNT", "1"), ("X-Requested-With", "XMLHttpRequest"), ("Referer", "http://example.com/"),
            ("Cookie", "a=b; c=d"), ("Pragma", "no-cache"), ("Origin", "http://example.com"),
            ("Content-Type", "application/json"), ("X-Forwarded-For", "10.1.2.3")]


def http_request(rng, host):
    method = rng.choice(["GET", "GET", "GET", "POST", "HEAD", "PUT", "OPTIONS"])
    path = "/" + "".join(rng.choice(list("abcdefghij/"), int(rng.integers(1, 40))))
    hdrs = [("Host", host), ("User-Agent", str(rng.choice(UA)))]
    k = int(rng.integers(2, 12))
    for i in rng.choice(len(HDR_POOL), k, replace=False):
        name, val = HDR_POOL[i]
        if rng.random() < 0.2:
            name = name.lower()
        hdrs.append((name, val))
    rng.shuffle(hdrs)
    s = f"{method} {path} HTTP/1.1\r\n" + "".join(f"{n}: {v}\r\n" for n, v in hdrs) + "\r\n"
    return s.encode()


RESP_HDRS = [("Server", "nginx/1.18.0"), ("Content-Type", "text/html; charset=UTF-8"), ("Date", "Mon, 01 Jan 2024 00:00:00 GMT"),
             ("Cache-Control", "max-age=3600"), ("Connection", "keep-alive"), ("ETag", '"abc"'), ("Vary", "Accept-Encoding"),
             ("Strict-Transport-Security", "max-age=31536000"), ("X-Cache", "HIT"), ("Content-Length", "1234")]


def http_response(rng):
    code = rng.choice(["200 OK", "301 Moved Permanently", "404 Not Found", "304 Not Modified", "302 Found"])
    k = int(rng.integers(2, len(RESP_HDRS)))
    hdrs = [RESP_HDRS[i] for i in rng.choice(len(RESP_HDRS), k, replace=False)]
    s = f"HTTP/1.1 {code}\r\n" + "".join(f"{n}: {v}\r\n" for n, v in hdrs) + "\r\n"
    return s.encode() + bytes(int(rng.integers(0, 300)))


SSH_BANNERS = ["SSH-2.0-OpenSSH_8.9p1 Ubuntu-3ubuntu0.6", "SSH-2.0-OpenSSH_9.6", "SSH-2.0-libssh_0.10.5",
               "SSH-2.0-PuTTY_Release_0.79", "SSH-2.0-Go", "SSH-2.0-dropbear_2022.83"]
KEX_LISTS = ["curve25519-sha256,curve25519-sha256@libssh.org,ecdh-sha2-nistp256,diffie-hellman-group14-sha256",
             "ssh-ed25519,ecdsa-sha2-nistp256,rsa-sha2-512,rsa-sha2-256",
             "chacha20-poly1305@openssh.com,aes128-ctr,aes192-ctr,aes256-ctr,aes128-gcm@openssh.com",
             "chacha20-poly1305@openssh.com,aes128-ctr,aes192-ctr,aes256-ctr,aes128-gcm@openssh.com",
             "umac-64-etm@openssh.com,hmac-sha2-256-etm@openssh.com,hmac-sha2-512",
             "umac-64-etm@openssh.com,hmac-sha2-256-etm@openssh.com,hmac-sha2-512",
             "none,zlib@openssh.com", "none,zlib@openssh.com", "", ""]


def ssh_kexinit(rng):
    p = b"\x14" + bytes(16)
    for s in KEX_LISTS:
        b = s.encode()
        p += struct.pack(">I", len(b)) + b
    p += b"\x00" + bytes(4)
    pad = 4 + (-(len(p) + 5) % 8)
    return struct.pack(">IB", len(p) + pad + 1, pad) + p + bytes(pad)


def syn_opts(rng, kind):
    if kind == 0:
        return b"\x02\x04\x05\xb4\x04\x02\x08\x0a" + bytes(8) + b"\x01\x03\x03\x07"
    if kind == 1:
        return b"\x02\x04\x05\xb4\x01\x03\x03\x08\x01\x01\x04\x02"
    if kind == 2:
        return b"\x02\x04\x05\xa0\x01\x01\x04\x02"
    return b"\x02\x04\x05\xb4"


NAMES = None


def names(rng, n=10000):
    global NAMES
    if NAMES is None:
        r = np.random.default_rng(1234)
        tlds = ["com", "net", "org", "io", "co.uk", "de", "cn", "ru", "microsoft.com", "googleapis.com"]
        NAMES = []
        for i in range(n):
            lab = "".join(r.choice(list("abcdefghijklmnopqrstuvwxyz0123456789-"), int(r.integers(3, 14))))
            NAMES.append(f"{lab}.{tlds[i % len(tlds)]}" if i % 3 else f"www.{lab}.{tlds[i % len(tlds)]}")
    return NAMES


def zipf_name(rng):
    nm = names(rng)
    k = int(min(len(nm) - 1, rng.zipf(1.1) - 1))
    return nm[k]


PROFILES = ["chrome", "chrome", "chrome", "edge", "chrome_pq", "firefox", "firefox", "safari", "openssl", "java",
            "legacy"]


def make_template(rng, cls):
    """One full Ethernet frame of class `cls`."""
    v6 = rng.random() < 0.1
    P6 = 41 if False else None  # noqa: F841
    if cls == "tls_ch":
        ch = client_hello(rng, str(rng.choice(PROFILES)), zipf_name(rng),
                          alpn=[("h2", "http/1.1"), ("http/1.1",), ()][int(rng.integers(0, 3))],
                          session_id=rng.random() < 0.7)
        ch = ch[:1460] if len(ch) > 1460 else ch   # beyond one MTU: first segment only (truncated)
        return frame(tcp(ch, sport=int(rng.integers(1024, 65535)), dport=443), 6, v6)
    if cls == "tls_sh":
        sh = server_hello(rng, cipher=int(rng.choice([0x1301, 0x1302, 0xc02f, 0xc030])), tls13=rng.random() < 0.6,
                          cert_bytes=int(rng.choice([0, 0, 1500, 3000])))
        return frame(tcp(sh, sport=443, dport=int(rng.integers(1024, 65535))), 6, v6)
    if cls == "dtls_ch":
        return frame(udp(dtls_client_hello(rng, zipf_name(rng)), sport=int(rng.integers(1024, 65535)), dport=443), 17, v6)
    if cls == "http_req":
        return frame(tcp(http_request(rng, zipf_name(rng)), sport=int(rng.integers(1024, 65535)), dport=80), 6, v6)
    if cls == "http_resp":
        return frame(tcp(http_response(rng), sport=80, dport=int(rng.integers(1024, 65535))), 6, v6)
    if cls == "ssh":
        k = int(rng.integers(0, 3))
        client = rng.random() < 0.5
        ports = dict(sport=int(rng.integers(1024, 65535)), dport=22) if client else dict(sport=22, dport=int(rng.integers(1024, 65535)))
        banner = str(rng.choice(SSH_BANNERS)).encode() + (b"\r\n" if rng.random() < 0.8 else b"\n")
        if k == 0:
            pl = banner
        elif k == 1:
            pl = banner + ssh_kexinit(rng)
        else:
            pl = ssh_kexinit(rng)
        return frame(tcp(pl, **ports), 6, v6)
    if cls == "syn":
        return frame(tcp(b"", sport=int(rng.integers(1024, 65535)), dport=int(rng.choice([443, 80, 22])), flags=0x02,
                         win=int(rng.choice([64240, 65535, 29200, 8192])), opts=syn_opts(rng, int(rng.integers(0, 4))),
                         ack=0), 6, v6)
    if cls == "synack":
        return frame(tcp(b"", sport=int(rng.choice([443, 80])), dport=int(rng.integers(1024, 65535)), flags=0x12,
                         win=int(rng.choice([65160, 28960])), opts=syn_opts(rng, int(rng.integers(0, 4)))), 6, v6)
    # no-output traffic
    k = int(rng.integers(0, 3))
    if k == 0:
        return frame(tcp(b"", flags=0x10), 6, v6)
    if k == 1:
        return frame(tcp(bytes(rng.integers(0, 256, int(rng.integers(50, 1400)), dtype=np.uint8)), flags=0x18), 6, v6)
    q = b"\x12\x34\x01\x00\x00\x01\x00\x00\x00\x00\x00\x00\x07example\x03com\x00\x00\x01\x00\x01"
    return frame(udp(q, dport=53), 17, v6)


MIX = [("tls_ch", 0.35), ("tls_sh", 0.05), ("dtls_ch", 0.02), ("http_req", 0.20), ("http_resp", 0.05),
       ("ssh", 0.05), ("syn", 0.15), ("synack", 0.03), ("noise", 0.10)]


def templates(seed, n_templates, workload="mixed"):
    rng = np.random.default_rng(seed)
    if workload == "tls_ch":
        classes = ["tls_ch"] * n_templates
    else:
        names_, p = zip(*MIX)
        classes = list(rng.choice(names_, n_templates, p=np.array(p) / sum(p)))
    return [make_template(rng, c) for c in classes], classes


def batch(n, seed=0x5EED0003, workload="mixed", n_templates=4096, randomize=True, align=1, draw_seed=None,
          diverse_tls=0.0):
    """n packets drawn from a seeded template pool; returns (arena, desc).
    `draw_seed` (default seed + 1) drives which templates are drawn and the
    per-packet randomisation, so shards can share one template pool.
    `diverse_tls`: the fraction of TLS ClientHellos whose first two cipher
    suites are re-drawn per packet (a fingerprint of its own: unknown to the
    archive, a new sighting for the prevalence LRU)."""
    tpl, _ = templates(seed, n_templates, workload)
    rng = np.random.default_rng(seed + 1 if draw_seed is None else draw_seed)
    tid = rng.integers(0, len(tpl), n)
    lens = np.array([len(t) for t in tpl], dtype=np.int64)
    plen = lens[tid]
    if align > 1:
        slot = (plen + align - 1) // align * align
    else:
        slot = plen
    offs = np.zeros(n, dtype=np.int64)
    np.cumsum(slot[:-1], out=offs[1:])
    total = int(offs[-1] + slot[-1]) if n else 0
    arena = np.zeros(total + 64, dtype=np.uint8)
    for t in range(len(tpl)):
        sel = np.nonzero(tid == t)[0]
        if len(sel) == 0:
            continue
        tb = np.frombuffer(tpl[t], dtype=np.uint8)
        idx = offs[sel][:, None] + np.arange(len(tb))[None, :]
        arena[idx] = tb
        if randomize:
            _randomize(arena, offs[sel], tpl[t], rng)
        if diverse_tls > 0:
            _diversify(arena, offs[sel], tpl[t], rng, diverse_tls)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["offset"] = offs
    desc["caplen"] = plen
    desc["linktype"] = 1
    return arena, desc


def _randomize(arena, offs, tb, rng):
    """Re-draw addresses/ports (and TLS client random) per packet."""
    et = (tb[12] << 8) | tb[13]
    m = len(offs)
    if et == 0x0800:
        ip = 14
        for k in range(4):       # src/dst addr low bytes
            arena[offs + ip + 12 + 2 + (k % 2)] = rng.integers(0, 256, m, dtype=np.uint8)
            arena[offs + ip + 16 + 2 + (k % 2)] = rng.integers(0, 256, m, dtype=np.uint8)
        l4 = ip + 20
        proto = tb[ip + 9]
    elif et == 0x86dd:
        ip = 14
        arena[offs + ip + 8 + 15] = rng.integers(0, 256, m, dtype=np.uint8)
        arena[offs + ip + 24 + 15] = rng.integers(0, 256, m, dtype=np.uint8)
        l4 = ip + 40
        proto = tb[ip + 6]
    else:
        return
    if proto not in (6, 17):
        return
    sport = (tb[l4] << 8) | tb[l4 + 1]
    dport = (tb[l4 + 2] << 8) | tb[l4 + 3]
    # keep the server port and the client/server order of ports (SSH direction)
    if sport > dport and sport >= 1024:
        new = rng.integers(max(1024, dport + 1), 65535, m)
        arena[offs + l4] = (new >> 8).astype(np.uint8)
        arena[offs + l4 + 1] = (new & 0xff).astype(np.uint8)
    elif dport > sport and dport >= 1024:
        new = rng.integers(max(1024, sport + 1), 65535, m)
        arena[offs + l4 + 2] = (new >> 8).astype(np.uint8)
        arena[offs + l4 + 3] = (new & 0xff).astype(np.uint8)
    if proto == 6:
        hl = (tb[l4 + 12] >> 4) * 4
        pl = l4 + hl
        if len(tb) >= pl + 43 and tb[pl] == 0x16 and tb[pl + 5] == 0x01:
            # client random (32 bytes after version)
            for k in range(32):
                arena[offs + pl + 11 + k] = rng.integers(0, 256, m, dtype=np.uint8)


def _diversify(arena, offs, tb, rng, frac):
    """Re-draw the first two cipher suites of a TLS ClientHello template's
    copies (a fraction `frac` of them) with random non-GREASE values."""
    et = (tb[12] << 8) | tb[13]
    ip = 14
    if et == 0x0800 and tb[ip + 9] == 6:
        l4 = ip + 20
    elif et == 0x86dd and tb[ip + 6] == 6:
        l4 = ip + 40
    else:
        return
    pl = l4 + (tb[l4 + 12] >> 4) * 4
    if len(tb) < pl + 48 or tb[pl] != 0x16 or tb[pl + 5] != 0x01:
        return
    c = pl + 9 + 2 + 32
    c += 1 + tb[c]                                   # session id
    if len(tb) < c + 6 or ((tb[c] << 8) | tb[c + 1]) < 4:
        return
    sel = offs[rng.random(len(offs)) < frac]
    for k in range(4):                               # bytes of the first two suites
        v = rng.integers(0, 256, len(sel), dtype=np.uint8)
        if k in (1, 3):
            v = np.where((v & 0x0f) == 0x0a, v ^ 0x01, v).astype(np.uint8)   # never a GREASE value
        arena[sel + c + 2 + k] = v


# ---------------------------------------------------------------------------
# fuzzing for parity stress
# ---------------------------------------------------------------------------


def fuzz(pkts, n, seed):
    """Mutate (linktype, bytes) packets: byte flips in the payload region,
    truncations, length-field edits.  Returns [(linktype, bytes)]."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        lt, p = pkts[int(rng.integers(0, len(pkts)))]
        b = bytearray(p)
        if not b:
            out.append((lt, bytes(b)))
            continue
        k = int(rng.integers(0, 5))
        if k == 0:      # truncate
            b = b[:int(rng.integers(0, len(b) + 1))]
        elif k == 1:    # flip random bytes
            for _ in range(int(rng.integers(1, 8))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        elif k == 2:    # flip bytes near the start of L4 payload
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(min(len(b) - 1, 34), len(b)))
                b[j] = int(rng.integers(0, 256))
        elif k == 3:    # GREASE-ish / special values at random 2-byte positions
            j = int(rng.integers(0, max(1, len(b) - 1)))
            v = int(rng.choice([0x0a0a, 0x1a1a, 0xfafa, 0x1a0a, 0x0000, 0xffff, 0xff01, 0x0039, 0x002b, 0x000a]))
            b[j:j + 2] = struct.pack(">H", v)[:len(b) - j]
        else:           # insert/delete a byte
            j = int(rng.integers(0, len(b)))
            if rng.random() < 0.5:
                del b[j]
            else:
                b.insert(j, int(rng.integers(0, 256)))
        out.append((lt, bytes(b)))
    return out


# ---------------------------------------------------------------------------
# unknown-TLS prevalence stream (fingerprint_prevalence LRU, analysis.h:362-421)
# ---------------------------------------------------------------------------
def lru_keys(capacity=100000, seed=0x5EED1234):
    """The key sequence of a stream that crosses the reference's LRU capacity:
    1.2 x capacity distinct fingerprints once each (the oldest fifth is
    evicted), the first tenth again (evicted: randomized again, evicting more),
    a tenth near the recent end (still in the set: unlabeled), then 0.3 x
    capacity draws around the eviction boundary, where each status depends on
    the exact recency order."""
    rng = np.random.default_rng(seed)
    c = capacity
    first = np.arange(int(1.2 * c))
    again_old = np.arange(int(0.1 * c))
    again_new = np.arange(int(1.0 * c), int(1.1 * c))
    mix = rng.integers(0, int(1.3 * c), int(0.3 * c))
    return np.concatenate([first, again_old, again_new, mix]).astype(np.int64)


def lru_batch(keys, seed=0x5EED1235):
    """One TLS ClientHello per key whose fingerprint is unique to the key (two
    cipher suites encode it; no other field varies), Ethernet/IPv4/TCP 443."""
    rng = np.random.default_rng(seed)
    base = bytearray(frame(tcp(client_hello(rng, "openssl", "lru.example.com"), sport=50000, dport=443), 6))
    # the cipher list: the openssl profile's first two suites are patched
    cs = struct.pack(">HH", OPENSSL_CIPHERS[0], OPENSSL_CIPHERS[1])
    at = bytes(base).index(cs)
    n = len(keys)
    L = len(base)
    arena = np.zeros(n * L + 64, np.uint8)
    arena[:n * L] = np.tile(np.frombuffer(bytes(base), np.uint8), n)
    k = np.asarray(keys, np.int64)
    c1 = 0x3000 + ((k >> 12) & 0xfff)
    c2 = 0x4000 + (k & 0xfff)
    offs = np.arange(n, dtype=np.int64) * L + at
    arena[offs] = (c1 >> 8) & 0xff
    arena[offs + 1] = c1 & 0xff
    arena[offs + 2] = (c2 >> 8) & 0xff
    arena[offs + 3] = c2 & 0xff
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["offset"] = np.arange(n, dtype=np.uint64) * L
    desc["caplen"] = L
    desc["linktype"] = 1
    return arena, desc
