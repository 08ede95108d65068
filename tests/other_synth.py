"""Packets that protocols outside the device path claim before one of its own
when the selection names them ("all" names every one): the matchers and ports
that traffic_selector consults first (proto_identify.h:620-895, 936-1075) and
the port table of the encapsulation walk (pkt_proc.cc:1000-1018).  Test
infrastructure for tests/golden/make_golden_all.py; the expected records are
the reference's.

Each scenario is a (label, frame) pair; the frames are Ethernet/IPv4.
"""
import struct

import numpy as np

from tests import quic_synth, stun_ovpn_synth, synth

HTTP_GET = b"GET /index.html HTTP/1.1\r\nHost: example.com\r\nUser-Agent: curl/8.0\r\nAccept: */*\r\n\r\n"
HTTP_RESP = b"HTTP/1.1 200 OK\r\nServer: nginx\r\nContent-Length: 0\r\n\r\n"


def tcp_frame(payload, sport, dport):
    return synth.frame(synth.tcp(payload, sport=sport, dport=dport), 6)


def udp_frame(payload, sport, dport):
    return synth.frame(synth.udp(payload, sport=sport, dport=dport), 17)


def openvpn_payload(rng):
    # an OpenVPN-over-TCP P_CONTROL_HARD_RESET_CLIENT_V2 record (openvpn.h)
    body = bytes([0x38]) + bytes(rng.integers(0, 256, 8, dtype=np.uint8)) + b"\x00" + b"\x00\x00\x00\x00"
    return struct.pack(">H", len(body)) + body


def scenarios(seed=0x5EED0A11):
    rng = np.random.default_rng(seed)
    out = []
    ch = synth.client_hello(rng, "firefox", "other.example.com")
    # HTTP behind the port table (get_tcp_msg_type_from_ports proto_identify.h:1015-1075)
    for lab, sp, dp in (("rdp", 50000, 3389), ("telnet", 50000, 23), ("krb5", 50000, 88), ("tacacs", 50000, 49),
                        ("mysql", 50000, 3306), ("redis_req", 50000, 6379), ("imap_req", 50000, 143),
                        ("ldap", 50000, 389), ("nbss", 50000, 139), ("ftp_resp", 21, 50000),
                        ("redis_resp", 6379, 50000), ("imap_resp", 143, 50000), ("redis_src_dst", 50000, 6380),
                        ("plain80", 50000, 80), ("plain8080", 50000, 8080)):
        out.append((f"http.{lab}", tcp_frame(HTTP_GET, sp, dp)))
        out.append((f"http_resp.{lab}", tcp_frame(HTTP_RESP, dp, sp)))
        out.append((f"tls.{lab}", tcp_frame(ch, sp, dp)))          # the TLS matcher comes first: a record
        out.append((f"ovpn.{lab}", tcp_frame(openvpn_payload(rng), sp, 1194)))
    # the tcp / tcp4 tables behind TLS and SSH, before the OpenVPN port and the keywords
    tcp_payloads = {
        "smtp_250": b"250-mail.example.com Hello\r\n250-SIZE 1000\r\n",
        "smtp_ehlo": b"EHLO client.example.com\r\n",
        "dns_tcp": b"\x00\x1d\x12\x34\x01\x00\x00\x01\x00\x00\x00\x00\x00\x00\x07example\x03com\x00\x00\x01\x00\x01",
        "smb1": b"\x00\x00\x00\x2f\xffSMB\x72" + bytes(40),
        "smb2": b"\x00\x00\x00\x40\xfeSMB\x40\x00" + bytes(56),
        "bt": b"\x13BitTorrent protocol" + bytes(48),
        "mysql": b"\x4a\x00\x00\x00\x0a5.7.33-log\x00" + bytes(40),
        "socks4": b"\x04\x01\x00\x50\x5d\xb8\xd8\x22user\x00",
        "socks4a": b"\x04\x01\x00\x50\x00\x00\x00\x01\x00example.com\x00",
        "socks5_hello": b"\x05\x02\x00\x02",
        "socks5_req": b"\x05\x01\x00\x01\x5d\xb8\xd8\x22\x00\x50",
        "socks5_dom": b"\x05\x01\x00\x03\x0bexample.com\x00\x50",
        "iec": b"\x68\x04\x07\x00\x00\x00",
        "dnp3": b"\x05\x64\x05\xc0\x01\x00\x00\x04\xe9\x21",
        "dnp3_bad": b"\x05\x64\x05\xc0\x01\x00\x00\x04\xe9",
        "get_short": b"GET ",
    }
    for lab, pl in tcp_payloads.items():
        for dp in (1194, 80, 50001):
            out.append((f"tcp.{lab}.{dp}", tcp_frame(pl, 50000, dp)))
    # UDP: ESP/IKE ports, the udp table before QUIC / DTLS / STUN, the port table
    qpk = [p for lab, p in quic_synth.scenarios(n_random=4) if lab in ("version-00000001", "version-6b3343cf")]
    quic_payloads = []
    for p in qpk:
        # the UDP payload of the scenario frame (Ethernet 14 + IPv4 20 + UDP 8)
        quic_payloads.append(p[42:])
    dtls = synth.dtls_client_hello(rng, "dtls.example.com")
    stun = stun_ovpn_synth.stun_msg(0x0001, [stun_ovpn_synth.stun_attr(0x8022, b"agent")])
    stun_classic_zero = struct.pack(">HH", 0x0001, 0) + bytes(16)          # dns_packet::matcher claims it
    wireguard_like = b"\x01\x00\x00\x00\x21\x12\xa4\x42" + bytes(12)       # STUN type 0x0100, length 0
    for lab, pl in (("quic", quic_payloads[0]), ("dtls", dtls), ("stun", stun), ("stun_zero", stun_classic_zero),
                    ("wg", wireguard_like)):
        for sp, dp in ((50000, 443), (50000, 4500), (4500, 50000), (50000, 500), (50000, 69), (50000, 161),
                       (138, 138), (50000, 514), (50000, 88), (50000, 3478)):
            out.append((f"udp.{lab}.{sp}.{dp}", udp_frame(pl, sp, dp)))
    for lab, pl in (("dht", b"d1:ad2:id20:" + bytes(30)), ("lsd", b"BT-SEARCH * HTTP/1.1\r\n\r\n"),
                    ("ssdp", b"M-SEARCH * HTTP/1.1\r\nHOST: 239.255.255.250:1900\r\n\r\n")):
        out.append((f"udp.{lab}", udp_frame(pl, 50000, 1900)))
    # encapsulations behind the port table: VXLAN / Geneve / GRE over UDP with
    # a source port the table claims first
    inner = synth.eth(synth.ipv4(synth.tcp(ch, sport=40000, dport=443), 6))
    vx = struct.pack(">BBHI", 0x08, 0, 0, 0x123400) + inner
    gen = struct.pack(">BBHI", 0, 0, 0x6558, 0x123400) + inner
    gre = struct.pack(">HH", 0, 0x0800) + synth.ipv4(synth.tcp(ch, sport=40000, dport=443), 6)
    for lab, pl, dp in (("vxlan", vx, 4789), ("geneve", gen, 6081), ("gre", gre, 4754)):
        for sp in (50000, 69, 88, 161, 162, 500, 4500, 514, 138):
            out.append((f"encap.{lab}.{sp}", udp_frame(pl, sp, dp)))
        out.append((f"encap.{lab}.syslog_dst", udp_frame(pl, 514, dp)))
    return out
