// mfp_encap.hpp -- host-side walk of a packet's encapsulation chain, for the
// outputs that describe it (not for fingerprinting, which the device does):
// the JSON writer's "encapsulations" array (encapsulations::write_json
// pkt_proc.cc:1033-1043; gre.h:69-75, vxlan.hpp:60-68, geneve.hpp:85-91,
// ip_encapsulation ip.h:788-793) and the reassembler's rebuilt frames, whose
// outer IP lengths it patches.
//
// The device record gives the innermost IP header's offset; this walk repeats
// the decapsulation of encapsulations::process_encapsulations
// (pkt_proc.cc:972-1028) from the link layer until it reaches that header and
// reports every level it crossed.  The protocol selection is not needed: the
// walk stops where the device stopped.
#pragma once
#include <cstdint>

namespace mfpe {

enum Kind : uint8_t { IPIP = 0, GRE, VXLAN, GENEVE };

struct Level {
    uint8_t kind;         // Kind
    uint8_t ipv;          // version of the IP header the entry's addresses come from
    uint16_t proto_type;  // GRE / Geneve protocol_type
    uint32_t ip_off;      // that IP header's offset
};

struct Chain {
    int n = 0;            // levels crossed (<= 4)
    Level lv[4];
};

// struct datum (datum.h) restricted to what the walk needs: a null cursor
// stays null
struct Cur {
    const uint8_t *d, *e;
    long len() const { return d ? (long)(e - d) : 0; }
    bool null() const { return d == nullptr; }
    void nullify() { d = e = nullptr; }
    bool skip(long n) {
        if (!d || n < 0 || n > e - d) { nullify(); return false; }
        d += n;
        return true;
    }
    bool rd(int n, uint64_t &v) {
        v = 0;
        if (!d || n > e - d) { nullify(); return false; }
        for (int i = 0; i < n; i++) v = v << 8 | d[i];
        d += n;
        return true;
    }
    void trim(long n) { if (d && n >= 0 && n < e - d) e = d + n; }
};

// ppp::is_ip ppp.h:76
inline bool ppp_is_ip(Cur &p) {
    uint64_t b;
    if (p.len() > 0 && p.d[0] == 0x7e) { if (!p.rd(1, b)) return false; }
    if (p.len() > 0 && p.d[0] == 0xff) { uint64_t t; p.rd(2, t); }
    if (p.null() || p.len() <= 0) return false;
    uint64_t proto;
    if (p.d[0] & 1) p.rd(1, proto); else p.rd(2, proto);
    return !p.null() && (proto == 0x21 || proto == 0x57);
}

// eth::get_ip eth.h:114-187
inline bool eth_get_ip(Cur &p) {
    uint64_t et;
    p.skip(12);
    if (!p.rd(2, et)) return false;
    if (et == 0x88a8) { p.skip(2); if (!p.rd(2, et)) return false; }
    while (et == 0x8100) { p.skip(2); if (!p.rd(2, et)) return false; }
    if (et == 0x8847) {
        uint64_t lbl = 0;
        while (!(lbl & 0x100)) { if (!p.rd(4, lbl)) return false; }
        et = 0x0800;
    }
    if (et == 0x8909) { p.skip(6); if (!p.rd(2, et)) return false; }
    if (et == 0x0800 || et == 0x86dd) return true;
    if (et == 0x8864) { p.skip(6); return !p.null() && ppp_is_ip(p); }
    return false;
}

inline bool loopback_ok(uint64_t v) {
    return v == 2 || v == 0x02000000 || v == 24 || v == 0x18000000 || v == 28 || v == 0x1c000000 || v == 30 ||
           v == 0x1e000000;
}

// the link layer down to the first IP header (pkt_proc.cc:1328-1383)
inline bool link_to_ip(Cur &p, uint32_t linktype) {
    uint64_t t, a, b;
    switch (linktype) {
    case 1: return eth_get_ip(p);
    case 9: return ppp_is_ip(p);
    case 101: return true;
    case 113:                                        // linux_sll.hpp
        p.rd(2, t); p.rd(2, a); p.rd(2, t); p.skip(8); p.rd(2, b);
        return !p.null() && (a == 1 || a == 772) && (b == 0x0800 || b == 0x86dd);
    case 276:                                        // linux_sll2.hpp
        p.rd(2, b); p.rd(2, t); p.rd(4, t); p.rd(2, a); p.rd(1, t); p.rd(1, t); p.skip(8);
        return !p.null() && (a == 1 || a == 772) && (b == 0x0800 || b == 0x86dd);
    case 0:                                          // loopback.hpp
        p.rd(4, t);
        return p.null() || loopback_ok(t);
    default:
        return false;
    }
}

// ip::parse ip.h:619-632 (ipv4 fixed 20 bytes, ipv6 + extension headers):
// the transport protocol, the header's offset and version; the cursor is
// left on the payload, trimmed to the header's length field
inline uint32_t ip_parse(Cur &p, const uint8_t *base, uint32_t &off, int &ipv) {
    ipv = 0;
    if (p.len() <= 0) return 255;
    const uint8_t v = p.d[0] & 0xf0;
    if (v == 0x40) {
        if (p.len() < 20) { p.nullify(); ipv = 4; return 255; }
        const uint8_t *h = p.d;
        off = (uint32_t)(h - base); ipv = 4;
        p.d += 20;
        p.trim((long)((uint32_t)h[2] << 8 | h[3]) - 20);
        return h[9];
    }
    if (v == 0x60) {
        if (p.len() < 40) { p.nullify(); ipv = 6; return 255; }
        const uint8_t *h = p.d;
        off = (uint32_t)(h - base); ipv = 6;
        p.d += 40;
        p.trim((long)((uint32_t)h[4] << 8 | h[5]));
        uint32_t nh = h[6];
        while (p.len() > 0) {
            if (!(nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135 || nh == 139 || nh == 140)) break;
            uint64_t nnh = 0, hl = 0;
            p.rd(1, nnh);
            if (nh == 44) p.skip(7);
            else if (nh == 51) { p.rd(1, hl); p.skip((long)hl * 4 + 6); }
            else { p.rd(1, hl); p.skip((long)hl * 8 + 6); }
            nh = (uint32_t)nnh;
        }
        return nh;
    }
    return 255;
}

// the levels from the link layer to the IP header at inner_off; false when
// the walk cannot reach it (the caller then has nothing to describe)
inline bool walk(const uint8_t *pkt, uint32_t caplen, uint32_t linktype, uint32_t inner_off, Chain &c) {
    c.n = 0;
    Cur p{pkt, pkt + caplen};
    if (!link_to_ip(p, linktype) || p.null()) return false;
    uint32_t off = ~0u;
    int ipv = 0;
    uint32_t proto = ip_parse(p, pkt, off, ipv);
    while (true) {
        if (off == inner_off && ipv) return true;
        if (c.n == 4 || p.null()) return false;
        Level L{IPIP, (uint8_t)ipv, 0, off};
        if (proto == 4 || proto == 41) {
            L.kind = IPIP;
        } else if (proto == 47) {                              // gre_header gre.h:38-57
            uint64_t crv, pt;
            p.rd(2, crv); p.rd(2, pt);
            if (crv & 0x8000) p.skip(4);
            if (p.null() || (pt != 0x0800 && pt != 0x86dd)) return false;
            L.kind = GRE; L.proto_type = (uint16_t)pt;
        } else if (proto == 17) {
            Cur u = p;
            uint64_t sp, dp, t;
            u.rd(2, sp); u.rd(2, dp); u.rd(4, t);
            if (u.null()) return false;
            if (dp == 4789) {                                 // vxlan.hpp:31-47
                uint64_t fl;
                u.rd(1, fl); u.skip(7);
                if (!(fl & 0x08) || !eth_get_ip(u)) return false;
                L.kind = VXLAN;
            } else if (dp == 6081) {                          // geneve.hpp:22-57
                uint64_t fb, x, pt;
                u.rd(1, fb); u.rd(1, x); u.rd(2, pt); u.skip(4); u.skip(4 * (long)(fb & 0x3f));
                if (u.null()) return false;
                if (pt == 0x6558) { if (!eth_get_ip(u)) return false; }
                else if (pt == 0x0800 || pt == 0x86dd) { }
                else if (pt == 0) { uint64_t lt; u.rd(4, lt); if (u.null() || !loopback_ok(lt)) return false; }
                else return false;
                L.kind = GENEVE; L.proto_type = (uint16_t)pt;
            } else if (dp == 4754) {                          // GRE over UDP
                uint64_t crv, pt;
                u.rd(2, crv); u.rd(2, pt);
                if (crv & 0x8000) u.skip(4);
                if (u.null() || (pt != 0x0800 && pt != 0x86dd)) return false;
                L.kind = GRE; L.proto_type = (uint16_t)pt;
            } else {
                return false;
            }
            p = u;
        } else {
            return false;
        }
        c.lv[c.n++] = L;
        proto = ip_parse(p, pkt, off, ipv);
    }
}

}  // namespace mfpe
