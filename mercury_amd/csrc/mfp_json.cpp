// mfp_json.cpp -- JSON record assembly from device records (host side).
//
// The reference writes one JSON line per packet inside its per-packet walk
// (stateful_pkt_proc::ip_write_json, pkt_proc.cc:1157-1253).  Here the walk
// runs on the GPU and leaves a 32-byte record per packet (mfp_record); this
// file turns a batch of records + the packet arena + the fingerprint arena
// into the same text, on host threads, after the D2H copy.  No packet is
// re-parsed: every byte range the JSON needs (server name, user agent,
// certificate list, innermost IP header) comes from the record.
//
// Record layout (pkt_proc.cc:1193-1238, metadata_output off):
//   {"fingerprints":{"<type>":"<fp>"}          fingerprint::write fingerprint.h:194
//    ,"tls"|"dtls":{"client":{"server_name":…}} tls_client_hello::write_json tls.h:1882
//    ,"tls":{"server":{"certs":[{"base64":…}]}} tls_server_hello_and_certificate tls.h:605,
//                                                tls_certificate tls.h:744, tls.h:2183
//    ,"dtls":{"server":{}}                     write_metadata pkt_proc_util.h:315
//    ,"http":{"request":{"user_agent":…}}      http_request::write_json http.cc:323
//    ,"reassembly_properties":{"truncated":true} reassembly.hpp:1231
//    ,"src_ip":…,"dst_ip":…,"protocol":…,"src_port":…,"dst_port":…  write_flow_key pkt_proc.cc:86
//    ,"event_start":<sec>.<usec>}\n              append_timestamp buffer_stream.h:256
// Strings go through the reference's UTF-8 escaper (utf8_string::write,
// utf8.hpp:200-340); IPv6 addresses through its zero-run compression
// (append_ipv6_addr buffer_stream.h:534-690, quirks included).

#include <algorithm>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <cmath>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mfp_encap.hpp"
#include "mfp_internal.h"

namespace {

const char HEX[] = "0123456789abcdef";

// 8 bytes -> 16 lowercase hex characters, first byte first (SWAR on two
// 64-bit words: nibbles spread to bytes, then '0'/'a' added by a carry test)
inline void hex8(const uint8_t *x, char *o) {
    uint64_t v;
    memcpy(&v, x, 8);
    auto spread = [](uint64_t b) {                 // 4 bytes (little-endian) -> 8 nibbles, high first
        b = (b | (b << 16)) & 0x0000ffff0000ffffull;
        b = (b | (b << 8)) & 0x00ff00ff00ff00ffull;
        const uint64_t nib = ((b >> 4) & 0x000f000f000f000full) | ((b & 0x000f000f000f000full) << 8);
        const uint64_t gt9 = ((nib + 0x7676767676767676ull) & 0x8080808080808080ull) >> 7;
        return nib + 0x3030303030303030ull + gt9 * 0x27;
    };
    const uint64_t lo = spread(v & 0xffffffffull), hi = spread(v >> 32);
    memcpy(o, &lo, 8);
    memcpy(o + 8, &hi, 8);
}
// two characters per byte value
struct Hex2 {
    char t[256][2];
    Hex2() { for (int i = 0; i < 256; i++) { t[i][0] = HEX[i >> 4]; t[i][1] = HEX[i & 15]; } }
};
const Hex2 HEX2;
// base64 of 12 bits -> 2 characters
struct B64T {
    char t[4096][2];
    B64T() {
        static const char T[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
        for (int i = 0; i < 4096; i++) { t[i][0] = T[i >> 6]; t[i][1] = T[i & 63]; }
    }
};
const B64T B64;

// fingerprint::get_type_name fingerprint.h:159-192
const char *fp_type_name(unsigned t) {
    static const char *name[] = {"unknown", "tls", "tls_server", "http", "http_server", "ssh", "ssh_kex",
                                 "tcp", "dhcp", "smtp_server", "dtls", "dtls_server", "quic", "tcp_server",
                                 "openvpn", "tofsee", "stun", "ssh_init", "ssh_server", "ssh_kex_server",
                                 "ssh_init_server"};
    return t <= 20 ? name[t] : name[0];
}

// Output buffer (one per thread, kept between calls) ...
struct alignas(64) Out {
    std::unique_ptr<char[]> buf;           // uninitialised: every byte below len is written
    size_t cap = 0, len = 0;
    void need(size_t n) {
        if (len + n <= cap) return;
        // the first reservation of a call is its estimate: exact; growth
        // while formatting: x1.5 (ample for records longer than estimated)
        size_t c = len == 0 ? n : std::max(len + n, cap + cap / 2);
        std::unique_ptr<char[]> b(new char[c]);
        if (len) memcpy(b.get(), buf.get(), len);
        buf.swap(b);
        cap = c;
    }
};

// ... and the write cursor over it: a local of write_record, so the cursor
// lives in a register (a cursor in memory would put a store-to-load
// dependency on every byte written).  write_record reserves the record's
// worst case first, so the writers carry no bounds checks.
struct W {
    char *p;
    void put(char c) { *p++ = c; }
    template <size_t N> void puts(const char (&s)[N]) { memcpy(p, s, N - 1); p += N - 1; }
    void putz(const char *s) { size_t n = strlen(s); memcpy(p, s, n); p += n; }
    void mem(const void *s, size_t n) { if (n) memcpy(p, s, n); p += n; }
    void u8dec(unsigned v) {                       // append_uint8 (no leading zeros)
        struct Tab {                               // "0".."255", 4 bytes each + length
            char s[256][4]; uint8_t n[256];
            Tab() { for (int i = 0; i < 256; i++) n[i] = (uint8_t)snprintf(s[i], 4, "%d", i); }
        };
        static const Tab tab;
        memcpy(p, tab.s[v & 255], 4);              // over-copy by design; need() reserved room
        p += tab.n[v & 255];
    }
    void hexb(const uint8_t *x, size_t n) {         // raw_as_hex
        size_t k = 0;
        for (; k + 8 <= n; k += 8) { hex8(x + k, p); p += 16; }
        for (; k < n; k++) { memcpy(p, HEX2.t[x[k]], 2); p += 2; }
    }
    void hexu(uint64_t v, int digits) {             // append_uint{8,16,32,64}_hex: fixed width
        for (int k = digits - 1; k >= 0; k--) put(HEX[(v >> (4 * k)) & 15]);
    }
    void udec(uint64_t v) {
        char t[24]; int n = 0;
        do { t[n++] = '0' + v % 10; v /= 10; } while (v);
        while (n) put(t[--n]);
    }
    void codepoint(unsigned c) {                   // utf8_string::write_codepoint utf8.hpp:87
        put('\\'); put('u');
        put(HEX[(c >> 12) & 15]); put(HEX[(c >> 8) & 15]); put(HEX[(c >> 4) & 15]); put(HEX[c & 15]);
    }
    // utf8_string::write utf8.hpp:200-340 (JSON-escaped, U+FFFD for invalid)
    void utf8(const uint8_t *x, size_t len) {
        static const char repl[] = "\\ufffd";
        auto cont = [](uint8_t b) { return (b & 0xc0) == 0x80; };
        auto second_ok = [&](uint8_t b1, uint8_t b2) {
            switch (b1) {
            case 0xe0: return b2 >= 0xa0 && b2 <= 0xbf;
            case 0xed: return b2 >= 0x80 && b2 <= 0x9f;
            case 0xf0: return b2 >= 0x90 && b2 <= 0xbf;
            case 0xf4: return b2 >= 0x80 && b2 <= 0x8f;
            default: return cont(b2);
            }
        };
        const uint8_t *end = x + len;
        while (x < end) {
            if (*x >= 0x80) {
                uint32_t cp = 0;
                if (*x >= 0xc2) {
                    if (*x >= 0xe0) {
                        if (*x >= 0xf0 && *x <= 0xf4) {
                            if (end - x < 4) { puts(repl); x++; continue; }
                            if (second_ok(x[0], x[1]) && cont(x[2]) && cont(x[3])) {
                                cp = ((uint32_t)(x[0] & 7) << 18) | ((uint32_t)(x[1] & 0x3f) << 12) |
                                     ((uint32_t)(x[2] & 0x3f) << 6) | (x[3] & 0x3f);
                                x += 3;
                            }
                        } else if (*x <= 0xef) {
                            if (end - x < 3) { puts(repl); x++; continue; }
                            if (second_ok(x[0], x[1]) && cont(x[2])) {
                                cp = ((uint32_t)(x[0] & 0x0f) << 12) | ((uint32_t)(x[1] & 0x3f) << 6) | (x[2] & 0x3f);
                                x += 2;
                            }
                        }
                    } else {
                        if (end - x < 2) { puts(repl); x++; continue; }
                        if (second_ok(x[0], x[1])) { cp = ((uint32_t)(x[0] & 0x1f) << 6) | (x[1] & 0x3f); x += 1; }
                    }
                    if (cp == 0) {
                        puts(repl);
                    } else if ((cp >= 0xe000 && cp <= 0xf8ff) || (cp >= 0xf0000 && cp <= 0xffffd) ||
                               (cp >= 0x100000 && cp <= 0x10fffd) || (cp >= 0xd800 && cp <= 0xdfff)) {
                        puts(repl);
                    } else if (cp > 0xffff) {
                        cp -= 0x10000;
                        codepoint((cp >> 10) + 0xd800);
                        codepoint((cp & 0x3ff) + 0xdc00);
                    } else {
                        codepoint(cp);
                    }
                } else {
                    puts(repl);
                }
            } else if (*x < 0x20 || *x == 0x7f) {
                codepoint(*x);
            } else {
                if (*x == '"' || *x == '\\') put('\\');
                put((char)*x);
            }
            x++;
        }
    }
    // append_raw_as_base64 buffer_stream.h:885-975 (quoted, '=' padded)
    void base64(const uint8_t *d, size_t n) {
        static const char T[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
        put('"');
        size_t i = 0, full = n - n % 3;
        for (; i < full; i += 3) {
            const uint32_t t = ((uint32_t)d[i] << 16) | ((uint32_t)d[i + 1] << 8) | d[i + 2];
            memcpy(p, B64.t[t >> 12], 2);
            memcpy(p + 2, B64.t[t & 4095], 2);
            p += 4;
        }
        if (n % 3) {
            uint32_t t = (uint32_t)d[i] << 16;
            if (n % 3 == 2) t |= (uint32_t)d[i + 1] << 8;
            put(T[t >> 18 & 63]); put(T[t >> 12 & 63]);
            if (n % 3 == 2) { put(T[t >> 6 & 63]); put('='); } else { put('='); put('='); }
        }
        put('"');
    }
    void ipv4(const uint8_t *a) {                  // append_ipv4_addr buffer_stream.h:748
        u8dec(a[0]); put('.'); u8dec(a[1]); put('.'); u8dec(a[2]); put('.'); u8dec(a[3]);
    }
    // append_ipv6_addr buffer_stream.h:534-690, literally: a zero run that
    // ends without beating the longest so far is not reset (the next zero
    // field continues it from its old start).
    void ipv6(const uint8_t *v6) {
        uint16_t w[8];
        for (int i = 0; i < 8; i++) w[i] = (uint16_t)(v6[2 * i] | v6[2 * i + 1] << 8);   // memory order
        int run = -1, run_len = 0, lr = -1, lr_len = 0;
        for (int u = 0; u < 8; u++) {
            if (w[u] == 0) {
                if (run_len == 0) run = u;
                run_len++;
            } else if (run_len != 0 && lr_len < run_len) {
                lr_len = run_len; lr = run; run_len = 0;
            }
        }
        if (lr_len < run_len) { lr_len = run_len; lr = run; }
        if (lr_len == 1) { lr_len = 0; lr = 8; }
        auto field = [&](int u) {
            const uint8_t *v = v6 + 2 * u;
            int k = (v[0] & 0xf0) ? 4 : (v[0] & 0x0f) ? 3 : (v[1] & 0xf0) ? 2 : 1;
            if (k >= 4) put(HEX[v[0] >> 4]);
            if (k >= 3) put(HEX[v[0] & 15]);
            if (k >= 2) put(HEX[v[1] >> 4]);
            put(HEX[v[1] & 15]);
        };
        int u = 0;
        const int stop = lr < 0 ? 0 : lr;              // nullptr: the first loop prints nothing
        while (u < stop) { field(u++); if (u != stop) put(':'); }
        u += lr_len;
        if (lr_len != 0) { put(':'); put(':'); }
        while (u < 8) { field(u++); if (u != 8) put(':'); }
    }
    // append_timestamp buffer_stream.h:256-310: seconds without leading zeros,
    // '.', six digits of microseconds.  Fast path with constant divisors; the
    // reference's loop (variable divisor, first "digit" = sec / 1e9 even when
    // that exceeds 9) is kept for sec >= 1e10.
    void timestamp(uint64_t sec, uint64_t nsec) {
        char o[32]; int i = 0;
        if (sec < 10000000000ull) {
            char t[12]; int k = 0;
            uint64_t v = sec;
            do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
            while (k) o[i++] = t[--k];
        } else {
            bool lead = true;
            uint64_t v = sec;
            for (uint64_t p = 1000000000; p >= 10; p /= 10) {
                int d = (int)(v / p); v %= p;
                if (d == 0 && lead) continue;
                lead = false; o[i++] = (char)('0' + d);
            }
            o[i++] = (char)('0' + v);
        }
        o[i++] = '.';
        uint32_t us = (uint32_t)(nsec / 1000);
        for (int k = 5; k >= 0; k--) { o[i + k] = (char)('0' + us % 10); us /= 10; }
        mem(o, i + 6);
    }
};

// json_object comma discipline (json_object.h:49-73)
struct Obj {
    W &o; bool comma = false;
    template <size_t N> void key(const char (&k)[N]) {
        char t[N + 3];
        size_t j = 0;
        if (comma) t[j++] = ',';
        comma = true;
        t[j++] = '"';
        memcpy(t + j, k, N - 1); j += N - 1;
        t[j++] = '"'; t[j++] = ':';
        o.mem(t, j);
    }
};

bool is_tcp_msg(unsigned m) {
    return m != MFP_MSG_DTLS_CH && m != MFP_MSG_DTLS_SH && m != MFP_MSG_DTLS_HVR && m != MFP_MSG_QUIC && m != MFP_MSG_STUN;
}

// "%f" (json_object::print_key_float json_object.h:174-177).  printf's %f
// is the exact decimal value rounded to 6 places, ties to even; for |d| <
// 1e12 that is computed here from the double's binary form (m * 2^e times
// 10^6, exactly, in 128 bits, then rounded), without snprintf's cost; other
// values (and NaN, infinities) go through snprintf.
void put_float(W &w, double d) {
    uint64_t bits;
    memcpy(&bits, &d, 8);
    const bool neg = (bits >> 63) != 0;
    const uint32_t be = (uint32_t)((bits >> 52) & 0x7ff);
    if (be < 0x7ff && std::fabs(d) < 1e12) {
        uint64_t m = bits & ((1ull << 52) - 1);
        int e;
        if (be == 0) e = -1074; else { m |= 1ull << 52; e = (int)be - 1075; }
        uint64_t q;
        if (e >= 0) {
            q = (m << e) * 1000000ull;                   // (|d| < 1e12: no overflow)
        } else {
            const unsigned __int128 x = (unsigned __int128)m * 1000000u;
            const int sh = -e;
            if (sh >= 128) {
                q = 0;
            } else {
                q = (uint64_t)(x >> sh);
                const unsigned __int128 rem = x & ((((unsigned __int128)1) << sh) - 1);
                const unsigned __int128 half = ((unsigned __int128)1) << (sh - 1);
                if (rem > half || (rem == half && (q & 1))) q++;
            }
        }
        if (neg) w.put('-');
        w.udec(q / 1000000u);
        w.put('.');
        uint32_t f = (uint32_t)(q % 1000000u);
        char t[6];
        for (int k = 5; k >= 0; k--) { t[k] = (char)('0' + f % 10); f /= 10; }
        w.mem(t, 6);
        return;
    }
    char t[352];   // %f of the largest double is 316 digits + sign, dot, 6 decimals
    const int n = snprintf(t, sizeof t, "%f", d);
    w.mem(t, n > 0 ? (size_t)n : 0);
}

// worst-case text of a record's "analysis" object
size_t analysis_bound(mfp_context ctx, const mfp_analysis &a) {
    size_t b = 400 + 16 * 64 + mfp_attribute_names_len(ctx);   // keys, numbers, 16 attribute entries, names
    if (a.process != MFP_NO_PROCESS) b += 256;      // max_proc holds at most 255 bytes (result.h:198)
    if (a.proc_slot != MFP_NO_PROCESS) {
        const int cnt = mfp_process_os_info(ctx, a.proc_slot, 0, nullptr, nullptr);
        for (int k = 0; k < cnt; k++) {
            const char *nm = nullptr;
            mfp_process_os_info(ctx, a.proc_slot, (uint32_t)k, &nm, nullptr);
            b += (nm ? strlen(nm) : 0) + 32;
        }
    }
    return b;
}

// analysis_result::write_json (result.h:207-252) with attribute_result::write_json (result.h:62-77)
void write_analysis(W &w, mfp_context ctx, const mfp_analysis &a, const double *ap) {
    w.puts("{");
    Obj o{w};
    auto process_part = [&]() {
        o.key("process"); w.put('"');
        const char *nm = mfp_process_name(ctx, a.process);
        if (nm) w.mem(nm, strnlen(nm, 255));        // strncpy(max_proc, proc, max_proc_len - 1)
        w.put('"');
        o.key("score"); put_float(w, a.score);
        if (a.flags & MFP_AN_CLASSIFY_MALWARE) {
            o.key("malware"); w.put((a.flags & MFP_AN_MALWARE) ? '1' : '0');
            o.key("p_malware"); put_float(w, a.malware_prob);
        }
        const int cnt = a.proc_slot == MFP_NO_PROCESS ? 0 : mfp_process_os_info(ctx, a.proc_slot, 0, nullptr, nullptr);
        if (cnt > 0) {
            o.key("os_info"); w.put('{');
            for (int k = 0; k < cnt; k++) {
                const char *nm2 = nullptr;
                uint64_t prev = 0;
                mfp_process_os_info(ctx, a.proc_slot, (uint32_t)k, &nm2, &prev);
                if (k) w.put(',');
                w.put('"'); w.putz(nm2 ? nm2 : ""); w.puts("\":"); w.udec(prev);
            }
            w.put('}');
        }
    };
    const bool named = a.process != MFP_NO_PROCESS && mfp_process_name(ctx, a.process) &&
                       mfp_process_name(ctx, a.process)[0] != 0;
    switch (a.status) {
    case 1:                                          // fingerprint_status_labeled
        process_part();
        break;
    case 2:                                          // fingerprint_status_randomized
        if (named) process_part();
        o.key("status"); w.puts("\"randomized_fingerprint\"");
        break;
    case 3:                                          // fingerprint_status_unlabled
        o.key("status"); w.puts("\"unlabeled_fingerprint\"");
        break;
    default:
        o.key("status"); w.puts("\"unknown\"");
        break;
    }
    o.key("attributes"); w.put('[');
    const int na = mfp_attribute_count(ctx);
    bool first = true;
    for (int k = 0; k < na && k < MFP_ATTR_MAX_TAGS; k++) {
        if (!((a.attr >> k) & 1u)) continue;
        if (!first) w.put(',');
        first = false;
        w.puts("{\"name\":\""); w.putz(mfp_attribute_name(ctx, (uint32_t)k)); w.puts("\",\"probability_score\":");
        double p = 1.0;                               // encrypted_dns, domain_faking, faketls (analysis.h:555-573)
        if (k >= MFP_ATTR_DB_FIRST) p = ap ? ap[k - MFP_ATTR_DB_FIRST] : 0.0;
        else if (k == 7) p = a.malware_prob;          // encrypted_channel (analysis.h:1161-1163)
        put_float(w, p);
        w.put('}');
    }
    w.puts("]}");
}

// one record; returns false when the record cannot be written exactly here
struct TsCache { uint64_t sec = ~0ull, usec = ~0ull; int len = 0; char text[40]; };

// ---- STUN and OpenVPN objects, rebuilt from the message bytes the record's
// server-name span holds (host cursor over struct datum semantics)
struct HC { const uint8_t *d, *e; };
inline long hlen(HC c) { return c.d ? (long)(c.e - c.d) : 0; }
inline void hnull(HC &c) { c.d = c.e = nullptr; }
inline uint64_t hrd(HC &c, int n) {                 // encoded<T>: 0 and null when short
    if (c.d && c.d + n <= c.e) { uint64_t v = 0; for (int i = 0; i < n; i++) v = v << 8 | c.d[i]; c.d += n; return v; }
    hnull(c); return 0;
}
inline HC hparse(HC &r, long n) {                   // datum(datum &, n)
    HC o;
    if (hlen(r) < n || n < 0) { hnull(r); hnull(o); return o; }
    o.d = r.d; o.e = r.d ? r.d + n : nullptr; if (r.d) r.d += n;
    return o;
}

// stun_params.h: method and attribute names (IANA registry names)
const char *stun_method_name(unsigned m) {
    switch (m) {
    case 0x001: return "Binding"; case 0x002: return "SharedSecret"; case 0x003: return "Allocate";
    case 0x004: return "Refresh"; case 0x006: return "Send"; case 0x007: return "Data";
    case 0x008: return "CreatePermission"; case 0x009: return "ChannelBind"; case 0x00A: return "Connect";
    case 0x00B: return "ConnectionBind"; case 0x00C: return "ConnectionAttempt"; case 0x080: return "GOOG_PING";
    }
    return nullptr;
}
const char *stun_attr_name(unsigned t) {
    static const struct { uint16_t t; const char *n; } tab[] = {
        {0x0001, "MAPPED_ADDRESS"}, {0x0002, "RESPONSE_ADDRESS"}, {0x0004, "SOURCE_ADDRESS"},
        {0x0005, "CHANGED_ADDRESS"}, {0x0006, "USERNAME"}, {0x0008, "MESSAGE_INTEGRITY"}, {0x0009, "ERROR_CODE"},
        {0x000A, "UNKNOWN_ATTRIBUTES"}, {0x000B, "REFLECTED_FROM"}, {0x000C, "CHANNEL_NUMBER"}, {0x000D, "LIFETIME"},
        {0x0010, "BANDWIDTH"}, {0x0012, "XOR_PEER_ADDRESS"}, {0x0013, "DATA"}, {0x0014, "REALM"}, {0x0015, "NONCE"},
        {0x0016, "XOR_RELAYED_ADDRESS"}, {0x0017, "REQUESTED_ADDRESS_FAMILY"}, {0x0018, "EVEN_PORT"},
        {0x0019, "REQUESTED_TRANSPORT"}, {0x001A, "DONT_FRAGMENT"}, {0x001B, "ACCESS_TOKEN"},
        {0x001C, "MESSAGE_INTEGRITY_SHA256"}, {0x001D, "PASSWORD_ALGORITHM"}, {0x001E, "USERHASH"},
        {0x0020, "XOR_MAPPED_ADDRESS"}, {0x0022, "RESERVATION_TOKEN"}, {0x0024, "PRIORITY"}, {0x0025, "USE_CANDIDATE"},
        {0x0026, "PADDING"}, {0x0027, "RESPONSE_PORT"}, {0x002A, "CONNECTION_ID"}, {0x8000, "ADDITIONAL_ADDRESS_FAMILY"},
        {0x8001, "ADDRESS_ERROR_CODE"}, {0x8002, "PASSWORD_ALGORITHMS"}, {0x8003, "ALTERNATE_DOMAIN"}, {0x8004, "ICMP"},
        {0x8008, "MS_VERSION"}, {0x8020, "MS_XOR_MAPPED_ADDRESS"}, {0x8022, "SOFTWARE"}, {0x8023, "ALTERNATE_SERVER"},
        {0x8025, "TRANSACTION_TRANSMIT_COUNTER"}, {0x8027, "CACHE_TIMEOUT"}, {0x8028, "FINGERPRINT"},
        {0x8029, "ICE_CONTROLLED"}, {0x802A, "ICE_CONTROLLING"}, {0x802B, "RESPONSE_ORIGIN"}, {0x802C, "OTHER_ADDRESS"},
        {0x802D, "ECN_CHECK_STUN"}, {0x802E, "THIRD_PARTY_AUTHORIZATION"}, {0x8030, "MOBILITY_TICKET"},
        {0x8032, "MS_ALTERNATE_HOST_NAME"}, {0x8037, "MS_APP_ID"}, {0x8039, "MS_SECURE_TAG"},
        {0x8050, "MS_SEQUENCE_NUMBER"}, {0x8055, "MS_SERVICE_QUALITY"}, {0x8056, "MS_BANDWIDTH_ADMISSION_CONTROL_MESSAGE"},
        {0x8070, "MS_IMPLEMENTATION_VERSION"}, {0x8090, "MS_ALTERNATE_MAPPED_ADDRESS"},
        {0x8095, "MS_MULTIPLEXED_TURN_SESSION_ID"}, {0xC000, "CISCO_STUN_FLOWDATA"}, {0xC001, "ENF_FLOW_DESCRIPTION"},
        {0xC002, "ENF_NETWORK_STATUS"}, {0xC057, "GOOG_NETWORK_INFO"}, {0xC058, "GOOG_LAST_ICE_CHECK_RECEIVED"},
        {0xC059, "GOOG_MISC_INFO"}, {0xC05A, "GOOG_OBSOLETE_1"}, {0xC05B, "GOOG_CONNECTION_ID"}, {0xC05C, "GOOG_DELTA"},
        {0xC05D, "GOOG_DELTA_ACK"}, {0xC060, "GOOG_MESSAGE_INTEGRITY_32"},
    };
    for (const auto &x : tab) if (x.t == t) return x.n;
    return nullptr;
}
// stun::method_usage / attribute_type_usage (stun.h:513-584): 1 stun, 2 turn, 4 ice
unsigned stun_method_usage(unsigned m) { return m == 1 || m == 2 ? 1u : (m >= 3 && m <= 9 && m != 5) ? 2u : 0u; }
unsigned stun_attr_usage(unsigned t) {
    switch (t) {
    case 0x0001: case 0x0002: case 0x0003: case 0x0004: case 0x0005: case 0x0006: case 0x0007: case 0x0008:
    case 0x0009: case 0x000A: case 0x000B: case 0x0010: case 0x0014: case 0x0015: case 0x001C: case 0x001D:
    case 0x001E: case 0x0020: case 0x8002: case 0x8003: case 0x8022: case 0x8023: case 0x8028: return 1;
    case 0x000C: case 0x000D: case 0x0012: case 0x0013: case 0x0016: case 0x0017: case 0x0018: case 0x0019:
    case 0x001A: case 0x0021: case 0x0022: case 0x8000: case 0x8001: case 0x8004: return 2;
    case 0x0024: case 0x0025: case 0x8029: case 0x802A: return 4;
    }
    return 0;
}
// stun::attribute (stun.h:323-338): false (cursor null) when incomplete
bool stun_attr(HC &d, unsigned &t, HC &v) {
    t = (unsigned)hrd(d, 2);
    const long l = (long)hrd(d, 2);
    v = hparse(d, d.d ? l : 0);
    const long pad = (4 - (l & 3)) & 3;
    if (d.d) { if (hlen(d) < pad) hnull(d); else d.d += pad; }
    return d.d != nullptr;
}
void unknown_code(W &w, uint64_t v, int digits) { w.puts("\"UNKNOWN ("); w.hexu(v, digits); w.puts(")\""); }

// stun::message::write_json (stun.h:795-826) with attribute::write_json (stun.h:340-439)
void write_stun(W &w, const uint8_t *m, size_t len) {
    const unsigned mtf = (unsigned)m[0] << 8 | m[1], ml = (unsigned)m[2] << 8 | m[3];
    const bool cookie = m[4] == 0x21 && m[5] == 0x12 && m[6] == 0xa4 && m[7] == 0x42;
    w.puts("{");
    Obj o{w};
    if (ml % 4) { o.key("malformed"); w.puts("true"); }
    const unsigned method = (mtf & 0x0f) | ((mtf & 0xe0) >> 1) | ((mtf & 0x3e00) >> 2);
    o.key("method");
    if (const char *n = stun_method_name(method)) { w.put('"'); w.putz(n); w.put('"'); } else unknown_code(w, method, 4);
    o.key("class");
    switch (mtf & 0x0110) {
    case 0x0000: w.puts("\"request\""); break;
    case 0x0010: w.puts("\"indication\""); break;
    case 0x0100: w.puts("\"success_resp\""); break;
    default: w.puts("\"err_resp\""); break;
    }
    o.key("message_length"); w.udec(ml);
    o.key("transaction_id"); w.put('"'); w.hexb(m + (cookie ? 8 : 4), cookie ? 12 : 16); w.put('"');
    o.key("magic_cookie"); if (cookie) w.puts("true"); else w.puts("false");
    o.key("attributes"); w.put('[');
    unsigned usage = stun_method_usage(method);
    HC tmp{m + 20, m + len};
    bool first = true;
    while (hlen(tmp) > 0) {
        HC la = tmp, v; unsigned t;
        if (!first) w.put(',');
        first = false;
        if (!stun_attr(la, t, v)) {
            w.puts("{\"unparseable\":\""); w.hexb(tmp.d, (size_t)hlen(tmp)); w.puts("\"}");
            break;
        }
        w.put('{');
        Obj a{w};
        a.key("type");
        if (const char *n = stun_attr_name(t)) { w.put('"'); w.putz(n); w.put('"'); } else unknown_code(w, t, 4);
        a.key("length"); w.udec((uint64_t)hlen(v));
        auto addr = [&](bool x) {                    // mapped_address / xor_mapped_address (stun.h:61-166)
            HC d = v;
            hrd(d, 1);
            const unsigned fam = (unsigned)hrd(d, 1), port = (unsigned)hrd(d, 2);
            HC ad = hparse(d, fam == 2 ? 16 : 4);
            if (!d.d || !(ad.d && ad.d < ad.e)) return;       // lookahead failed / !valid()
            a.key("family"); w.put('"'); w.putz(fam == 1 ? "ipv4" : fam == 2 ? "ipv6" : "UNKNOWN"); w.put('"');
            if (!x) {
                a.key("port"); w.udec(port);
                if (fam == 1) { if (hlen(ad) == 4) { a.key("address"); w.put('"'); w.ipv4(ad.d); w.put('"'); } }
                else if (fam == 2) { if (hlen(ad) == 16) { a.key("address"); w.put('"'); w.ipv6(ad.d); w.put('"'); } }
                else { a.key("address"); w.puts("\"malformed\""); }
            } else {
                a.key("x_port"); w.udec((port ^ 0x2112u) & 0xffff);
                if (fam == 1) {
                    const uint32_t xa = ((uint32_t)ad.d[0] << 24 | (uint32_t)ad.d[1] << 16 | (uint32_t)ad.d[2] << 8 | ad.d[3]) ^
                                        0x2112a442u;
                    const uint8_t b[4] = {(uint8_t)(xa >> 24), (uint8_t)(xa >> 16), (uint8_t)(xa >> 8), (uint8_t)xa};
                    a.key("x_address"); w.put('"'); w.ipv4(b); w.put('"');
                } else {
                    a.key("x_address"); w.put('"'); w.hexb(ad.d, (size_t)hlen(ad)); w.put('"');
                }
            }
        };
        auto u32 = [&](const char *k) {
            HC d = v; const uint64_t x = hrd(d, 4);
            if (d.d) { w.put(','); w.put('"'); w.putz(k); w.puts("\":"); w.udec(x); }
        };
        switch (t) {
        case 0x0025: break;                                            // USE_CANDIDATE
        case 0x0001: case 0x0002: case 0x0004: case 0x0005: case 0x000B: case 0x8023: case 0x802B: case 0x802C:
            addr(false); break;
        case 0x0020: case 0x0012: case 0x0016: addr(true); break;
        case 0x8022: case 0x0006: case 0x0015:                         // utf8_string
            if (v.d) { a.key("value"); w.put('"'); w.utf8(v.d, (size_t)hlen(v)); w.put('"'); }
            break;
        case 0x0009: {                                                 // error_code
            HC d = v; const uint64_t rc = hrd(d, 4);
            if (d.d) {
                a.key("class"); w.udec((rc >> 8) & 7);
                a.key("number"); w.udec(rc & 0xff);
                if (hlen(d) > 0) { a.key("reason_phrase"); w.put('"'); w.utf8(d.d, (size_t)hlen(d)); w.put('"'); }
            }
            break;
        }
        case 0x0024: u32("priority"); break;
        case 0x8029: case 0x802A: {
            HC d = v; const uint64_t x = hrd(d, 8);
            if (d.d) { a.key("tiebreaker"); w.put('"'); w.hexu(x, 16); w.put('"'); }
            break;
        }
        case 0x000C: {
            HC d = v; const uint64_t x = hrd(d, 2); hrd(d, 2);
            if (d.d) { a.key("channel_number"); w.udec(x); }
            break;
        }
        case 0x000D: u32("seconds"); break;
        case 0x0010: u32("kbps"); break;
        case 0x0019: {                                                 // skip_bytes<3>: datum::skip clamps
            HC d = v; const uint64_t x = hrd(d, 1); if (d.d) d.d = hlen(d) < 3 ? d.e : d.d + 3;
            if (d.d) { a.key("protocol"); w.udec(x); }
            break;
        }
        case 0x8056: {
            HC d = v; if (d.d) d.d = hlen(d) < 2 ? d.e : d.d + 2; const unsigned x = (unsigned)hrd(d, 2);
            if (d.d) {
                a.key("message_type");
                if (x <= 2) { w.put('"'); w.putz(x == 0 ? "reservation_check" : x == 1 ? "reservation_commit" : "reservation_update"); w.put('"'); }
                else unknown_code(w, x, 4);
            }
            break;
        }
        case 0x8070: u32("number"); break;
        default:
            a.key("hex_value"); w.put('"'); if (v.d && v.e > v.d) w.hexb(v.d, (size_t)hlen(v)); w.put('"');
        }
        w.put('}');
        usage |= stun_attr_usage(t);
        tmp = la;
    }
    w.put(']');
    o.key("usage");
    w.put('"'); w.putz(usage == 1 ? "stun" : (usage == 2 || usage == 3) ? "turn" : (usage == 4 || usage == 5) ? "ice" : "unknown");
    w.put('"');
    w.put('}');
}

void client_hello_json(W &w, Obj &rec, mfpe::Cur p);

// openvpn_tcp::write_json (openvpn.h:411-442) + tls_client_hello::write_json
// (tls.h:1882-1917, metadata off)
bool write_openvpn(W &w, Obj &rec, const uint8_t *m, size_t len) {
    struct R { unsigned op, replay, nid, msg; bool ctrl; };
    std::vector<R> ctrl, ack;
    uint8_t buf[800];
    size_t used = 0;
    bool buf_null = false;
    uint64_t total = 0;
    unsigned nrec = 0;
    HC d{m, m + len};
    while (hlen(d) > 0) {                                   // openvpn_tcp_record / openvpn_payload
        const unsigned plen = (unsigned)hrd(d, 2), code = (unsigned)hrd(d, 1);
        const unsigned op = code >> 3;
        const int type = (op >= 1 && op <= 4) || op == 7 || op == 8 || op == 10 || op == 11 ? 1 : op == 5 ? 0
                         : (op == 6 || op == 9) ? 2 : 3;
        R r{op, 0, 0, 0, type == 1};
        hrd(d, 8);
        uint64_t hm = 0;
        { HC la = d; hm = hrd(la, 4); }
        unsigned zeros = 0;
        for (int k = 0; k < 4; k++) zeros += ((hm >> (8 * k)) & 0xff) == 0;
        unsigned hmac_len = 0;
        if (zeros <= 1) {
            if (hlen(d) < 16) return true;                  // invalid record: no object (valid stays false)
            long at = 0, z = 0;
            const long dl = hlen(d);
            while (z < 2 && at < dl) { z = d.d[at] == 0 ? z + 1 : 0; at++; }
            const unsigned hl = (unsigned)(uint8_t)((z == 2 ? at : -at) - 2);
            if (hl < 16 || (long)hl >= hlen(d)) return true;
            hmac_len = hl;
            d.d += hl;
        }
        r.replay = (unsigned)hrd(d, 4);
        bool net_time = false;
        { HC dc = d; const unsigned b1 = (unsigned)hrd(dc, 1), b2 = (unsigned)hrd(dc, 1); if ((long)b1 * 4 > hlen(dc) || b2) net_time = true; }
        if (net_time) hrd(d, 4);
        r.nid = (unsigned)hrd(d, 1);
        if (hlen(d) < 4 * (long)r.nid) return true;
        if (r.nid) { hparse(d, 4 * (long)r.nid); hrd(d, 8); }
        if (r.ctrl) r.msg = (unsigned)hrd(d, 4);
        const unsigned hdr = 1 + 8 + hmac_len + 4 + (net_time ? 4 : 0) + 1 + 4 * r.nid + (r.nid ? 8 : 0) + (r.ctrl ? 4 : 0);
        if (op == 4) {
            if (hdr >= plen) return true;
            const long dl = (long)((plen - hdr) & 0xffff);
            if (hlen(d) < dl) return true;
            // data_buffer<800>::parse consumes the record's data datum when it
            // fits, so total_data (openvpn.h:388-395) counts only the data
            // from the first record that did not fit onward
            if (!buf_null) {
                if (used + (size_t)dl > sizeof buf) buf_null = true;
                else { memcpy(buf + used, d.d, (size_t)dl); used += (size_t)dl; }
            }
            if (buf_null) total += (uint64_t)dl;
            d.d += dl;
        }
        if (!d.d || type == 3) return true;                 // the packet has no record
        if (type == 0) ack.push_back(r); else if (type == 1) ctrl.push_back(r);
        nrec++;
    }
    if ((uint8_t)nrec == 0) return true;
    // the ClientHello: tls_record -> tls_handshake -> tls_client_hello
    HC chb{nullptr, nullptr};
    bool hello = false;
    if (!ctrl.empty() && !buf_null && used) {
        // tls_record::parse tls.h:153 / tls_handshake::parse tls.h:244 (outer-bounded),
        // tls_client_hello::parse tls.h:1811
        auto outer = [](HC &r, uint64_t n) {
            HC o{nullptr, nullptr};
            if (!(r.d && r.d < r.e)) return o;
            o.d = r.d; o.e = n > (uint64_t)(r.e - r.d) ? r.e : r.d + n; r.d = o.e;
            return o;
        };
        HC p{buf, buf + used}, frag{nullptr, nullptr}, body{nullptr, nullptr};
        if (hlen(p) >= 5) { hrd(p, 1); hrd(p, 2); frag = outer(p, hrd(p, 2)); }
        if (hlen(frag) >= 4) { hrd(frag, 1); const uint64_t hl = hrd(frag, 3); if (hl <= 32768) body = outer(frag, hl); }
        chb = body;
        HC b = body;
        HC ver = hparse(b, 2);
        if (ver.d && ver.e > ver.d) {
            const bool dtls = ver.d[0] == 0xfe;
            hparse(b, 32);
            bool ok = true;
            if (!b.d || hlen(b) < 1) ok = false;
            if (ok) { const long sl = (long)hrd(b, 1); hparse(b, sl); }
            if (ok && dtls) {
                if (hlen(b) < 1) ok = false;
                else { const long cl0 = b.d[0]; if (cl0 + 1 > hlen(b)) { b.d = b.e; ok = false; } else b.d += cl0 + 1; }
            }
            if (ok && hlen(b) < 2) ok = false;
            long cl = 0;
            if (ok) { cl = (long)hrd(b, 2); if (cl & 1) ok = false; }
            HC cm{nullptr, nullptr};
            if (ok) { hparse(b, cl); if (hlen(b) < 1) ok = false; }
            if (ok) { const long ml = (long)hrd(b, 1); cm = hparse(b, ml); }
            hello = cm.d && cm.e > cm.d;
        }
    }
    rec.key("openvpn");
    w.put('{');
    Obj o{w};
    o.key("num_records"); w.udec((uint8_t)nrec);
    o.key("records"); w.put('[');
    bool first = true;
    static const char *names[12] = {nullptr, "P_CONTROL_HARD_RESET_CLIENT_V1", "P_CONTROL_HARD_RESET_SERVER_V1",
                                    "P_CONTROL_SOFT_RESET_V1", "P_CONTROL_V1", "P_ACK_V1", "P_DATA_V1",
                                    "P_CONTROL_HARD_RESET_CLIENT_V2", "P_CONTROL_HARD_RESET_SERVER_V2", "P_DATA_V2",
                                    "P_CONTROL_HARD_RESET_CLIENT_V3", "P_CONTROL_WKC_V1"};
    for (int pass = 0; pass < 2; pass++)
        for (const R &r : pass ? ack : ctrl) {
            if (!first) w.put(',');
            first = false;
            w.puts("{\"opcode\":\""); w.putz(names[r.op]); w.puts("\",\"replay_pkt_id\":"); w.udec(r.replay);
            w.puts(",\"id_array_len\":"); w.udec(r.nid);
            if (r.ctrl) { w.puts(",\"msg_pkt_id\":"); w.udec(r.msg); }
            w.put('}');
        }
    w.put(']');
    if (total) { o.key("data_len"); w.udec(total); }
    if (hello) { o.key("has_tls"); w.puts("true"); }
    w.put('}');
    if (hello) client_hello_json(w, rec, mfpe::Cur{chb.d, chb.e});   // openvpn.h:438-440
    return true;
}

// tcp_reassembler::write_json (reassembly.hpp:860-880) from the props bits of
// mfp_process_batch_reassembly
void write_reassembled(W &w, uint16_t props) {
    static const char *flag[7] = {"missing_segment", "timeout", "out_of_order", "out_of_buffer", "max_segments_exceed",
                                  "segment_overlaps", "truncated"};
    static const char *ovl[4] = {"back_partial_overlap", "back_subset_overlap", "front_partial_overlap",
                                 "front_superset_overlap"};
    w.puts("{\"reassembled\":true");
    for (int k = 0; k < 7; k++) if (props >> (1 + k) & 1) { w.puts(",\""); w.putz(flag[k]); w.puts("\":true"); }
    for (int k = 0; k < 4; k++) if (props >> (8 + k) & 1) { w.puts(",\""); w.putz(ovl[k]); w.puts("\":true"); }
    w.put('}');
}

// ---- QUIC Initial records (quic_init::write_json quic.h:1662-1690, the
// pre-decrypted quic_init_decry::write_json quic.h:1438-1452): the long header
// fields come from the packet, the plaintext, the handshake bytes, the cc
// frame's place and the decryption salt from k_quic's sidecar (include/mfp.h)
struct QuicJson {
    const uint8_t *pay = nullptr, *pt = nullptr, *hs = nullptr;
    uint32_t pay_len = 0, pt_len = 0, hs_len = 0, cc_off = 0xffff, salt = 0xff;
    bool pre = false, hello = false;
};

uint32_t rd16le(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }

bool quic_block(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, const char *fp_arena, QuicJson &q) {
    if (!(r.flags & MFP_FLAG_SIDECAR)) return false;
    const uint8_t *sc = (const uint8_t *)fp_arena + r.fp_offset + ((r.fp_len + 7) & ~7u) + 8;
    const uint32_t jo = rd16le(sc + 6);
    if (!jo) return false;
    const uint8_t *j = sc + jo;
    const uint32_t po = rd16le(j);
    q.pay_len = rd16le(j + 2); q.pt_len = rd16le(j + 4); q.hs_len = rd16le(j + 6); q.cc_off = rd16le(j + 8);
    q.pre = j[10] & 1; q.hello = (j[10] >> 1) & 1; q.salt = j[11];
    if ((uint64_t)po + q.pay_len > caplen) return false;
    q.pay = pkt + po;
    q.pt = j + 16;
    q.hs = q.pt + q.pt_len;
    return true;
}

// datum::parse: too short nulls both (datum.h:294-304)
mfpe::Cur take(mfpe::Cur &d, long n) {
    mfpe::Cur r{nullptr, nullptr};
    if (d.null() || n < 0 || d.len() < n) { d.nullify(); return r; }
    r.d = d.d; r.e = d.d + n; d.d += n;
    return r;
}
// variable_length_integer (quic_vli.hpp): a short read nulls the datum
uint64_t vli(mfpe::Cur &d) {
    uint64_t b = 0;
    if (!d.rd(1, b)) return 0;
    const int len = (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1;
    uint64_t v = b & 0x3f, x = 0;
    for (int k = 1; k < len; k++) { if (!d.rd(1, x)) return 0; v = v * 256 + x; }
    return v;
}

void quic_cc(W &w, Obj &qo, const uint8_t *f, const uint8_t *end) {   // quic_frame::write_json (quic.h:1184-1200)
    mfpe::Cur d{f + 1, end};
    const uint8_t t = f[0];
    if (t == 0x1c) {                                       // connection_close quic.h:354-372
        const uint64_t ec = vli(d), ft = vli(d), rl = vli(d);
        const mfpe::Cur rp = take(d, (long)rl);
        if (rp.null() || rp.len() <= 0) return;
        qo.key("connection_close");
        w.puts("{\"error_code\":"); w.udec(ec);
        w.puts(",\"frame_type\":"); w.udec(ft);
        w.puts(",\"reason_phrase\":\""); w.utf8(rp.d, (size_t)rp.len()); w.puts("\"}");
        return;
    }
    // ack (quic.h:123-150) / ack_ecn (quic.h:160-178)
    const uint64_t la = vli(d), dl = vli(d), rc = vli(d), fr = vli(d);
    bool ok = true;
    if (rc > 1000) ok = false;
    else for (uint64_t k = 0; k < rc && d.len() > 0; k++) { vli(d); vli(d); }
    if (d.null()) ok = false;
    auto ack = [&]() {
        w.puts("{\"largest_acked\":"); w.udec(la); w.puts(",\"ack_delay\":"); w.udec(dl);
        w.puts(",\"ack_range_count\":"); w.udec(rc); w.puts(",\"first_ack_range\":"); w.udec(fr); w.put('}');
    };
    if (t == 0x02) {
        if (ok) { qo.key("ack"); ack(); }
        return;
    }
    if (!ok) return;                                       // ack_ecn keeps reading from a null datum: invalid
    const uint64_t e0 = vli(d), e1 = vli(d), ce = vli(d);
    if (d.null()) return;
    qo.key("ack_ecn");
    w.puts("{\"ect0\":"); w.udec(e0); w.puts(",\"ect1\":"); w.udec(e1); w.puts(",\"ecn_ce\":"); w.udec(ce);
    w.puts(",\"ack\":"); ack(); w.put('}');
}

// the "tls" (or "dtls") object of a ClientHello (tls_client_hello::write_json
// tls.h:1882-1917, metadata off) from its handshake body: the first
// server_name, every quic_transport_parameters extension with the user agents
// inside it (tls.h:1264-1311).  Used for TLS ClientHellos over TCP, DTLS
// ClientHellos, QUIC hellos and OpenVPN's, so that the JSON text follows the
// reference's own parse of the hello rather than the classifier's view in the
// record (whose server name is the LAST server_name extension,
// tls_extensions::set_meta_data tls.h:1316-1345).
// tls_client_hello::parse tls.h:1811-1869 over a handshake body: false unless
// the hello is not empty (compression methods present, tls.h:443); the
// extensions (soft-failed to the bytes present), whether the cipher-suite
// vector is readable, and the DTLS bit (a 0xfe.. version: cookie, "dtls")
bool hello_extensions(mfpe::Cur p, mfpe::Cur &ext, bool &ciphers_ok, bool &dtls) {
    ext = mfpe::Cur{nullptr, nullptr};
    ciphers_ok = false;
    const mfpe::Cur ver = take(p, 2);
    if (ver.null() || ver.len() <= 0) return false;
    dtls = ver.d[0] == 0xfe;                               // tls.h:1823-1825
    take(p, 32);
    uint64_t l = 0;
    if (!p.rd(1, l)) return false;
    take(p, (long)l);
    if (dtls) {                                            // tls.h:1836-1844
        if (p.null() || p.len() < 1) return false;
        if (!p.skip((long)p.d[0] + 1)) return false;
    }
    if (!p.rd(2, l) || (l & 1)) return false;
    const mfpe::Cur ciphers = take(p, (long)l);
    if (!p.rd(1, l)) return false;
    const mfpe::Cur comp = take(p, (long)l);
    if (comp.null() || comp.len() <= 0) return false;      // hello.is_not_empty()
    ciphers_ok = !ciphers.null() && ciphers.len() > 0;     // !ciphersuite_vector.is_not_readable()
    if (p.rd(2, l)) { ext.d = p.d; ext.e = p.d + ((long)l < p.len() ? (long)l : p.len()); }   // parse_soft_fail
    return true;
}

void client_hello_json(W &w, Obj &rec, mfpe::Cur p) {
    mfpe::Cur ext;
    bool ciphers_ok = false, dtls = false;
    if (!hello_extensions(p, ext, ciphers_ok, dtls) || !ciphers_ok) return;   // tls.h:1883-1885
    if (dtls) rec.key("dtls"); else rec.key("tls");
    w.puts("{\"client\":{");
    Obj cl{w};
    // get_server_name (tls.h:1052-1080): the first SNI extension, past its 5-byte header
    for (mfpe::Cur e = ext; e.len() > 0;) {
        const uint8_t *st = e.d;
        uint64_t t, el;
        if (!e.rd(2, t) || !e.rd(2, el) || !e.skip((long)el)) break;
        if (t == 0) {
            mfpe::Cur sn{st, e.d};
            sn.skip(9);
            if (!sn.null() && sn.len() > 0) { cl.key("server_name"); w.put('"'); w.utf8(sn.d, (size_t)sn.len()); w.put('"'); }
            break;
        }
    }
    for (mfpe::Cur e = ext; e.len() > 0;) {
        const uint8_t *st = e.d;
        uint64_t t, el;
        if (!e.rd(2, t) || !e.rd(2, el) || !e.skip((long)el)) break;
        if (t != 0x0039 && t != 0xffa5) continue;
        if (t == 0x0039) cl.key("quic_transport_parameters"); else cl.key("quic_transport_parameters_draft");
        w.put('"'); w.hexb(st, (size_t)(e.d - st)); w.put('"');
        mfpe::Cur q{st + 4, e.d};
        while (q.len() > 0) {                              // quic_transport_parameter tls.h:1237-1262
            const uint64_t id = vli(q);
            const uint64_t vl = vli(q);
            const mfpe::Cur v = take(q, (long)vl);
            if (id == 0x3129 && !v.null() && v.len() > 0) {
                cl.key("google_user_agent"); w.put('"'); w.utf8(v.d, (size_t)v.len()); w.put('"');
            }
        }
    }
    w.puts("}}");
}

// a QUIC hello's handshake message (tls_handshake::parse tls.h:244-262)
void quic_tls(W &w, Obj &rec, const uint8_t *hs, uint32_t hs_len) {
    mfpe::Cur d{hs, hs + hs_len};
    if (d.len() < 4) return;
    uint64_t mt, hl;
    d.rd(1, mt); d.rd(3, hl);
    if (hl > 32768) return;
    client_hello_json(w, rec, mfpe::Cur{d.d, hl < (uint64_t)d.len() ? d.d + hl : d.e});
}

// The handshake body of a TLS_CH / DTLS_CH record, found again from the
// record's innermost IP header (ip::parse ip.h:619-632): the TCP payload
// (tcp_packet::parse tcpip.h:154-163) through tls_record / tls_handshake
// (tls.h:145-262, as set_tcp_protocol builds the hello, pkt_proc.cc:525-534),
// or the UDP payload (udp.h:89-110) through dtls_record / dtls_handshake
// (dtls.h:19-96, dtls_client_hello dtls.h:121-127).
bool client_hello_body(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, mfpe::Cur &body) {
    const uint32_t ip = r.net & 0xffff;
    if (ip >= caplen) return false;
    mfpe::Cur p{pkt + ip, pkt + caplen};
    uint32_t off = 0;
    int ipv = 0;
    mfpe::ip_parse(p, pkt, off, ipv);
    if (p.null()) return false;
    uint64_t x, l;
    if (r.msg == MFP_MSG_TLS_CH) {
        if (p.len() < 20) return false;
        const long opt = (long)(p.d[12] >> 4) * 4 - 20;
        p.d += 20;
        if (!p.skip(opt)) return false;
        if (p.len() < 5) return false;
        p.rd(1, x); p.rd(2, x); p.rd(2, l);
        mfpe::Cur frag{p.d, p.d + std::min<long>((long)l, p.len())};
        if (frag.len() < 4) return false;
        frag.rd(1, x); frag.rd(3, l);
        if (l > 32768) return false;
        body = mfpe::Cur{frag.d, frag.d + std::min<long>((long)l, frag.len())};
        return true;
    }
    if (!p.skip(8) || p.len() < 13) return false;
    p.rd(1, x); p.rd(2, x); p.rd(2, x); p.rd(6, x); p.rd(2, l);
    mfpe::Cur frag = take(p, (long)l);
    if (frag.null() || frag.len() < 12) return false;
    frag.rd(1, x); frag.rd(3, x); frag.rd(2, x); frag.rd(3, x); frag.rd(3, l);
    body = take(frag, (long)l);
    return !body.null();
}

bool write_quic(W &w, Obj &rec, const QuicJson &q) {
    static const char *salts[6] = {"d22", "d23_d28", "d29_d32", "d33_v1", "d1_d7_v2", "v2"};
    if (q.hello && q.hs_len) quic_tls(w, rec, q.hs, q.hs_len);
    // quic_initial_packet::write_json quic.h:531-540, fields re-read from the long header
    mfpe::Cur d{q.pay, q.pay + q.pay_len};
    uint64_t ci = 0, n = 0;
    d.rd(1, ci);
    const mfpe::Cur ver = take(d, 4);
    d.rd(1, n);
    const mfpe::Cur dcid = take(d, (long)n);
    d.rd(1, n);
    const mfpe::Cur scid = take(d, (long)n);
    const uint64_t tl = vli(d);
    const mfpe::Cur token = take(d, (long)tl);
    auto hex = [&](const mfpe::Cur &c) { w.put('"'); if (!c.null() && c.len() > 0) w.hexb(c.d, (size_t)c.len()); w.put('"'); };
    rec.key("quic");
    w.put('{');
    Obj qo{w};
    qo.key("connection_info");
    w.put('"'); for (int b = 7; b >= 0; b--) w.put((ci >> b) & 1 ? '1' : '0'); w.put('"');
    qo.key("version"); hex(ver);
    qo.key("dcid"); hex(dcid);
    qo.key("scid"); hex(scid);
    qo.key("token"); hex(token);
    if (q.cc_off != 0xffff && q.cc_off < q.pt_len) quic_cc(w, qo, q.pt + q.cc_off, q.pt + q.pt_len);
    if (q.pt_len) {
        if (!q.pre && q.salt < 6) { qo.key("salt_string"); w.put('"'); w.putz(salts[q.salt]); w.put('"'); }   // quic.h:905-907
        qo.key("plaintext"); w.put('"'); w.hexb(q.pt, q.pt_len); w.put('"');
    } else {
        qo.key("raw_packet_data"); w.put('"'); w.hexb(q.pay, q.pay_len); w.put('"');
    }
    w.put('}');
    return true;
}

bool write_record(Out &o, TsCache &tc, const uint8_t *pkt, uint32_t caplen, uint32_t linktype, const mfp_record &r,
                  const char *fp_arena,
                  uint64_t sec, uint64_t nsec, mfp_context ctx, const mfp_analysis *an, const double *ap,
                  uint16_t props) {
    if (!(r.flags & MFP_FLAG_EMIT)) return true;
    // QUIC records: the "tls" and "quic" objects from k_quic's sidecar
    QuicJson qj;
    if (r.msg == MFP_MSG_QUIC && !quic_block(pkt, caplen, r, fp_arena, qj)) return false;

    const uint32_t ip = r.net & 0xffff, ipv = (r.net >> 16) & 15;
    // the encapsulation levels above the innermost IP header (IP-in-IP, GRE,
    // VXLAN, Geneve), found again from the link layer (mfp_encap.hpp)
    mfpe::Chain chain;
    if ((r.flags & MFP_FLAG_ENCAP) && (!mfpe::walk(pkt, caplen, linktype, ip, chain) || chain.n == 0)) return false;
    if ((ipv != 4 && ipv != 6) || ip + (ipv == 4 ? 20u : 40u) > caplen) return false;
    // worst case: fixed keys/addresses/numbers and 4 encapsulations < 1000 B, the fp string, and at most
    // 6 output bytes per input byte of a JSON string ("\\ufffd") or a base64 cert list
    const bool with_an = ctx && an && (an->flags & MFP_AN_VALID);
    const size_t sni_x = r.msg == MFP_MSG_STUN ? 32 : r.msg == MFP_MSG_OPENVPN ? 16 : 6;   // object text per input byte
    o.need(1000 + (size_t)r.fp_len + sni_x * (r.sni_len == 0xffff ? 0 : r.sni_len) +
           6 * (r.ua_len == 0xffff ? 0 : r.ua_len) +
           (r.msg == MFP_MSG_QUIC ? 2 * (size_t)(qj.pay_len + qj.pt_len) + 6 * (size_t)qj.hs_len + 600 : 0) +
           (r.msg == MFP_MSG_TLS_CH || r.msg == MFP_MSG_DTLS_CH ? 8 * (size_t)caplen : 0) +
           (with_an ? analysis_bound(ctx, *an) : 0));
    W w{o.buf.get() + o.len};
    // a readable, non-empty datum (print_key_json_string skips empty ones, json_object.h:104-108)
    auto span_ok = [&](uint32_t off, uint32_t len) { return len != 0xffff && len && (uint64_t)off + len <= caplen; };

    w.put('{');
    Obj rec{w};
    if (r.fp_type) {
        rec.key("fingerprints");
        w.put('{'); w.put('"'); w.putz(fp_type_name(r.fp_type)); w.puts("\":\"");
        w.mem(fp_arena + r.fp_offset, r.fp_len); w.puts("\"}");
    }
    switch (r.msg) {
    case MFP_MSG_TLS_CH:
    case MFP_MSG_DTLS_CH: {
        // the hello's own parse (the record's sni span is the classifier's,
        // the last server_name extension)
        mfpe::Cur body{nullptr, nullptr};
        if (!(r.flags & MFP_FLAG_NO_CIPHERS) && client_hello_body(pkt, caplen, r, body)) client_hello_json(w, rec, body);
        break;
    }
    case MFP_MSG_TLS_SH:
    case MFP_MSG_TLS_CERT:
        if (span_ok(r.sni_off, r.sni_len)) {
            const char *role = r.msg == MFP_MSG_TLS_SH ? "server"
                             : (r.flags & MFP_FLAG_CERT_CLIENT) ? "client"
                             : (r.flags & MFP_FLAG_CERT_SERVER) ? "server" : "undetermined";
            rec.key("tls");
            w.puts("{\""); w.putz(role); w.puts("\":{\"certs\":[");
            // tls_server_certificate::for_each_certificate tls.h:2152-2181
            const uint8_t *p = pkt + r.sni_off, *e = p + r.sni_len;
            bool first = true;
            while (p < e) {
                if (e - p < 3) break;
                uint64_t l = ((uint64_t)p[0] << 16) | ((uint64_t)p[1] << 8) | p[2];
                p += 3;
                if (l > (uint64_t)(e - p)) l = (uint64_t)(e - p);
                if (l == 0) break;
                if (!first) w.put(',');
                first = false;
                w.puts("{\"base64\":"); w.base64(p, l); w.put('}');
                p += l;
            }
            w.puts("]}}");
        }
        break;
    case MFP_MSG_QUIC:
        write_quic(w, rec, qj);
        break;
    case MFP_MSG_DTLS_SH:                                // write_metadata pkt_proc_util.h:315-321
        rec.key("dtls");
        w.puts("{\"server\":{}}");
        break;
    case MFP_MSG_STUN:                                   // stun::message::write_json (stun.h:795)
        if (span_ok(r.sni_off, r.sni_len) && r.sni_len >= 20) { rec.key("stun"); write_stun(w, pkt + r.sni_off, r.sni_len); }
        break;
    case MFP_MSG_OPENVPN:                                // openvpn_tcp::write_json (openvpn.h:411)
        if (span_ok(r.sni_off, r.sni_len) && !write_openvpn(w, rec, pkt + r.sni_off, r.sni_len)) return false;
        break;
    case MFP_MSG_HTTP_REQ:
        rec.key("http");
        w.puts("{\"request\":{");
        if (span_ok(r.ua_off, r.ua_len)) { w.puts("\"user_agent\":\""); w.utf8(pkt + r.ua_off, r.ua_len); w.put('"'); }
        w.puts("}}");
        break;
    default:
        break;
    }
    if (with_an) { rec.key("analysis"); write_analysis(w, ctx, *an, ap); }   // pkt_proc.cc:1211-1213
    if (props & 1) { rec.key("reassembly_properties"); write_reassembled(w, props); }   // reassembly.hpp:1238-1241
    else if (r.flags & MFP_FLAG_TRUNCATED) { rec.key("reassembly_properties"); w.puts("{\"truncated\":true}"); }
    if (r.flags & MFP_FLAG_ENCAP) {                      // encapsulations::write_json pkt_proc.cc:1033-1043
        static const char *type[4] = {"ip encapsulation", "gre", "vxlan", "geneve"};
        rec.key("encapsulations");
        w.put('[');
        for (int k = 0; k < chain.n; k++) {               // ip.h:788-793, gre.h:69-75, vxlan.hpp:60-68, geneve.hpp:85-91
            const mfpe::Level &L = chain.lv[k];
            const uint8_t *oh = pkt + L.ip_off;
            if (k) w.put(',');
            w.puts("{\"type\":\""); w.putz(type[L.kind]); w.puts("\",\"src_ip\":\"");   // key::write_ip_address
            if (L.ipv == 4) w.ipv4(oh + 12); else w.ipv6(oh + 8);
            w.puts("\",\"dst_ip\":\"");
            if (L.ipv == 4) w.ipv4(oh + 16); else w.ipv6(oh + 24);
            w.put('"');
            if (L.kind == mfpe::GRE || L.kind == mfpe::GENEVE) { w.puts(",\"protocol_type\":"); w.udec(L.proto_type); }
            w.put('}');
        }
        w.put(']');
    }
    const uint8_t *iph = pkt + ip;
    rec.key("src_ip"); w.put('"');
    if (ipv == 4) w.ipv4(iph + 12); else w.ipv6(iph + 8);
    w.put('"');
    rec.key("dst_ip"); w.put('"');
    if (ipv == 4) w.ipv4(iph + 16); else w.ipv6(iph + 24);
    w.put('"');
    rec.key("protocol"); w.u8dec(is_tcp_msg(r.msg) ? 6 : 17);
    rec.key("src_port"); w.udec(r.src_port);
    rec.key("dst_port"); w.udec(r.dst_port);
    rec.key("event_start");
    if (sec != tc.sec || nsec / 1000 != tc.usec) {      // consecutive packets share most timestamps
        W t{tc.text};
        t.timestamp(sec, nsec);
        tc.sec = sec; tc.usec = nsec / 1000; tc.len = (int)(t.p - tc.text);
    }
    w.mem(tc.text, (size_t)tc.len);
    w.puts("}\n");
    o.len = (size_t)(w.p - o.buf.get());
    return true;
}

}  // namespace

// The ALPN protocol_name_list of a (D)TLS ClientHello record, re-read from the
// packet (tls_extensions::set_meta_data tls.h:1357-1362: the last ALPN
// extension; a list shorter than its length field is none) -- for records
// whose ua span holds a draft user agent instead (MFP_XF_TLS_UA).
bool mfp_hello_alpn(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, const uint8_t **alpn, uint32_t *len) {
    *alpn = nullptr; *len = 0;
    mfpe::Cur body{nullptr, nullptr}, ext;
    bool ciphers_ok = false, dtls = false;
    if (!client_hello_body(pkt, caplen, r, body) || !hello_extensions(body, ext, ciphers_ok, dtls)) return false;
    bool found = false;
    for (mfpe::Cur e = ext; e.len() > 0;) {
        const uint8_t *st = e.d;
        uint64_t t, el;
        if (!e.rd(2, t) || !e.rd(2, el) || !e.skip((long)el)) break;
        if (t != 16) continue;
        mfpe::Cur a{st + 4, e.d};
        uint64_t al = 0;
        found = a.rd(2, al) && (uint64_t)a.len() >= al;
        if (found) { *alpn = a.d; *len = (uint32_t)al; }
        else { *alpn = nullptr; *len = 0; }
    }
    return found;
}

// sink != nullptr: the threads' parts go to sink in packet order instead of
// into out (the batch packet processors, mfp_pktproc.cpp); out_cap unused
static long long write_json_batch(mfp_context ctx, const uint16_t *props, const uint8_t *arena, const mfp_pkt_desc *desc,
                                   size_t n,
                                   const mfp_record *rec, const char *fp_arena, const mfp_analysis *an, const double *ap,
                                   const uint64_t *ts_ns, char *out, size_t out_cap, uint64_t *line_end,
                                   uint64_t *skipped, int threads, mfp_json_sink sink = nullptr, void *user = nullptr) {
    if ((n && (!arena || !desc || !rec || !fp_arena || !line_end)) || (out_cap && !out && !sink)) {
        mfp_set_error("mfp_write_json_batch: null argument");
        return -1;
    }
    struct timespec now{};
    clock_gettime(CLOCK_REALTIME, &now);     // pkt_proc.cc:1086-1089: tv_sec == 0 means "now"
    if (threads <= 0) threads = 1;
    if ((size_t)threads > n / 4096 + 1) threads = (int)(n / 4096 + 1);
    // per-thread output buffers are kept between calls: a fresh multi-GB
    // allocation per batch costs more in page faults than the formatting
    static std::mutex pool_mu;
    static std::vector<Out> pool;
    std::vector<Out> part;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        part.swap(pool);                       // a concurrent caller finds the pool empty and allocates
    }
    part.resize((size_t)threads);
    for (auto &o : part) o.len = 0;
    std::vector<uint64_t> bad((size_t)threads, 0);
    const size_t per = (n + threads - 1) / (threads ? threads : 1);
    auto run = [&](auto &&fn) {
        if (threads == 1) { fn(0); return; }
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(fn, t);
        for (auto &x : th) x.join();
    };
    run([&](int t) {
        size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
        Out o = std::move(part[(size_t)t]);   // thread-local copy: no shared lines while formatting
        TsCache tc;
        o.need((hi > lo ? hi - lo : 0) * 320 + 65536);   // exact; grows x1.5 if the records are longer
        for (size_t i = lo; i < hi; i++) {
            uint64_t sec = 0, nsec = 0;
            if (ts_ns) { sec = ts_ns[i] / 1000000000ull; nsec = ts_ns[i] % 1000000000ull; }
            if (sec == 0) { sec = (uint64_t)now.tv_sec; nsec = (uint64_t)now.tv_nsec; }
            size_t mark = o.len;
            if (!write_record(o, tc, arena + desc[i].offset, desc[i].caplen, desc[i].linktype, rec[i], fp_arena, sec, nsec,
                              ctx,
                              an ? an + i : nullptr, ap ? ap + i * MFP_ATTR_DB_TAGS : nullptr, props ? props[i] : (uint16_t)0)) {
                o.len = mark;
                bad[(size_t)t]++;
            }
            line_end[i] = o.len;               // thread-local for now, rebased below
        }
        part[(size_t)t] = std::move(o);
    });
    uint64_t total = 0, nbad = 0;
    std::vector<uint64_t> base((size_t)threads, 0);
    for (int t = 0; t < threads; t++) { base[(size_t)t] = total; total += part[(size_t)t].len; nbad += bad[(size_t)t]; }
    if (skipped) *skipped = nbad;
    auto give_back = [&]() {
        // keep buffers for the next call (page faults on a fresh multi-GB
        // buffer cost more than the formatting), but not oversized ones: a
        // huge batch must not pin its footprint for the life of the process
        static const size_t kKeep = (size_t)256 << 20;
        for (auto &o : part) if (o.cap > kKeep) { o.buf.reset(); o.cap = 0; }
        std::lock_guard<std::mutex> lk(pool_mu);
        if (pool.size() < part.size()) pool.swap(part);
    };
    if (sink) {
        for (int t = 1; t < threads; t++) {   // line ends in the stream of this call
            const size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
            for (size_t i = lo; i < hi; i++) line_end[i] += base[(size_t)t];
        }
        for (int t = 0; t < threads; t++)
            if (part[(size_t)t].len && sink(user, part[(size_t)t].buf.get(), part[(size_t)t].len) != 0) {
                give_back();
                mfp_set_error("JSON output: the sink failed");
                return -3;
            }
        give_back();
        return (long long)total;
    }
    if (total > out_cap) {
        give_back();
        mfp_set_error("mfp_write_json_batch: output buffer too small (need %llu bytes)", (unsigned long long)total);
        return -2;
    }
    run([&](int t) {                           // each thread places its own part
        size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
        for (size_t i = lo; i < hi; i++) line_end[i] += base[(size_t)t];
        if (part[(size_t)t].len) memcpy(out + base[(size_t)t], part[(size_t)t].buf.get(), part[(size_t)t].len);
    });
    give_back();
    return (long long)total;
}

MFP_EXPORT long long mfp_write_json_batch(const uint8_t *arena, const mfp_pkt_desc *desc, size_t n,
                                          const mfp_record *rec, const char *fp_arena, const uint64_t *ts_ns,
                                          char *out, size_t out_cap, uint64_t *line_end, uint64_t *skipped,
                                          int threads) {
    return write_json_batch(nullptr, nullptr, arena, desc, n, rec, fp_arena, nullptr, nullptr, ts_ns, out, out_cap, line_end,
                            skipped, threads);
}

MFP_EXPORT long long mfp_write_json_batch_analysis(mfp_context ctx, const uint8_t *arena, const mfp_pkt_desc *desc,
                                                   size_t n, const mfp_record *rec, const char *fp_arena,
                                                   const mfp_analysis *analysis, const double *attr_prob,
                                                   const uint64_t *ts_ns, char *out, size_t out_cap,
                                                   uint64_t *line_end, uint64_t *skipped, int threads) {
    if (!ctx || !mfp_analysis_enabled(ctx)) {
        mfp_set_error("mfp_write_json_batch_analysis: the context has no classifier");
        return -1;
    }
    if (n && !analysis) { mfp_set_error("mfp_write_json_batch_analysis: null analysis"); return -1; }
    if (!attr_prob)   // an archive tag on any record needs its probability
        for (size_t i = 0; i < n; i++)
            if ((analysis[i].flags & MFP_AN_VALID) && (analysis[i].attr >> MFP_ATTR_DB_FIRST)) {
                mfp_set_error("mfp_write_json_batch_analysis: record %zu carries archive tags but attr_prob is NULL", i);
                return -1;
            }
    return write_json_batch(ctx, nullptr, arena, desc, n, rec, fp_arena, analysis, attr_prob, ts_ns, out, out_cap,
                            line_end, skipped, threads);
}

// the records of mfp_process_batch_reassembly: arena ++ its frames with its
// out_desc, and its props (the reassembler's "reassembly_properties")
MFP_EXPORT long long mfp_write_json_batch_reassembly(const uint8_t *arena, const mfp_pkt_desc *desc, size_t n,
                                                     const mfp_record *rec, const char *fp_arena, const uint16_t *props,
                                                     const uint64_t *ts_ns, char *out, size_t out_cap,
                                                     uint64_t *line_end, uint64_t *skipped, int threads) {
    if (n && !props) { mfp_set_error("mfp_write_json_batch_reassembly: null props"); return -1; }
    return write_json_batch(nullptr, props, arena, desc, n, rec, fp_arena, nullptr, nullptr, ts_ns, out, out_cap,
                            line_end, skipped, threads);
}

// ... and with the --analysis objects (mfp_process_batch_reassembly_analysis)
MFP_EXPORT long long mfp_write_json_batch_reassembly_analysis(mfp_context ctx, const uint8_t *arena,
                                                              const mfp_pkt_desc *desc, size_t n, const mfp_record *rec,
                                                              const char *fp_arena, const uint16_t *props,
                                                              const mfp_analysis *analysis, const double *attr_prob,
                                                              const uint64_t *ts_ns, char *out, size_t out_cap,
                                                              uint64_t *line_end, uint64_t *skipped, int threads) {
    if (!ctx || !mfp_analysis_enabled(ctx)) { mfp_set_error("the context has no classifier"); return -1; }
    if (n && (!props || !analysis)) { mfp_set_error("mfp_write_json_batch_reassembly_analysis: null argument"); return -1; }
    return write_json_batch(ctx, props, arena, desc, n, rec, fp_arena, analysis, attr_prob, ts_ns, out, out_cap,
                            line_end, skipped, threads);
}

// the batch packet processors' form (mfp_pktproc.cpp): any of the four
// writers above, the text handed to sink in packet order
long long mfp_write_json_to_sink(mfp_context ctx, const uint16_t *props, const uint8_t *arena, const mfp_pkt_desc *desc,
                                 size_t n, const mfp_record *rec, const char *fp_arena, const mfp_analysis *analysis,
                                 const double *attr_prob, const uint64_t *ts_ns, uint64_t *line_end, uint64_t *skipped,
                                 int threads, mfp_json_sink sink, void *user) {
    if (analysis && (!ctx || !mfp_analysis_enabled(ctx))) { mfp_set_error("the context has no classifier"); return -1; }
    return write_json_batch(analysis ? ctx : nullptr, props, arena, desc, n, rec, fp_arena, analysis, attr_prob, ts_ns,
                            nullptr, 0, line_end, skipped, threads, sink, user);
}
