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
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "mfp_internal.h"

namespace {

const char HEX[] = "0123456789abcdef";

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
            uint32_t t = ((uint32_t)d[i] << 16) | ((uint32_t)d[i + 1] << 8) | d[i + 2];
            put(T[t >> 18 & 63]); put(T[t >> 12 & 63]); put(T[t >> 6 & 63]); put(T[t & 63]);
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

bool is_tcp_msg(unsigned m) { return m != MFP_MSG_DTLS_CH && m != MFP_MSG_DTLS_SH && m != MFP_MSG_DTLS_HVR; }

// "%f" (json_object::print_key_float json_object.h:174-177)
void put_float(W &w, double d) {
    char t[352];   // %f of the largest double is 316 digits + sign, dot, 6 decimals
    const int n = snprintf(t, sizeof t, "%f", d);
    w.mem(t, n > 0 ? (size_t)n : 0);
}

// worst-case text of a record's "analysis" object
size_t analysis_bound(mfp_context ctx, const mfp_analysis &a) {
    size_t b = 400 + 16 * 64;                       // keys, numbers, 16 attribute entries
    const int na = mfp_attribute_count(ctx);
    for (int k = 0; k < na; k++) { const char *nm = mfp_attribute_name(ctx, (uint32_t)k); b += nm ? strlen(nm) : 0; }
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

bool write_record(Out &o, TsCache &tc, const uint8_t *pkt, uint32_t caplen, const mfp_record &r, const char *fp_arena,
                  uint64_t sec, uint64_t nsec, mfp_context ctx, const mfp_analysis *an, const double *ap,
                  uint16_t props) {
    if (!(r.flags & MFP_FLAG_EMIT)) return true;
    // QUIC records carry a "quic" object with the decrypted payload
    // (quic_init::write_json quic.h:1662-1690), which the device does not return
    if (r.msg == MFP_MSG_QUIC) return false;
    // STUN and OpenVPN records carry "stun" / "openvpn" objects (stun.h:795-826,
    // openvpn.h:411-442) that are not rebuilt here yet
    if (r.msg == MFP_MSG_STUN || r.msg == MFP_MSG_OPENVPN) return false;
    const uint32_t ip = r.net & 0xffff, ipv = (r.net >> 16) & 15;
    // IP-in-IP: outer headers sit back to back before the inner one (IPv4
    // fixed 20 B, ip.h:124-137; IPv6 40 B when it has no extension headers)
    const uint32_t levels = (r.net >> 20) & 7;
    uint32_t outer[4], outer_v[4];
    if (r.flags & MFP_FLAG_ENCAP) {
        if (levels == 0 || levels > 4 || (r.net >> 27) & 1) return false;   // irregular: not rebuilt
        uint32_t at = ip;
        for (int k = (int)levels - 1; k >= 0; k--) {
            outer_v[k] = (r.net >> (23 + k)) & 1 ? 6 : 4;
            const uint32_t sz = outer_v[k] == 6 ? 40 : 20;
            if (at < sz) return false;
            at -= sz;
            outer[k] = at;
        }
    }
    if ((ipv != 4 && ipv != 6) || ip + (ipv == 4 ? 20u : 40u) > caplen) return false;
    // worst case: fixed keys/addresses/numbers and 4 encapsulations < 1000 B, the fp string, and at most
    // 6 output bytes per input byte of a JSON string ("\\ufffd") or a base64 cert list
    const bool with_an = ctx && an && (an->flags & MFP_AN_VALID);
    o.need(1000 + (size_t)r.fp_len + 6 * ((r.sni_len == 0xffff ? 0 : r.sni_len) + (r.ua_len == 0xffff ? 0 : r.ua_len)) +
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
    case MFP_MSG_DTLS_CH:
        if (r.flags & MFP_FLAG_NO_CIPHERS) break;      // tls_client_hello::write_json tls.h:1882-1885
        if (r.msg == MFP_MSG_TLS_CH) rec.key("tls"); else rec.key("dtls");
        w.puts("{\"client\":{");
        if (span_ok(r.sni_off, r.sni_len)) { w.puts("\"server_name\":\""); w.utf8(pkt + r.sni_off, r.sni_len); w.put('"'); }
        w.puts("}}");
        break;
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
    case MFP_MSG_DTLS_SH:                                // write_metadata pkt_proc_util.h:315-321
        rec.key("dtls");
        w.puts("{\"server\":{}}");
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
    if (r.flags & MFP_FLAG_ENCAP) {                      // encapsulations::write_json pkt_proc.cc:1021-1031
        rec.key("encapsulations");
        w.put('[');
        for (uint32_t k = 0; k < levels; k++) {           // ip_encapsulation::write_json ip.h:788-793
            const uint8_t *oh = pkt + outer[k];
            if (k) w.put(',');
            w.puts("{\"type\":\"ip encapsulation\",\"src_ip\":\"");
            if (outer_v[k] == 4) w.ipv4(oh + 12); else w.ipv6(oh + 8);
            w.puts("\",\"dst_ip\":\"");
            if (outer_v[k] == 4) w.ipv4(oh + 16); else w.ipv6(oh + 24);
            w.puts("\"}");
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

static long long write_json_batch(mfp_context ctx, const uint16_t *props, const uint8_t *arena, const mfp_pkt_desc *desc,
                                   size_t n,
                                   const mfp_record *rec, const char *fp_arena, const mfp_analysis *an, const double *ap,
                                   const uint64_t *ts_ns, char *out, size_t out_cap, uint64_t *line_end,
                                   uint64_t *skipped, int threads) {
    if ((n && (!arena || !desc || !rec || !fp_arena || !line_end)) || (out_cap && !out)) {
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
        o.need((hi > lo ? hi - lo : 0) * 320 + 65536);   // grows (x2) if the records are longer
        for (size_t i = lo; i < hi; i++) {
            uint64_t sec = 0, nsec = 0;
            if (ts_ns) { sec = ts_ns[i] / 1000000000ull; nsec = ts_ns[i] % 1000000000ull; }
            if (sec == 0) { sec = (uint64_t)now.tv_sec; nsec = (uint64_t)now.tv_nsec; }
            size_t mark = o.len;
            if (!write_record(o, tc, arena + desc[i].offset, desc[i].caplen, rec[i], fp_arena, sec, nsec, ctx,
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
