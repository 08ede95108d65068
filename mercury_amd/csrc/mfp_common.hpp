// mfp_common.hpp -- code shared by the host classifier loader
// (mfp_classifier.cpp) and the device classifier kernel (mfp_analysis.hip):
// the string hash used by every device hash table, and the server-name
// normalisation of the reference (server_identifier, watchlist.hpp:242-390;
// dns_string watchlist.hpp:27-83; ipv4/ipv6 address strings
// ip_address.hpp:455-880; normalize ip_address.hpp:404-416;
// get_tld_domain_name naive_bayes.hpp:557-576).
//
// Everything here is plain C++ that compiles for the host and for gfx950.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define MFP_HD __host__ __device__ inline
#else
#define MFP_HD inline
#endif

namespace mfpc {

// ---------------------------------------------------------------------------
// string hash: XOR of position-salted 64-bit mixes of the 8-byte words, so
// a wave can hash a string with one word per lane and an XOR reduction
// ---------------------------------------------------------------------------
MFP_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}
#ifdef MFP_PROBE_CHEAPHASH   // (profiling probe only: what the per-word mixing costs; breaks the classifier's keys)
MFP_HD uint64_t word_term(uint64_t w, uint32_t j) { return w + j; }
#else
MFP_HD uint64_t word_term(uint64_t w, uint32_t j) { return mix64(w + (uint64_t)(j + 1) * 0x9e3779b97f4a7c15ULL); }
#endif
MFP_HD uint64_t hash_final(uint64_t acc, uint32_t len) { return mix64(acc ^ ((uint64_t)len * 0x2545f4914f6cdd1dULL)); }
MFP_HD uint64_t load_word(const uint8_t *s, uint32_t len, uint32_t j) {
    uint64_t w = 0;
    for (uint32_t k = 0; k < 8 && 8 * j + k < len; k++) w |= (uint64_t)s[8 * j + k] << (8 * k);
    return w;
}
MFP_HD uint64_t str_hash(const uint8_t *s, uint32_t len) {
    uint64_t acc = 0;
    for (uint32_t j = 0; 8 * j < len; j++) acc ^= word_term(load_word(s, len, j), j);
    return hash_final(acc, len);
}
// key of a feature-table slot: (fingerprint entry, feature kind, value key)
MFP_HD uint64_t feat_slot_hash(uint32_t entry, uint32_t kind, uint64_t key) {
    return mix64(key ^ ((uint64_t)entry << 8 | kind) * 0xd6e8feb86659fd93ULL);
}

enum FeatureKind : uint32_t { F_ASN = 0, F_PORT = 1, F_IPV4 = 2, F_IPV6 = 3, F_UA = 4, F_DOMAIN = 5, F_SNI = 6 };

// ---------------------------------------------------------------------------
// utf8_safe_string<512> (utf8.hpp:1059-1088) as stun::message::do_analysis
// hands the SOFTWARE value to the classifier (stun.h:1021-1036): the text of
// utf8_string::write (utf8.hpp:200-340: JSON escapes, \uXXXX for control
// characters and every non-ASCII codepoint, surrogate pairs above U+FFFF) in a
// 512-byte output_buffer, then strncpy 511.  The buffer's datum is null --
// the user agent empty -- when the input is not valid UTF-8 (write returns
// false) or the text does not fit: append_putc keeps one byte for the NUL
// (buffer_stream.h:134-157) and the four hex digits go through append_memcpy,
// whose bound is strict (doff < dlen - 1 - 4, buffer_stream.h:159-176).
// Writes at most 511 bytes to out; returns the length (0: empty).
// ---------------------------------------------------------------------------
MFP_HD uint32_t utf8_safe_512(const uint8_t *x, uint32_t len, char *out) {
    const char hex[] = "0123456789abcdef";
    uint32_t k = 0;
    bool ok = true;
    auto putc = [&](char c) { if (k < 511) out[k++] = c; else ok = false; };
    auto cp4 = [&](uint32_t c) {
        putc('\\'); putc('u');
        if (ok && k < 507) {
            out[k] = hex[(c >> 12) & 15]; out[k + 1] = hex[(c >> 8) & 15];
            out[k + 2] = hex[(c >> 4) & 15]; out[k + 3] = hex[c & 15];
            k += 4;
        } else {
            ok = false;
        }
    };
    auto cont = [](uint32_t b) { return (b & 0xc0) == 0x80; };
    uint32_t j = 0;
    while (j < len && ok) {
        const uint32_t b0 = x[j];
        if (b0 >= 0x80) {
            if (b0 < 0xc2) return 0;                         // invalid lead byte
            uint32_t cp = 0, n = 0;
            if (b0 >= 0xf0 && b0 <= 0xf4) n = 4;
            else if (b0 >= 0xe0 && b0 <= 0xef) n = 3;
            else if (b0 < 0xe0) n = 2;
            else return 0;                                   // 0xf5..0xff
            if (len - j < n) return 0;                       // sequence too short
            const uint32_t b1 = x[j + 1];
            bool second;                                     // is_second_byte_valid (RFC 3629)
            switch (b0) {
            case 0xe0: second = b1 >= 0xa0 && b1 <= 0xbf; break;
            case 0xed: second = b1 >= 0x80 && b1 <= 0x9f; break;
            case 0xf0: second = b1 >= 0x90 && b1 <= 0xbf; break;
            case 0xf4: second = b1 >= 0x80 && b1 <= 0x8f; break;
            default: second = cont(b1);
            }
            if (!second) return 0;
            if (n == 2) cp = ((b0 & 0x1f) << 6) | (b1 & 0x3f);
            else if (n == 3) {
                if (!cont(x[j + 2])) return 0;
                cp = ((b0 & 0x0f) << 12) | ((b1 & 0x3f) << 6) | (x[j + 2] & 0x3f);
            } else {
                if (!cont(x[j + 2]) || !cont(x[j + 3])) return 0;
                cp = ((b0 & 0x07) << 18) | ((b1 & 0x3f) << 12) | ((uint32_t)(x[j + 2] & 0x3f) << 6) | (x[j + 3] & 0x3f);
            }
            if (cp == 0) return 0;
            if ((cp >= 0xe000 && cp <= 0xf8ff) || (cp >= 0xf0000 && cp <= 0xffffd) || (cp >= 0x100000 && cp <= 0x10fffd) ||
                (cp >= 0xd800 && cp <= 0xdfff))
                return 0;                                    // private use, surrogate half
            if (cp > 0xffff) {
                cp -= 0x10000;
                cp4((cp >> 10) + 0xd800);
                cp4((cp & 0x3ff) + 0xdc00);
            } else {
                cp4(cp);
            }
            j += n;
        } else {
            if (b0 < 0x20 || b0 == 0x7f) cp4(b0);
            else {
                if (b0 == '"' || b0 == '\\') putc('\\');
                putc((char)b0);
            }
            j++;
        }
    }
    return ok ? k : 0;
}

// ---------------------------------------------------------------------------
// server_identifier::get_normalized_domain_name(detail::on)
// input: the server name as the reference's C string sees it (destination
// context strncpy: at most MAX_SNI_LEN-1 = 256 bytes, stops at NUL)
// output: the normalized name, written to out (capacity >= 320)
// ---------------------------------------------------------------------------
MFP_HD bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }
MFP_HD bool is_alpha(uint32_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
MFP_HD bool is_label_char(uint32_t c) { return is_alpha(c) || is_digit(c) || c == '-' || c == '_'; }
MFP_HD int hexval(uint32_t c) {
    if (c >= '0' && c <= '9') return (int)c - '0';
    if (c >= 'a' && c <= 'f') return (int)c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return (int)c - 'A' + 10;
    return -1;
}
MFP_HD int put_str(char *out, int o, const char *s) {
    while (*s) out[o++] = *s++;
    return o;
}
MFP_HD int put_uint(char *out, int o, uint32_t v) {
    char tmp[12];
    int k = 0;
    do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) out[o++] = tmp[--k];
    return o;
}
MFP_HD int put_hex(char *out, int o, uint32_t v) {   // %x
    char tmp[8];
    int k = 0;
    do { uint32_t d = v & 15; tmp[k++] = (char)(d < 10 ? '0' + d : 'a' + d - 10); v >>= 4; } while (v);
    while (k) out[o++] = tmp[--k];
    return o;
}

// ipv4_address_string (ip_address.hpp:474-520): four base256 fields
// separated by dots; a field is zero or more digits with value <= 255
MFP_HD bool parse_ipv4(const uint8_t *s, int len, int &pos, uint32_t &value) {
    int p = pos;
    uint32_t f[4];
    for (int k = 0; k < 4; k++) {
        if (k) {
            if (p < len && s[p] == '.') p++;
            else return false;
        }
        uint32_t v = 0;
        while (p < len && is_digit(s[p])) {
            v = 10 * v + (s[p] - '0');
            if (v > 255) return false;
            p++;
        }
        f[k] = v;
    }
    value = f[0] | f[1] << 8 | f[2] << 16 | f[3] << 24;
    pos = p;
    return true;
}

// ipv6_address_string (ip_address.hpp:643-790) -> 16 address bytes
MFP_HD bool parse_ipv6(const uint8_t *s, int len, int &pos, uint8_t out[16]) {
    int p = pos;
    uint16_t pieces[16];
    int np = 0, dci = -1;
    if (p < len && s[p] == '[') p++;
    while (p < len) {
        if (s[p] == ':') {
            p++;
            if (p < len && s[p] == ':') {
                p++;
                if (dci != -1) return false;
                dci = np;
                // "::ffff:w.x.y.z"
                if (p + 5 <= len && s[p] == 'f' && s[p + 1] == 'f' && s[p + 2] == 'f' && s[p + 3] == 'f' &&
                    s[p + 4] == ':') {
                    if (np != 0) return false;
                    pieces[np++] = 0xffff;
                    int q = p + 5;
                    uint32_t v4;
                    if (parse_ipv4(s, len, q, v4)) {
                        // pieces from the big-endian hex of the address
                        uint32_t be = (v4 & 0xff) << 24 | (v4 >> 8 & 0xff) << 16 | (v4 >> 16 & 0xff) << 8 | (v4 >> 24);
                        pieces[np++] = (uint16_t)(be >> 16);
                        pieces[np++] = (uint16_t)(be & 0xffff);
                        p = q;
                        if (p < len && s[p] == ']') p++;
                        goto build;
                    }
                    p += 5;   // lookahead consumed "ffff:" (ip_address.hpp:686)
                }
            }
        } else {
            if (s[p] == ']') { p++; break; }
            uint32_t v = 0;
            int nd = 0;
            while (p < len && hexval(s[p]) >= 0) { v = 16 * v + (uint32_t)hexval(s[p]); p++; nd++; }
            if (nd == 0 || np >= 15) return false;
            pieces[np++] = (uint16_t)v;
        }
    }
    if (dci == -1) {
        if (np != 8) return false;
    } else if (np > 7) {
        return false;
    }
build: {
        int prefix = dci == -1 ? np : dci, zeros = dci == -1 ? 0 : 8 - np, j = 0;
        for (int i = 0; i < prefix; i++) { out[j++] = (uint8_t)(pieces[i] > 255 ? pieces[i] >> 8 : 0); out[j++] = (uint8_t)pieces[i]; }
        for (int i = 0; i < zeros; i++) { out[j++] = 0; out[j++] = 0; }
        for (int i = prefix; i < np; i++) { out[j++] = (uint8_t)(pieces[i] > 255 ? pieces[i] >> 8 : 0); out[j++] = (uint8_t)pieces[i]; }
    }
    pos = p;
    return true;
}

// normalize() ip_address.hpp:404-416 (private / non-global -> representative)
MFP_HD uint32_t normalize_ipv4(uint32_t v) {
    if ((v & 0xff) == 0x0a || (v & 0xf0ff) == 0x10ac || (v & 0xffff) == 0xa8c0) return 0x0100000a;
    return v;
}
MFP_HD void normalize_ipv6(uint8_t a[16]) {
    bool global_unicast = (a[0] & 0xe0) == 0x20;
    bool mapped = true;
    for (int i = 0; i < 10; i++) mapped &= a[i] == 0;
    mapped &= a[10] == 0xff && a[11] == 0xff;
    if (!(global_unicast || mapped)) {
        for (int i = 0; i < 16; i++) a[i] = 0;
        a[0] = 0xfd;
        a[15] = 1;
    }
}

// append_ipv6_addr buffer_stream.h:534-640, including its run bookkeeping
// (a run that does not beat the longest keeps counting into the next one)
MFP_HD int put_ipv6(char *out, int o, const uint8_t a[16]) {
    uint32_t pc[8];
    for (int i = 0; i < 8; i++) pc[i] = (uint32_t)a[2 * i] << 8 | a[2 * i + 1];
    int run = -1, run_len = 0, longest = -1, longest_len = 0;
    for (int i = 0; i < 8; i++) {
        if (pc[i] == 0) {
            if (run_len == 0) run = i;
            run_len++;
        } else if (run_len != 0 && longest_len < run_len) {
            longest_len = run_len; longest = run; run_len = 0;
        }
    }
    if (longest_len < run_len) { longest_len = run_len; longest = run; }
    if (longest_len == 1) { longest_len = 0; longest = 8; }
    int u = 0;
    const int stop = longest < 0 ? 0 : longest;
    while (u < stop) {
        o = put_hex(out, o, pc[u++]);
        if (u != stop) out[o++] = ':';
    }
    u += longest_len;
    if (longest_len != 0) { out[o++] = ':'; out[o++] = ':'; }
    while (u < 8) {
        o = put_hex(out, o, pc[u++]);
        if (u != 8) out[o++] = ':';
    }
    return o;
}

// The classifier sees a flow's destination as text (key::sprintf_dst_addr
// flow_key.h:206-231, i.e. append_ipv6_addr above) parsed back
// (ipv6_address_string ip_address.hpp:643-880).  With the printer's run
// bookkeeping the "::" can stand for pieces that are not zero, so the
// address it classifies is the packet's with pieces [lr, lr + lr_len) zeroed.
// hi/lo: the address as two big-endian halves.
MFP_HD void v6_text_roundtrip(uint64_t &hi, uint64_t &lo) {
    uint32_t pc[8];
    for (int i = 0; i < 4; i++) {
        pc[i] = (uint32_t)(hi >> (48 - 16 * i)) & 0xffff;
        pc[4 + i] = (uint32_t)(lo >> (48 - 16 * i)) & 0xffff;
    }
    int run = -1, run_len = 0, lr = -1, lr_len = 0;
    for (int i = 0; i < 8; i++) {
        if (pc[i] == 0) {
            if (run_len == 0) run = i;
            run_len++;
        } else if (run_len != 0 && lr_len < run_len) {
            lr_len = run_len; lr = run; run_len = 0;
        }
    }
    if (lr_len < run_len) { lr_len = run_len; lr = run; }
    if (lr_len < 2) return;   // no "::": all eight pieces printed
    for (int i = lr; i < lr + lr_len && i < 8; i++) {
        if (i < 4) hi &= ~((uint64_t)0xffff << (48 - 16 * i));
        else lo &= ~((uint64_t)0xffff << (48 - 16 * (i - 4)));
    }
}

// returns the normalized length; out must hold >= 330 bytes
MFP_HD int normalize_server_name(const uint8_t *s, int len, char *out) {
    int o = 0;
    // C-string view (strncpy into MAX_SNI_LEN=257: at most 256 bytes, NUL stops)
    int n = 0;
    while (n < len && n < 256 && s[n] != 0) n++;
    if (n == 0 || s[0] == '#') return put_str(out, 0, "missing.alt");
    int p = 0;
    while (p < n && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n' || s[p] == '\r' || s[p] == '\v' || s[p] == '\f')) p++;
    // host identifier: 0 none, 1 ipv4, 2 ipv6, 3 dns
    int kind = 0;
    uint32_t v4 = 0;
    uint8_t v6[16];
    int dns_s = 0, dns_e = 0, labels = 0;
    {
        int q = p;
        if (parse_ipv6(s, n, q, v6)) {
            kind = 2;
            p = q;
        }
    }
    if (kind == 0 && p == n) return 0;   // dns_string of an empty remainder: valid, empty name
    if (kind == 0) {
        // dns_string watchlist.hpp:33-70
        int q = p, nl = 0, last_s = -1, last_e = -1;
        bool ok = true;
        if (q < n && s[q] == '*') {
            q++;
            if (q < n && s[q] == '.') { q++; nl++; }
            else ok = false;
        }
        if (ok) {
            while (q < n) {
                int a = q;
                while (q < n && is_label_char(s[q])) q++;
                if (q == a) break;
                last_s = a; last_e = q; nl++;
                if (q < n && s[q] == '.') q++;
                else break;
            }
            bool alpha = false;
            for (int k = last_s; k >= 0 && k < last_e; k++) alpha |= is_alpha(s[k]);
            if (!alpha) ok = false;
        }
        if (ok) {
            kind = 3; dns_s = p; dns_e = last_e; labels = nl;
            p = q;                                   // dns_string stops after a consumed dot
            if (p < n && s[p] == '.') p++;           // server_identifier's optional '.'
        }
    }
    if (kind == 0) {
        int q = p;
        if (parse_ipv4(s, n, q, v4)) { kind = 1; p = q; }
    }
    bool empty = false, have_port = false;
    uint32_t port = 0;
    if (p < n) {
        // port_number watchlist.hpp:86-113: ':' digits (value check only ends parsing)
        if (s[p] == ':' && p + 1 < n && is_digit(s[p + 1])) {
            int q = p + 1;
            while (q < n && is_digit(s[q])) { port = 10 * port + (s[q] - '0'); if (port > 65535) break; q++; }
            have_port = port <= 65535;
            if (have_port) { if (kind == 0) empty = true; }
            else kind = 0;
        } else {
            kind = 0;   // invalid trailing data
        }
    }
    if (have_port) { out[o++] = '_'; o = put_uint(out, o, port & 0xffff); out[o++] = '.'; }
    if (kind == 1) {
        uint32_t a = normalize_ipv4(v4);
        for (int k = 0; k < 4; k++) { o = put_uint(out, o, (a >> (8 * k)) & 0xff); out[o++] = k < 3 ? '-' : '.'; }
        return put_str(out, o, "address.alt");
    }
    if (kind == 2) {
        normalize_ipv6(v6);
        int o0 = o;
        o = put_ipv6(out, o, v6);
        for (int k = o0; k < o; k++) if (out[k] == ':') out[k] = '-';
        out[o++] = '.';
        return put_str(out, o, "address.alt");
    }
    if (kind == 0) return put_str(out, o, empty ? "missing.alt" : "other.alt");
    int dl = dns_e - dns_s;
    if (dl == 4 && s[dns_s] == 'N' && s[dns_s + 1] == 'o' && s[dns_s + 2] == 'n' && s[dns_s + 3] == 'e')
        return put_str(out, o, "missing.alt");
    bool localhost = dl == 9;
    const char *lh = "localhost";
    for (int k = 0; localhost && k < 9; k++) localhost = s[dns_s + k] == (uint8_t)lh[k];
    if (!localhost && labels == 1) return put_str(out, o, "unqualified.alt");
    for (int k = dns_s; k < dns_e; k++) out[o++] = (char)s[k];
    return o;
}

// get_tld_domain_name naive_bayes.hpp:557: offset of the top two labels
MFP_HD int tld_domain_offset(const char *s, int len) {
    int sep = -1, prev = -1;
    for (int k = 0; k < len; k++) {
        if (s[k] == '.') {
            if (sep >= 0) prev = sep;
            sep = k;
        }
    }
    return prev >= 0 ? prev + 1 : 0;
}

}  // namespace mfpc
