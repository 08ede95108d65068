// mfp_wave.hpp -- wave-per-packet fingerprint walker for gfx950.
//
// One 64-lane wavefront owns one packet at a time:
//   * the packet is staged in the wave's LDS slice with coalesced 16-byte
//     loads (whole wave), so every later byte read is an LDS read;
//   * the protocol walk (link -> IP -> TCP/UDP -> protocol identification ->
//     TLS/DTLS/SSH/HTTP/TCP parsers) is WAVE-UNIFORM: every byte it reads is
//     broadcast from LDS and moved to an SGPR (readfirstlane), so all parse
//     control flow is scalar and the wave never diverges;
//   * the fingerprint string is not produced byte by byte during the walk:
//     the walker appends SEGMENTS (raw bytes or hex-encoded bytes of the
//     packet, literals and computed values in a small LDS scratch pool) to a
//     per-wave segment table; afterwards all 64 lanes expand the segments in
//     parallel (8 output characters per lane per round, binary search over
//     the segment ends) and write the string with coalesced 8-byte stores;
//   * variable-length scans (HTTP delimiters, header names, SSH banner) use
//     the whole wave: 64 bytes per step, ballot + find-first-set.
//
// Semantics are those of the reference (file:line cites are relative to
// /root/reference/src/libmerc/) and identical to the lane-per-packet walker
// in mfp_device.hpp, which remains as the fallback lane for packets that do
// not fit this kernel's LDS budget.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mfp.h"
#include "mfp_device.hpp"

namespace mfpw {

#define WDEV __device__ __forceinline__

constexpr int WAVES = 4;            // waves per workgroup
constexpr int PKT_CAP = 2048;       // staged packet bytes (incl. 16-byte alignment slack)
constexpr int SCR_CAP = 768;        // literal / computed-byte pool (last 16 bytes: write sink)
constexpr int SEG_CAP = 256;        // segments per fingerprint
constexpr int MAX_PKT = PKT_CAP - 16;
constexpr uint32_t FP_MAX = 8192;   // fingerprint::MAX_FP_STR_LEN fingerprint.h:15

struct WaveLds {
    uint8_t buf[PKT_CAP + SCR_CAP];  // [0,PKT_CAP) packet, then scratch
    uint64_t cmask[PKT_CAP / 64 + 2];   // HTTP header block: ':' positions per 64-byte chunk
    uint16_t seg_end[SEG_CAP];       // exclusive end (characters) of each segment
    uint32_t seg_info[SEG_CAP];      // src offset in buf | kind << 16
};

enum : uint32_t { K_RAW = 0, K_HEX = 1, K_HEXDG = 2 };

WDEV uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
WDEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
WDEV uint64_t ballot(bool p) { return __ballot(p); }

// cursor == struct datum (datum.h:220-850) over the wave's byte space; d < 0 is null
struct C {
    int d, e;
};
WDEV C cmk(int d, int e) { C c; c.d = d; c.e = e; return c; }
WDEV C cnul() { C c; c.d = -1; c.e = -1; return c; }
WDEV int clen(C c) { return c.d >= 0 ? c.e - c.d : 0; }
WDEV bool cnull(C c) { return c.d < 0; }
WDEV bool cnotempty(C c) { return c.d >= 0 && c.d < c.e; }
WDEV void cset_null(C &c) { c.d = c.e = -1; }

struct Out {
    uint32_t fp_type, msg, flags;
    uint32_t sni_off, sni_len, ua_off, ua_len;
    uint32_t src_port, dst_port;
    uint32_t net;        // innermost IP header offset | version << 16
};
struct Cfg {
    uint32_t select, tls_format, mode;
};
using mfp::SEL_TLS_CH; using mfp::SEL_TLS_SH; using mfp::SEL_TLS_CERT; using mfp::SEL_SSH_CLIENT;
using mfp::SEL_SSH_SERVER; using mfp::SEL_HTTP_REQ; using mfp::SEL_HTTP_RESP; using mfp::SEL_TCP_SYN;
using mfp::SEL_TCP_SYNACK; using mfp::SEL_DTLS; using mfp::wave_xor64;

// ---------------------------------------------------------------------------
// the wave walker: parse state + segment emitter (buffer_stream semantics,
// buffer_stream.h:100-240: a fingerprint longer than FP_MAX-2 is dropped)
// ---------------------------------------------------------------------------
// protocol families a W instance can fingerprint (per-bin specialisations
// keep the hot code of a bin kernel small; a packet of a family that is
// compiled out is handed to the fallback lane, `punt`)
enum : uint32_t { SPEC_TLS = 1, SPEC_SSH = 2, SPEC_HTTP = 4, SPEC_DTLS = 8, SPEC_ALL = 15 };

template <uint32_t SPEC = SPEC_ALL>
struct W {
    WaveLds &L;
    Cfg cfg;
    Out o;
    uint32_t lane;
    // emitter state (all wave-uniform)
    uint32_t n;          // characters produced
    bool last_putc;
    int nseg, scr;
    bool ovf;            // segment table / scratch overflow -> fallback lane
    bool punt;           // protocol family not compiled into this instance -> fallback lane
    // pending (not yet stored) segment
    uint32_t pk_kind;
    int pk_src, pk_len;  // pk_len in source bytes; 0 = none

    WDEV W(WaveLds &l, const Cfg &c) : L(l), cfg(c) {
        lane = lane_id();
        n = 0; last_putc = false; nseg = 0; scr = 0; ovf = false; punt = false; pk_kind = 0; pk_src = 0; pk_len = 0;
        refill(0);
    }

    // ---- uniform byte reads from the staged packet ----
    // A 256-byte window of the packet is held in one VGPR (lane l holds the
    // dword at wbase + 4 l); a uniform read is v_readlane + shift, and only
    // a read outside the window goes back to LDS (one ds_read_b32 per lane).
    uint32_t win;
    int wbase;
    WDEV void refill(int o_) {
        wbase = o_ & ~3;
        const int a = wbase + 4 * (int)lane;
        win = a + 4 <= PKT_CAP + SCR_CAP ? *(const uint32_t *)(L.buf + a) : 0u;
    }
    WDEV uint32_t rdlane(int k) { return (uint32_t)__builtin_amdgcn_readlane((int)win, k); }
    WDEV uint32_t ld(int o_) {
        uint32_t rel = (uint32_t)(o_ - wbase);
        if (rel > 255) { refill(o_); rel = (uint32_t)(o_ - wbase); }
        return (rdlane((int)(rel >> 2)) >> ((rel & 3) * 8)) & 0xff;
    }
    // 4 bytes at o_, little-endian order (byte o_ in bits 0..7)
    WDEV uint32_t ld4le(int o_) {
        uint32_t rel = (uint32_t)(o_ - wbase);
        if (rel > 248) { refill(o_); rel = (uint32_t)(o_ - wbase); }
        uint32_t lo = rdlane((int)(rel >> 2));
        if ((rel & 3) == 0) return lo;
        uint32_t hi = rdlane((int)(rel >> 2) + 1);
        return (uint32_t)((((uint64_t)hi << 32) | lo) >> ((rel & 3) * 8));
    }
    // bswap lowers to v_perm_b32 (VALU); readfirstlane brings the result
    // back to an SGPR so the parse arithmetic that follows stays scalar
    WDEV uint32_t be32(int o_) { return rfl(__builtin_bswap32(ld4le(o_))); }
    WDEV uint32_t be16(int o_) { return be32(o_) >> 16; }
    WDEV uint64_t le8(int o_) { return (uint64_t)ld4le(o_) | ((uint64_t)ld4le(o_ + 4) << 32); }

    // ---- datum operations (datum.h) ----
    WDEV bool cskip(C &c, int k) {                       // datum::skip datum.h:365
        if (c.d < 0) return false;
        if (k > c.e - c.d) { c.d = c.e; return false; }
        c.d += k;
        return true;
    }
    WDEV void cparse(C &dst, C &r, long k) {             // datum::parse datum.h:294
        if (clen(r) < k || k < 0) { cset_null(r); cset_null(dst); return; }
        dst.d = r.d; dst.e = r.d >= 0 ? r.d + (int)k : -1;
        if (r.d >= 0) r.d += (int)k;
    }
    WDEV void cparse_soft(C &dst, C &r, long k) {        // datum::parse_soft_fail datum.h:305
        long l = clen(r);
        if (l < k) k = l;
        dst.d = r.d; dst.e = r.d >= 0 ? r.d + (int)k : -1;
        if (r.d >= 0) r.d += (int)k;
    }
    WDEV uint64_t rd_be(int o_, int k) {                 // k (1..8) bytes, big-endian
        if (k <= 4) return be32(o_) >> (32 - 8 * k);
        return ((uint64_t)be32(o_) << (8 * (k - 4))) | (be32(o_ + 4) >> (32 - 8 * (k - 4)));
    }
    WDEV bool rd_uint(C &c, int k, uint64_t &out) {      // datum::read_uint datum.h:795
        if (c.d >= 0 && c.d + k <= c.e) {
            out = rd_be(c.d, k);
            c.d += k; return true;
        }
        cset_null(c); out = 0; return false;
    }
    WDEV uint32_t rd_u8(C &c) {                          // datum::read_uint8 datum.h:749
        if (c.d >= 0 && c.e > c.d) { uint32_t v = ld(c.d); c.d += 1; return v; }
        cset_null(c); return 0;
    }
    WDEV uint32_t look_u8(C &c) {                        // datum::lookahead_uint8 datum.h:702
        if (c.d >= 0 && c.e > c.d) return ld(c.d);
        cset_null(c); return 0;
    }
    WDEV bool look_uint(C &c, int k, uint64_t &out) {    // datum::lookahead_uint datum.h:712
        if (c.d >= 0 && c.d + k <= c.e) {
            out = rd_be(c.d, k); return true;
        }
        return false;
    }
    WDEV void cinit_outer(C &dst, C &outer, uint64_t len) {   // datum::init_from_outer_parser datum.h:825
        if (!cnotempty(outer)) return;
        int end = (len > (uint64_t)(outer.e - outer.d)) ? outer.e : outer.d + (int)len;
        dst.d = outer.d; dst.e = end; outer.d = end;
    }
    WDEV int cget_ptr(C &c, int k) {                     // datum::get_pointer datum.h:737
        if (c.d >= 0 && c.d + k <= c.e) { int p = c.d; c.d += k; return p; }
        return -1;
    }
    WDEV void ctrim_to_length(C &c, long len) {          // datum::trim_to_length datum.h:383
        if (c.d >= 0 && len <= (long)(c.e - c.d)) c.e = c.d + (int)len;
    }

    // ---- cooperative scans: first offset in [a, e) whose byte satisfies P ----
    template <class P>
    WDEV int scan(int a, int e, P pred) {
        for (int base = a; base < e; base += 64) {
            int q = base + (int)lane;
            uint32_t c = L.buf[q < e ? q : base];
            uint64_t m = ballot(q < e && pred(c));
            if (m) return base + (int)__builtin_ctzll(m);
        }
        return e;
    }
    WDEV void cparse_to_delim(C &dst, C &r, uint32_t delim) {   // datum::parse_up_to_delim datum.h:313
        if (!cnotempty(r)) { cset_null(r); cset_null(dst); return; }
        dst.d = r.d;
        int q = scan(r.d, r.e, [=](uint32_t c) { return c == delim; });
        if (q < r.e) { dst.e = r.d = q; return; }
        dst.e = r.e;
    }
    WDEV uint32_t cparse_to_delims(C &dst, C &r, uint32_t d1, uint32_t d2) {   // datum.h:328
        dst.d = r.d;
        if (r.d >= 0) {
            int q = scan(r.d, r.e, [=](uint32_t c) { return c == d1 || c == d2; });
            if (q < r.e) { dst.e = r.d = q; return ld(q); }
            r.d = r.e;
        }
        dst.e = r.e;
        return 0;
    }
    // datum::compare_nbytes datum.h:873 (byte ranges inside buf)
    WDEV bool ccompare_n(C c, int x, int k) {
        if (!(c.d >= 0 && clen(c) >= k)) return false;
        for (int base = 0; base < k; base += 64) {
            int j = base + (int)lane;
            int jj = j < k ? j : 0;
            bool bad = j < k && L.buf[c.d + jj] != L.buf[x + jj];
            if (ballot(bad)) return false;
        }
        return true;
    }
    // datum::cmp datum.h:456
    WDEV int ccmp(C a, C b) {
        if (cnull(a)) return cnull(b) ? 0 : -1;
        if (cnull(b)) return 1;
        int la = clen(a), lb = clen(b), m = la < lb ? la : lb;
        for (int base = 0; base < m; base += 64) {
            int j = base + (int)lane;
            int jj = j < m ? j : 0;
            bool diff = j < m && L.buf[a.d + jj] != L.buf[b.d + jj];
            uint64_t bm = ballot(diff);
            if (bm) {
                int k = base + (int)__builtin_ctzll(bm);
                return (int)ld(a.d + k) - (int)ld(b.d + k);
            }
        }
        return la - lb;
    }

    // ---- emitter ----
    WDEV void seg_store(uint32_t end_chars) {
        if (nseg >= SEG_CAP) { ovf = true; return; }
        // every lane stores the same value: no exec-mask region in the walk
        L.seg_end[nseg] = (uint16_t)end_chars;
        L.seg_info[nseg] = (uint32_t)pk_src | (pk_kind << 16);
        nseg++;
    }
    WDEV void add(uint32_t kind, int src, int len) {
        if (len <= 0) return;
        uint32_t chars = kind == K_RAW ? (uint32_t)len : 2u * (uint32_t)len;
        if (n + chars > FP_MAX) { n += chars; pk_len = 0; return; }   // dropped anyway
        if (pk_len && pk_kind == kind && pk_src + pk_len == src) {
            pk_len += len;
        } else {
            if (pk_len) seg_store(n);
            pk_kind = kind; pk_src = src; pk_len = len;
        }
        n += chars;
    }
    WDEV void flush() {
        if (pk_len && n <= FP_MAX) seg_store(n);
        pk_len = 0;
    }
    // write k (1..8) bytes of v (little-endian) to the scratch pool as RAW
    WDEV void raw_bytes(uint64_t v, int k) {
        if (scr + k > SCR_CAP - 16) { ovf = true; n += (uint32_t)k; return; }
        // lanes >= k store into the sink at the end of the scratch pool.  The
        // lane id goes through an opaque move so the per-lane byte shifts of
        // literal strings are not hoisted out of the packet loop (LICM would
        // keep one VGPR pair per literal live across the whole kernel).
        uint32_t ln;
        asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
        const int dst = (int)ln < k ? PKT_CAP + scr + (int)ln : PKT_CAP + SCR_CAP - 16;
        L.buf[dst] = (uint8_t)(v >> (8 * (ln & 7)));
        add(K_RAW, PKT_CAP + scr, k);
        scr += k;
    }
    WDEV void putc(uint32_t c) { raw_bytes(c & 0xff, 1); last_putc = true; }
    WDEV void put2(uint32_t c0, uint32_t c1) { raw_bytes((c0 & 0xff) | ((c1 & 0xff) << 8), 2); last_putc = true; }
    WDEV static uint32_t hexc(uint32_t nib) { return nib + (nib < 10 ? '0' : 'a' - 10); }
    WDEV void hex(int src, int len) {                    // raw_as_hex buffer_stream.h:1087
        if (src < 0 || len <= 0) return;
        last_putc = false;
        add(K_HEX, src, len);
    }
    WDEV void hex_c(C c) { if (!cnull(c)) hex(c.d, clen(c)); }
    WDEV void hex16(uint32_t v) {                        // append_uint16_hex buffer_stream.h:425
        last_putc = false;
        uint64_t w = (uint64_t)hexc((v >> 12) & 15) | ((uint64_t)hexc((v >> 8) & 15) << 8) |
                     ((uint64_t)hexc((v >> 4) & 15) << 16) | ((uint64_t)hexc(v & 15) << 24);
        raw_bytes(w, 4);
        last_putc = false;
    }
    WDEV void hex8(uint32_t v) {
        raw_bytes((uint64_t)hexc((v >> 4) & 15) | ((uint64_t)hexc(v & 15) << 8), 2);
        last_putc = false;
    }
    WDEV void lit(const char *s) {
        uint64_t w = 0; int k = 0;
        for (; *s; s++) {
            w |= (uint64_t)(uint8_t)*s << (8 * k);
            if (++k == 8) { raw_bytes(w, 8); w = 0; k = 0; }
        }
        if (k) raw_bytes(w, k);
        last_putc = false;
    }
    // valid iff no append truncated (same rule as mfp::Em::valid)
    WDEV bool valid() const { return n <= FP_MAX - 2 || (n == FP_MAX - 1 && last_putc); }

    // raw_as_hex_degrease tls.h:802 (odd trailing byte dropped)
    WDEV void hex_degrease(int src, int len) {
        if (src < 0 || len <= 0) return;
        if (len & 1) len--;
        if (len <= 0) return;
        last_putc = false;
        add(K_HEXDG, src, len);
    }

    // =======================================================================
    // TLS (tls.h)
    // =======================================================================
    struct Ext {
        uint32_t type, length, encoded_type;
        int type_ptr, length_ptr;
        C value;
        bool ok;
    };
    WDEV Ext ext_parse(C &p) {                           // tls_extension ctor tls.h:1383
        Ext x;
        x.type = x.length = x.encoded_type = 0;
        x.type_ptr = p.d; x.length_ptr = -1; x.ok = false; cset_null(x.value);
        uint64_t v;
        if (!rd_uint(p, 2, v)) return x;
        x.type = (uint32_t)v;
        x.length_ptr = p.d;
        if (!rd_uint(p, 2, v)) return x;
        x.length = (uint32_t)v;
        if ((long)x.length <= clen(p)) {
            x.value.d = p.d; x.value.e = p.d + (int)x.length; p.d += (int)x.length; x.ok = true;
        }
        x.encoded_type = ((x.type & 0x0f0f) == 0x0a0a) ? 0x0a0a : x.type;
        return x;
    }
    WDEV void ext_degreased_value(const Ext &x, int ungreased) {   // tls.h:1513
        if (!cnotempty(x.value)) return;
        int vl = clen(x.value), skip, gl;
        if (ungreased < vl) { skip = ungreased; gl = vl - ungreased; } else { skip = vl; gl = 0; }
        hex(x.value.d, skip);
        hex_degrease(x.value.d + skip, gl);
    }
    // QUIC transport parameters (tls.h:1237-1262, quic_vli.hpp)
    WDEV static int vli_len(uint32_t b) {
        return (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1;
    }
    WDEV uint64_t vli_value(C c) {
        uint32_t b = rd_u8(c);
        int len = vli_len(b);
        uint64_t v = b & 0x3f;
        for (int i = 1; i < len; i++) v = v * 256 + rd_u8(c);
        return v;
    }
    WDEV bool qtp_parse(C &d, C &id) {                   // quic_transport_parameter ctor tls.h:1247
        uint32_t b = look_u8(d);
        cparse(id, d, vli_len(b));
        uint32_t bb = rd_u8(d);
        int l2 = vli_len(bb);
        uint64_t v = bb & 0x3f;
        for (int i = 1; i < l2; i++) v = v * 256 + rd_u8(d);
        C val;
        long vlen = (v > 0x7fffffffffffffffULL) ? -1 : (long)v;
        cparse(val, d, vlen);
        return !cnull(val);
    }
    WDEV bool qtp_is_grease(C id) { return vli_value(id) % 31 == 27; }
    WDEV void qtp_write_id(C id) {
        if (!qtp_is_grease(id)) hex(id.d, clen(id));
        else put2('1', 'b');
    }
    WDEV bool qtp_less(C a, C b) {                       // fmt-1 id comparator tls.h:1453
        bool ga = qtp_is_grease(a), gb = qtp_is_grease(b);
        if (ga) { if (gb) return false; return 0x1b < vli_value(b); }
        if (gb) return vli_value(a) < 0x1b;
        return ccmp(a, b) < 0;
    }
    // tls_extension::fingerprint_format1 tls.h:1413
    WDEV void ext_fp1(Ext &x, int role) {
        if (mfp::is_static_ext(x.type)) {
            if (x.type == 0x000a || x.type == 0x002b) {
                putc('('); hex16(x.encoded_type);
                if (x.length_ptr >= 0) hex_degrease(x.length_ptr, 2);
                ext_degreased_value(x, x.type == 0x000a ? 2 : (role == 0 ? 1 : 0));
                putc(')');
            } else if (x.type == 0x39 || x.type == 0xffa5) {
                put2('(', '('); hex16(x.encoded_type); putc(')');
                putc('[');
                C prev = cnul();
                bool have_prev = false;
                long prev_pos = -1;
                while (true) {
                    C best = cnul(); long best_pos = -1;
                    C v = x.value; long pos = 0;
                    while (!cnull(v)) {
                        C id;
                        bool ok = qtp_parse(v, id);
                        if (ok) {
                            bool after = !have_prev || qtp_less(prev, id) || (!qtp_less(id, prev) && pos > prev_pos);
                            if (after) {
                                bool better = best_pos < 0 || qtp_less(id, best) || (!qtp_less(best, id) && pos < best_pos);
                                if (better) { best = id; best_pos = pos; }
                            }
                            pos++;
                        }
                    }
                    if (best_pos < 0) break;
                    putc('('); qtp_write_id(best); putc(')');
                    prev = best; prev_pos = best_pos; have_prev = true;
                }
                putc(']');
                putc(')');
            } else {
                putc('('); hex16(x.encoded_type);
                if (x.length_ptr >= 0) hex_degrease(x.length_ptr, 2);
                if (cnotempty(x.value)) hex(x.value.d, clen(x.value));
                putc(')');
            }
        } else {
            putc('('); hex16(x.encoded_type); putc(')');
        }
    }
    // format 0: tls_extensions::fingerprint tls.h:1549
    WDEV void exts_fp0(C exts, int role) {
        C p = exts;
        putc('(');
        while (clen(p) > 0 && !ovf) {
            Ext x = ext_parse(p);
            if (!x.ok) break;
            if (mfp::is_static_ext(x.type)) {
                if (x.type == 0x000a || x.type == 0x002b) {
                    putc('(');
                    hex_degrease(x.type_ptr, 2);
                    if (x.length_ptr >= 0) hex_degrease(x.length_ptr, 2);
                    ext_degreased_value(x, x.type == 0x000a ? 2 : (role == 0 ? 1 : 0));
                    putc(')');
                } else if (x.type == 0x39 || x.type == 0xffa5) {
                    put2('(', '(');
                    hex_degrease(x.type_ptr, 2);
                    put2(')', '(');
                    C v = x.value;
                    while (!cnull(v)) {
                        C id;
                        if (qtp_parse(v, id)) { putc('('); qtp_write_id(id); putc(')'); }
                    }
                    put2(')', ')');
                } else {
                    putc('(');
                    hex_degrease(x.type_ptr, 2);
                    if (x.length_ptr >= 0) hex_degrease(x.length_ptr, 2);
                    if (cnotempty(x.value)) hex(x.value.d, clen(x.value));
                    putc(')');
                }
            } else {
                // "(" + degreased type + ")" as one computed RAW run
                uint32_t t = mfp::degrease16(x.type);
                uint64_t w = (uint64_t)'(' | ((uint64_t)hexc((t >> 12) & 15) << 8) | ((uint64_t)hexc((t >> 8) & 15) << 16) |
                             ((uint64_t)hexc((t >> 4) & 15) << 24) | ((uint64_t)hexc(t & 15) << 32) | ((uint64_t)')' << 40);
                raw_bytes(w, 6);
                last_putc = true;
            }
        }
        putc(')');
    }
    // formats 1 and 2: kept extensions in lanes, rank by the reference's
    // comparator (tls.h:1637-1655, 1709-1724), emit in rank order
    WDEV void exts_fp12(C exts, int role, int fmt) {
#ifdef MFP_PROBE_NOFMT12
        return;
#endif
        putc('[');
        uint32_t my_key = 0xffffffffu;
        int my_off = 0, nk = 0;
        C p = exts;
        while (clen(p) > 0) {
            int start = p.d;
            Ext x = ext_parse(p);
            if (!x.ok) break;
            int bucket = 0;
            if (fmt == 2) {
                bucket = mfp::fmt2_bucket_t(x.type, x.encoded_type);
                if (bucket < 0) continue;
                // keep the first three per bucket (tls.h:1695-1701)
                uint64_t same = ballot((int)lane < nk && (my_key >> 24) == (uint32_t)bucket);
                if (__builtin_popcountll(same) >= 3) continue;
            }
            if (nk >= 64) { ovf = true; break; }
            uint32_t key;
            bool g = mfp::ext_is_grease(x.type);
            if (fmt == 1) key = g ? (0x0a0aU << 16) : ((x.type << 16) | x.length);
            else key = ((uint32_t)bucket << 24) | (g ? 0 : (1u << 23)) | (g ? 0 : x.length);
            if ((int)lane == nk) { my_key = key; my_off = start; }
            nk++;
        }
        if (!ovf && nk > 0) {
            // rank of each kept extension: key, then value bytes (non-grease),
            // then wire position (ties emit identical bytes)
            int rank = 0;
            for (int j = 0; j < nk; j++) {
                uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)my_key, j);
                int oj = __builtin_amdgcn_readlane(my_off, j);
                bool less = false;
                if ((int)lane < nk && j != (int)lane) {
                    if (kj != my_key) less = kj < my_key;
                    else less = j < (int)lane;
                }
                // equal keys need the value comparison: rare, done wave-uniformly
                uint64_t eq = ballot((int)lane < nk && j != (int)lane && kj == my_key);
                while (eq) {
                    int i = (int)__builtin_ctzll(eq);
                    eq &= eq - 1;
                    int oi = __builtin_amdgcn_readlane(my_off, i);
                    C qa = cmk(oj, exts.e), qb = cmk(oi, exts.e);
                    Ext a = ext_parse(qa), b = ext_parse(qb);
                    bool lt = false, gt = false;
                    if (!mfp::ext_is_grease(a.type) && !mfp::ext_is_grease(b.type)) {
                        int c = ccmp(a.value, b.value);
                        lt = c < 0; gt = c > 0;
                    }
                    if ((int)lane == i) less = lt || (!gt && j < i);
                }
                rank += less ? 1 : 0;
            }
            for (int r = 0; r < nk && !ovf; r++) {
                uint64_t m = ballot((int)lane < nk && rank == r);
                int src_lane = (int)__builtin_ctzll(m);
                int off = __builtin_amdgcn_readlane(my_off, src_lane);
                C q = cmk(off, exts.e);
                Ext x = ext_parse(q);
                if (fmt == 2) (void)mfp::fmt2_bucket_t(x.type, x.encoded_type);
                ext_fp1(x, role);
            }
        }
        putc(']');
    }

    // -----------------------------------------------------------------------
    // Extension list, lane-parallel: lane k owns extension k.  The offset
    // chain (type, length) is walked once with window reads; each lane then
    // formats its own extension (tls.h:1549-1616 format 0, 1413-1499 format
    // 1, 1664-1732 format 2), the wave orders them (wire order, or the rank
    // under the reference's comparator for formats 1/2), and exclusive
    // prefix sums place every lane's characters, scratch bytes and segments.
    // Returns false (nothing emitted) when the list needs the serial path:
    // more than 64 extensions or a QUIC transport-parameter extension.
    // -----------------------------------------------------------------------
    WDEV static uint32_t wave_excl_scan(uint32_t v, uint32_t lane_) {
        uint32_t incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(incl, d, 64);
            if ((int)lane_ >= d) incl += y;
        }
        return incl - v;
    }
    WDEV bool exts_par(C exts, int role, int fmt) {
#ifdef MFP_PROBE_NOPAR
        return false;
#endif
        // 1. offset chain (ext_parse semantics: header and value must fit)
        int my_off = 0, nk = 0;
        {
            int p = exts.d, e = exts.e;
            if (p < 0) { p = 0; e = 0; }
            while (p < e) {
                if (e - p < 4) break;
                uint32_t h = be32(p);
                int len = (int)(h & 0xffff);
                if (len > e - p - 4) break;
                uint32_t t = h >> 16;
                if (t == 0x39 || t == 0xffa5 || nk == 64) return false;
                my_off = ((int)lane == nk) ? p : my_off;
                nk++;
                p += 4 + len;
            }
        }
        const bool mine = (int)lane < nk;
        // 2. per-lane extension fields
        uint32_t type = 0, len = 0;
        if (mine) {
            const uint8_t *b = L.buf + my_off;
            type = ((uint32_t)b[0] << 8) | b[1];
            len = ((uint32_t)b[2] << 8) | b[3];
        }
        const bool grease = (type & 0x0f0f) == 0x0a0a;
        uint32_t enc = grease ? 0x0a0a : type;
        int bucket = 0;
        bool keep = mine;
        if (fmt == 2 && mine) {
            bucket = mfp::fmt2_bucket_t(type, enc);
            keep = bucket >= 0;
        }
        if (fmt == 2) {
            // the first three per bucket in wire order are kept (tls.h:1695-1701)
            int seen = 0;
            for (int j = 0; j < nk; j++) {
                int bj = __builtin_amdgcn_readlane(bucket, j);
                int kj = __builtin_amdgcn_readlane((int)keep, j);
                if (kj && bj == bucket && j < (int)lane) seen++;
            }
            if (seen >= 3) keep = false;
        }
        // 3. order: wire order (fmt 0) or rank under the fmt 1/2 comparator
        int pos = (int)lane;
        if (fmt != 0) {
            uint32_t key = 0xffffffffu;
            if (keep) {
                if (fmt == 1) key = grease ? (0x0a0aU << 16) : ((type << 16) | len);
                else key = ((uint32_t)bucket << 24) | (grease ? 0 : (1u << 23)) | (grease ? 0 : len);
            }
            int rank = 0;
            for (int j = 0; j < nk; j++) {
                uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, j);
                if (kj == 0xffffffffu) continue;
                bool less = false;
                if (keep && j != (int)lane) {
                    if (kj != key) less = kj < key;
                    else less = j < (int)lane;
                }
                // equal keys of non-grease extensions: value bytes decide
                uint64_t eq = ballot(keep && j != (int)lane && kj == key && !grease && (kj >> 16) != 0x0a0a);
                if (eq && fmt == 2) eq = ballot(keep && j != (int)lane && kj == key && !grease);
                while (eq) {
                    int i = (int)__builtin_ctzll(eq);
                    eq &= eq - 1;
                    int oj = __builtin_amdgcn_readlane(my_off, j), oi = __builtin_amdgcn_readlane(my_off, i);
                    uint32_t tj = be16(oj);
                    if ((tj & 0x0f0f) == 0x0a0a) continue;
                    int c = ccmp(cmk(oj + 4, oj + 4 + (int)be16(oj + 2)), cmk(oi + 4, oi + 4 + (int)be16(oi + 2)));
                    if ((int)lane == i) less = c < 0 || (c == 0 && j < i);
                }
                rank += less ? 1 : 0;
            }
            pos = keep ? rank : 64;
        }
        // 4. per-extension output shape
        //   non-static: "(" hex16(t) ")"                          6 chars, 6 scratch, 1 segment
        //   static:     "(" hex16(t) hex16(dg len) | value | ")"  9 scratch + value hex + 1 scratch
        //   type printed: fmt 0 degrease16(type), fmt 1/2 encoded type
        const bool st = keep && mfp::is_static_ext(type);
        uint32_t tprint = fmt == 0 ? mfp::degrease16(type) : enc;
        int skip = 0, gl = 0;
        if (st) {
            if (type == 0x000a || type == 0x002b) {
                int ug = type == 0x000a ? 2 : (role == 0 ? 1 : 0);
                skip = (int)len < ug ? (int)len : ug;
                gl = ((int)len - skip) & ~1;
            } else {
                skip = (int)len;
            }
        }
        uint32_t chars = !keep ? 0u : st ? (uint32_t)(10 + 2 * skip + 2 * gl) : 6u;
        uint32_t sbytes = !keep ? 0u : st ? 10u : 6u;
        uint32_t segs = !keep ? 0u : st ? (uint32_t)(2 + (skip > 0) + (gl > 0)) : 1u;
        // values in output order: lane r holds the extension of rank r
        const int nout = fmt == 0 ? nk : (int)__builtin_popcountll(ballot(keep));
        if (fmt != 0) {
            // inverse permutation through LDS scratch is avoided: bpermute pulls
            // each output slot's values from the lane that owns that rank
            int src = 64;
            for (int j = 0; j < nk; j++) {
                int pj = __builtin_amdgcn_readlane(pos, j);
                if (pj == (int)lane) src = j;
            }
            int sl = src < 64 ? src : 0;
            uint32_t c2 = __builtin_amdgcn_ds_bpermute(sl << 2, (int)chars);
            uint32_t s2 = __builtin_amdgcn_ds_bpermute(sl << 2, (int)sbytes);
            uint32_t g2 = __builtin_amdgcn_ds_bpermute(sl << 2, (int)segs);
            if (src == 64) { c2 = 0; s2 = 0; g2 = 0; }
            uint32_t ec = wave_excl_scan(c2, lane), es = wave_excl_scan(s2, lane), eg = wave_excl_scan(g2, lane);
            // back to the owning lane
            int ps = pos < 64 ? pos : 0;
            uint32_t c3 = __builtin_amdgcn_ds_bpermute(ps << 2, (int)ec);
            uint32_t s3 = __builtin_amdgcn_ds_bpermute(ps << 2, (int)es);
            uint32_t g3 = __builtin_amdgcn_ds_bpermute(ps << 2, (int)eg);
            return exts_par_write(fmt, nout, keep, my_off, len, tprint, st, skip, gl, chars, sbytes, segs, c3, s3, g3);
        }
        uint32_t ec = wave_excl_scan(chars, lane), es = wave_excl_scan(sbytes, lane), eg = wave_excl_scan(segs, lane);
        return exts_par_write(fmt, nout, keep, my_off, len, tprint, st, skip, gl, chars, sbytes, segs, ec, es, eg);
    }
    WDEV bool exts_par_write(int fmt, int nout, bool keep, int off, uint32_t len, uint32_t tprint, bool st, int skip,
                             int gl, uint32_t chars, uint32_t sbytes, uint32_t segs, uint32_t ec, uint32_t es,
                             uint32_t eg) {
        // totals (sum over all lanes; lanes without an extension add zeros)
        uint32_t tc = chars, ts = sbytes, tg = segs;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            tc += __shfl_xor(tc, d, 64);
            ts += __shfl_xor(ts, d, 64);
            tg += __shfl_xor(tg, d, 64);
        }
        tc = rfl(tc); ts = rfl(ts); tg = rfl(tg);
        (void)nout; (void)len; (void)fmt;
        flush();
        const uint32_t lead = fmt == 0 ? '(' : '[', trail = fmt == 0 ? ')' : ']';
        putc(lead);
        flush();
        if (n + tc > FP_MAX) { n += tc; putc(trail); return true; }
        if (nseg + (int)tg > SEG_CAP || scr + (int)ts > SCR_CAP - 16) { ovf = true; return true; }
        if (keep) {
            const int sbase = PKT_CAP + scr + (int)es;
            uint8_t *sp = L.buf + sbase;
            sp[0] = '(';
            sp[1] = (uint8_t)hexc((tprint >> 12) & 15);
            sp[2] = (uint8_t)hexc((tprint >> 8) & 15);
            sp[3] = (uint8_t)hexc((tprint >> 4) & 15);
            sp[4] = (uint8_t)hexc(tprint & 15);
            uint32_t c0 = n + ec;
            int g = nseg + (int)eg;
            if (!st) {
                sp[5] = ')';
                L.seg_end[g] = (uint16_t)(c0 + 6);
                L.seg_info[g] = (uint32_t)sbase | (K_RAW << 16);
            } else {
                uint32_t ldg = mfp::degrease16(len);
                sp[5] = (uint8_t)hexc((ldg >> 12) & 15);
                sp[6] = (uint8_t)hexc((ldg >> 8) & 15);
                sp[7] = (uint8_t)hexc((ldg >> 4) & 15);
                sp[8] = (uint8_t)hexc(ldg & 15);
                sp[9] = ')';
                uint32_t c = c0 + 9;
                L.seg_end[g] = (uint16_t)c;
                L.seg_info[g] = (uint32_t)sbase | (K_RAW << 16);
                g++;
                if (skip > 0) {
                    c += 2 * skip;
                    L.seg_end[g] = (uint16_t)c;
                    L.seg_info[g] = (uint32_t)(off + 4) | (K_HEX << 16);
                    g++;
                }
                if (gl > 0) {
                    c += 2 * gl;
                    L.seg_end[g] = (uint16_t)c;
                    L.seg_info[g] = (uint32_t)(off + 4 + skip) | (K_HEXDG << 16);
                    g++;
                }
                c += 1;
                L.seg_end[g] = (uint16_t)c;
                L.seg_info[g] = (uint32_t)(sbase + 9) | (K_RAW << 16);
            }
        }
        n += tc; nseg += (int)tg; scr += (int)ts;
        putc(trail);
        return true;
    }

    WDEV C tls_record_fragment(C &d) {                   // tls_record::parse tls.h:153
        C f = cnul();
        if (clen(d) < 5) return f;
        uint64_t t, len;
        rd_uint(d, 1, t); rd_uint(d, 2, t); rd_uint(d, 2, len);
        cinit_outer(f, d, len);
        return f;
    }
    struct Hs { uint32_t msg_type; uint64_t length; C body; uint64_t more; };
    WDEV Hs tls_hs_parse(C &d) {                         // tls_handshake::parse tls.h:244
        Hs h; h.msg_type = 0; h.length = 0; cset_null(h.body); h.more = 0;
        if (clen(d) < 4) return h;
        uint64_t t;
        rd_uint(d, 1, t); h.msg_type = (uint32_t)t;
        rd_uint(d, 3, t); h.length = t;
        if (h.length > 32768) return h;
        cinit_outer(h.body, d, h.length);
        h.more = h.length - (uint64_t)clen(h.body);
        return h;
    }
    struct Ch { C version, ciphers, compression, extensions; };
    WDEV Ch tls_ch_parse(C p) {                          // tls_client_hello::parse tls.h:1811
        Ch ch; cset_null(ch.version); cset_null(ch.ciphers); cset_null(ch.compression); cset_null(ch.extensions);
        uint64_t l;
        C t;
        cparse(ch.version, p, 2);
        if (!cnotempty(ch.version)) return ch;
        bool dtls = ld(ch.version.d) == 0xfe;
        cparse(t, p, 32);
        if (!rd_uint(p, 1, l)) return ch;
        cparse(t, p, (long)l);
        if (dtls) {
            if (!look_uint(p, 1, l)) return ch;
            if (!cskip(p, (int)l + 1)) return ch;
        }
        if (!rd_uint(p, 2, l)) return ch;
        if (l & 1) return ch;
        cparse(ch.ciphers, p, (long)l);
        if (!rd_uint(p, 1, l)) return ch;
        cparse(ch.compression, p, (long)l);
        if (!rd_uint(p, 2, l)) return ch;
        cparse_soft(ch.extensions, p, (long)l);
        return ch;
    }
    WDEV void tls_ch_fp(const Ch &ch, int fmt) {         // tls_client_hello::fingerprint tls.h:1928
        if (fmt >= 1 && fmt <= 2) put2('0' + fmt, '/');
        putc('('); hex_c(ch.version); putc(')');
        putc('('); hex_degrease(ch.ciphers.d, clen(ch.ciphers)); putc(')');
        if (exts_par(ch.extensions, 0, fmt)) return;
        if (fmt == 0) exts_fp0(ch.extensions, 0);
        else exts_fp12(ch.extensions, 0, fmt);
    }
    // tls_extensions::set_meta_data tls.h:1316 (server_name; last one wins)
    WDEV void tls_sni(C exts, int base) {
        C p = exts;
        while (clen(p) > 0) {
            int start = p.d;
            uint64_t t, l;
            if (!rd_uint(p, 2, t)) break;
            if (!rd_uint(p, 2, l)) break;
            if (!cskip(p, (int)l)) break;
            if (t == 0) {
                C e = cmk(start, p.d);
                cskip(e, 9);
                o.sni_off = (uint32_t)(e.d - base); o.sni_len = (uint32_t)clen(e);
            }
        }
    }
    struct Sh { C version, cipher, extensions; };
    WDEV Sh tls_sh_parse(C &rec) {                       // parse_tls_server_hello tls.h:2097
        Sh s; cset_null(s.version); cset_null(s.cipher); cset_null(s.extensions);
        uint64_t l; C t;
        cparse(s.version, rec, 2);
        cparse(t, rec, 32);
        if (!look_uint(rec, 1, l)) return s;
        if (!cskip(rec, (int)l + 1)) return s;
        cparse(s.cipher, rec, 2);
        cparse(t, rec, 1);
        if (!rd_uint(rec, 2, l)) return s;
        cparse(s.extensions, rec, (long)l);
        return s;
    }
    WDEV bool tls_sh_not_empty(const Sh &s) {            // tls_server_hello::is_not_empty tls.h:513
        C t = s.version; uint64_t v;
        rd_uint(t, 2, v);
        if (!(v == 0x0303 || v == 0x0302 || v == 0x0301 || v == 0x0300 || v == 0xfeff || v == 0xfefd)) return false;
        return cnotempty(s.cipher);
    }
    WDEV void tls_sh_fp(const Sh &s) {                   // tls_server_hello::fingerprint tls.h:2126
        putc('('); hex_c(s.version); putc(')');
        putc('('); hex_c(s.cipher); putc(')');
        if (!exts_par(s.extensions, 1, 0)) exts_fp0(s.extensions, 1);
    }
    struct Cert { C list; uint64_t more; };
    WDEV void cert_record(Out &o, C l, int base) {       // see mfp_device.hpp
        if (cnotempty(l)) { o.sni_off = (uint32_t)(l.d - base); o.sni_len = (uint32_t)clen(l); }
    }
    WDEV void tls_cert_parse(Cert &c, C &d) {            // tls_server_certificate::parse tls.h:281
        uint64_t t = 0;
        if (!rd_uint(d, 3, t)) return;
        if (t > 65536) { cset_null(d); return; }
        cinit_outer(c.list, d, t);
        c.more = t - (uint64_t)clen(c.list);
    }

    // =======================================================================
    // SSH (ssh.h)
    // =======================================================================
    struct SshBin { C payload; uint64_t more; };
    WDEV SshBin ssh_bin_parse(C &p) {                    // ssh_binary_packet ssh.h:56
        SshBin b; cset_null(b.payload); b.more = 0;
        uint64_t plen, pad;
        rd_uint(p, 4, plen);
        rd_uint(p, 1, pad);
        if (plen > 16384 || plen < 1) { if (p.d >= 0) p.d = p.e; return b; }
        if (!cnotempty(p)) return b;
        long left = (long)plen - 1;
        if (left > clen(p)) b.more = left - clen(p);
        cparse_soft(b.payload, p, left);
        return b;
    }
    WDEV void name_list_parse(C &nl, C &p) {             // name_list::parse ssh.h:110
        uint64_t l;
        rd_uint(p, 4, l);
        if (l > 2048) { if (p.d >= 0) p.d = p.e; return; }
        cparse(nl, p, (long)l);
    }
    WDEV bool ssh_kex_fp(bool emit, C payload) {         // ssh_kex_init::fingerprint ssh.h:240
        C p = payload, t, nl[10];
        cparse(t, p, 1);
        cparse(t, p, 16);
        for (int i = 0; i < 10; i++) { cset_null(nl[i]); name_list_parse(nl[i], p); }
        if (!cnotempty(nl[0])) return false;
        if (emit) {
            for (int i = 0; i < 10; i++) {
                putc('(');
                if (cnotempty(nl[i])) hex(nl[i].d, clen(nl[i]));
                putc(')');
            }
        }
        return true;
    }

    // =======================================================================
    // HTTP (http.h, http.cc)
    // =======================================================================
    // perfect_hash::lookup perfect_hash.h:256: exact ASCII-case-insensitive
    // match; lane j compares byte j of the name
    WDEV int name_lookup(const mfp::HdrName *tab, int ntab, C nm) {
        int l = clen(nm);
        if (l <= 0 || l > 32) return -1;
        uint32_t mine = (int)lane < l ? mfp::c_tolower(L.buf[nm.d + (int)(lane & 31)]) : 0u;
        uint64_t live = l == 64 ? ~0ull : ((1ull << l) - 1);
        for (int i = 0; i < ntab; i++) {
            if (tab[i].len != l) continue;
            uint32_t want = (int)lane < l ? (uint8_t)tab[i].s[lane] : 0;
            if ((ballot(mine == want) & live) == live) return i;
        }
        return -1;
    }
    WDEV bool http_delim(C &p, C del) {                  // delimiter(datum&, const datum&) http.h:113
        C dl = cnul();
        if (ccompare_n(p, del.d, clen(del))) cparse(dl, p, clen(del));
        else if (p.d >= 0 && clen(p) >= 2 && ld(p.d) == '\r' && ld(p.d + 1) == '\n') cparse(dl, p, 2);
        else if (p.d >= 0 && clen(p) >= 1 && ld(p.d) == '\n') cparse(dl, p, 1);
        return cnotempty(dl);
    }
    // new_http_headers::fingerprint http.h:335 + httpheader http.h:146
    // -----------------------------------------------------------------------
    // Header block, lane-parallel (new_http_headers::fingerprint http.h:335,
    // httpheader http.h:146): lane k owns header line k.  Taken only when
    // the delimiter is "\r\n" and the block is well formed -- every CR is
    // followed by LF and every LF preceded by CR, every line before the empty
    // line has a ':' -- which is exactly when the reference's loop visits the
    // lines one after another; anything else returns false before emitting
    // and the serial loop below runs.
    // -----------------------------------------------------------------------
    // 8 bytes of the staged buffer at byte offset x (any alignment)
    WDEV uint64_t lds_u64(int x) {
        const int a = x & ~7;
        const uint32_t sh = (uint32_t)(x & 7) * 8;
        const uint64_t lo = *(const uint64_t *)(L.buf + a), hi = *(const uint64_t *)(L.buf + a + 8);
        return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    }
    WDEV bool http_headers_par(C body, bool req, C &host, C &ua) {
        if (body.d < 0) return false;
        const mfp::HdrKey *tab = req ? mfp::k_req_keys : mfp::k_resp_keys;
        const int ntab = req ? mfp::N_REQ_NAMES : mfp::N_RESP_NAMES;
        // 1. line ends: LF positions up to the empty line (CRLF CRLF) or the end
        int my_start = 0, my_end = 0, nl = 0;     // line [start, end) excludes CRLF
        bool partial = false, done = false;
        int p = body.d;
        const int e = body.e;
        uint32_t carry_cr = 0;
        int base = p;
        const int p0 = p;
        for (; base < e && !done; base += 64) {
            const int q = base + (int)lane;
            const uint32_t c = L.buf[q < e ? q : base];
            const uint64_t lf = ballot(q < e && c == '\n');
            const uint64_t cr = ballot(q < e && c == '\r');
            const uint64_t cm = ballot(q < e && c == ':');
            if (lane == 0) L.cmask[(base - p0) >> 6] = cm;
            // CR/LF pairing: every LF sits right after a CR and vice versa
            if (((cr << 1) | carry_cr) != lf) return false;
            carry_cr = (uint32_t)(cr >> 63);
            uint64_t m = lf;
            while (m) {
                const int pos = base + (int)__builtin_ctzll(m);
                m &= m - 1;
                const int ls = p, le = pos - 1;       // exclude CR
                if (le == ls) { done = true; break; }  // empty line ends the block
                if (nl == 64) return false;
                if ((int)lane == nl) { my_start = ls; my_end = le; }
                nl++;
                p = pos + 1;
            }
        }
        if (!done) {
            if (carry_cr) return false;                // data ends with a bare CR
            if (p < e) {                                // last line without CRLF
                if (nl == 64) return false;
                if ((int)lane == nl) { my_start = p; my_end = e; }
                nl++;
                partial = true;
            }
        }
        const bool mine = (int)lane < nl;
        // 2. per line: colon (first ':' of the line, from the chunk masks), LWS, value
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        int colon = -1;
        if (mine) {
            for (int x = my_start; x < my_end;) {
                const int rel = x - p0;
                const uint64_t m = L.cmask[rel >> 6] >> (rel & 63);
                if (m) {
                    const int pos = x + (int)__builtin_ctzll(m);
                    if (pos < my_end) colon = pos;
                    break;
                }
                x = p0 + ((rel >> 6) + 1) * 64;
            }
        }
        // a line without ':' makes the reference's name scan run into the
        // next line; the final partial line without ':' just ends the loop
        const bool lastp = partial && (int)lane == nl - 1;
        if (ballot(mine && colon < 0 && !lastp)) return false;
        const bool valid = mine && colon >= 0;
        int vs = 0;
        if (valid) {
            vs = colon + 1;
            while (vs < my_end && (L.buf[vs] == ' ' || L.buf[vs] == '\t')) vs++;
        }
        // 3. name lookup: ASCII case-insensitive exact match (perfect_hash.h:256),
        // the lowercased name as four words against the packed tables
        int idx = -1;
        uint32_t info = 0;
        const int nlen = valid ? colon - my_start : 0;
        if (valid && nlen > 0 && nlen <= 32) {
            uint64_t nw[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint64_t w = 8 * k < nlen ? mfp::swar_tolower(lds_u64(my_start + 8 * k)) : 0ull;
                if (nlen - 8 * k < 8 && nlen > 8 * k) w &= (1ull << (8 * (nlen - 8 * k))) - 1;
                nw[k] = w;
            }
            for (int i = 0; i < ntab; i++) {
                const mfp::HdrKey &k = tab[i];
                if (idx < 0 && k.len == (uint32_t)nlen && k.w[0] == nw[0] && k.w[1] == nw[1] && k.w[2] == nw[2] &&
                    k.w[3] == nw[3]) {
                    idx = i;
                    info = k.info;
                }
            }
        }
        const bool emit = idx >= 0;
        const bool incl_value = (info & 0xff) != 0;
        const uint32_t capture = info >> 8;
        // host / user-agent: first occurrence wins (http.h:364-366)
        if (req) {
            const bool is_host = emit && capture == 1, is_ua = emit && capture == 2;
            const uint64_t hm = ballot(is_host), um = ballot(is_ua);
            if (hm) {
                int k = (int)__builtin_ctzll(hm);
                host = cmk(__builtin_amdgcn_readlane(vs, k), __builtin_amdgcn_readlane(my_end, k));
            }
            if (um) {
                int k = (int)__builtin_ctzll(um);
                ua = cmk(__builtin_amdgcn_readlane(vs, k), __builtin_amdgcn_readlane(my_end, k));
            }
        }
        // 4. "(" hex(span) ")" per emitted line, in line order
        const int span_end = emit ? (incl_value ? my_end : colon) : 0;
        const uint32_t chars = emit ? (uint32_t)(2 + 2 * (span_end - my_start)) : 0u;
        const uint32_t sbytes = emit ? 2u : 0u, segs = emit ? 3u : 0u;
        const uint32_t ec = wave_excl_scan(chars, lane), es = wave_excl_scan(sbytes, lane),
                       eg = wave_excl_scan(segs, lane);
        uint32_t tc = chars, ts = sbytes, tg = segs;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            tc += __shfl_xor(tc, d, 64);
            ts += __shfl_xor(ts, d, 64);
            tg += __shfl_xor(tg, d, 64);
        }
        tc = rfl(tc); ts = rfl(ts); tg = rfl(tg);
        flush();
        if (n + tc > FP_MAX) { n += tc; return true; }
        if (nseg + (int)tg > SEG_CAP || scr + (int)ts > SCR_CAP - 16) { ovf = true; return true; }
        if (emit) {
            const int sbase = PKT_CAP + scr + (int)es;
            L.buf[sbase] = '(';
            L.buf[sbase + 1] = ')';
            const int g = nseg + (int)eg;
            const uint32_t c0 = n + ec;
            L.seg_end[g] = (uint16_t)(c0 + 1);
            L.seg_info[g] = (uint32_t)sbase | (K_RAW << 16);
            L.seg_end[g + 1] = (uint16_t)(c0 + chars - 1);
            L.seg_info[g + 1] = (uint32_t)my_start | (K_HEX << 16);
            L.seg_end[g + 2] = (uint16_t)(c0 + chars);
            L.seg_info[g + 2] = (uint32_t)(sbase + 1) | (K_RAW << 16);
        }
        n += tc; nseg += (int)tg; scr += (int)ts;
        if (tc) last_putc = true;
        return true;
    }
    WDEV void http_headers_fp(C body, C delim, bool req, C &host, C &ua) {
        C tmp = body;
        const mfp::HdrName *tab = req ? mfp::k_req_names : mfp::k_resp_names;
        int ntab = req ? mfp::N_REQ_NAMES : mfp::N_RESP_NAMES;
        while (!ovf) {
            if (http_delim(tmp, delim)) break;
            C hdr_body = tmp, name = cnul();
            if (!cnotempty(tmp)) { cset_null(tmp); }
            else {
                name.d = tmp.d; name.e = tmp.e;
                int q = scan(tmp.d, tmp.e, [](uint32_t c) { return c == ':'; });
                if (q < tmp.e) { name.e = q; tmp.d = q; }
            }
            if (tmp.d >= 0 && tmp.e > tmp.d && ld(tmp.d) == ':') tmp.d++; else cset_null(tmp);
            if (tmp.d >= 0) tmp.d = scan(tmp.d, tmp.e, [](uint32_t c) { return !(c == '\t' || c == ' '); });
            C value;
            cparse_to_delims(value, tmp, '\r', '\n');
            http_delim(tmp, delim);
            hdr_body.e = value.e;
            if (cnull(tmp)) break;
            int idx = name_lookup(tab, ntab, name);
            if (idx >= 0) {
                putc('(');
                if (tab[idx].incl_value) hex(hdr_body.d, clen(hdr_body)); else hex(name.d, clen(name));
                putc(')');
                if (req) {
                    if (tab[idx].capture == 1 && cnull(host)) host = value;
                    if (tab[idx].capture == 2 && cnull(ua)) ua = value;
                }
            }
        }
    }
    WDEV void fp_type_prefix(uint32_t t) {               // fingerprint::set_type fingerprint.h:44
        switch (t) {
        case 1: lit("tls/"); break;
        case 2: lit("tls_server/"); break;
        case 3: lit("http/"); break;
        case 4: lit("http_server/"); break;
        case 5: lit("ssh/"); break;
        case 6: lit("ssh_kex/"); break;
        case 7: lit("tcp/"); break;
        case 10: lit("dtls/"); break;
        case 11: lit("dtls_server/"); break;
        case 13: lit("tcp_server/"); break;
        case 17: lit("ssh_init/"); break;
        case 18: lit("ssh_server/"); break;
        case 19: lit("ssh_kex_server/"); break;
        case 20: lit("ssh_init_server/"); break;
        }
        last_putc = true;   // set_type ends with write_char('/')
    }
    // HTTP request/response parse + fingerprint (http.cc:105-128, 369-383, 426-553)
    WDEV bool http_msg(C p, bool req, int base) {
#ifdef MFP_PROBE_NOHTTP
        return false;
#endif
        C f1 = cnul(), f2 = cnul(), f3 = cnul();
        if (req) {
            C uri;
            cparse_to_delim(f1, p, ' ');
            int ml = clen(f1);
            if (ml < 3 || ml > 16) return false;
            if (scan(f1.d, f1.e, [](uint32_t c) { return !mfp::c_isupper(c); }) < f1.e) return false;
            cskip(p, 1);
            cparse_to_delim(uri, p, ' ');
            cskip(p, 1);
            cparse_to_delims(f2, p, '\r', '\n');
            if (!(f2.d >= 0 && clen(f2) >= 5 && ld(f2.d) == 'H' && ld(f2.d + 1) == 'T' && ld(f2.d + 2) == 'T' &&
                  ld(f2.d + 3) == 'P' && ld(f2.d + 4) == '/'))
                return false;
        } else {
            cparse_to_delim(f1, p, ' ');
            cskip(p, 1);
            cparse_to_delim(f2, p, ' ');
            cskip(p, 1);
            cparse_to_delims(f3, p, '\r', '\n');
            if (!cnotempty(f2)) return false;
        }
        C delim; delim.d = p.d;
        if (p.d >= 0) p.d = scan(p.d, p.e, [](uint32_t c) { return mfp::c_isalpha(c); });
        delim.e = p.d;
        fp_type_prefix(req ? 3 : 4);
        putc('('); hex_c(f1); putc(')');
        putc('('); hex_c(f2); putc(')');
        if (!req) { putc('('); hex_c(f3); putc(')'); }
        putc('(');
        C host = cnul(), ua = cnul();
        const bool crlf = clen(delim) == 2 && ld(delim.d) == '\r' && ld(delim.d + 1) == '\n';
#ifndef MFP_PROBE_NOHDR
        if (!(crlf && http_headers_par(p, req, host, ua))) http_headers_fp(p, delim, req, host, ua);
#endif
        putc(')');
        if (req) {
            if (!cnull(host)) { o.sni_off = (uint32_t)(host.d - base); o.sni_len = (uint32_t)clen(host); }
            if (!cnull(ua)) { o.ua_off = (uint32_t)(ua.d - base); o.ua_len = (uint32_t)clen(ua); }
        }
        return true;
    }

    // =======================================================================
    // transport dispatch
    // =======================================================================
    WDEV bool m8(C p, uint64_t mask, uint64_t val, uint64_t w) {
        return p.d >= 0 && clen(p) >= 8 && (w & mask) == val;
    }
    // set_tcp_protocol pkt_proc.cc:488 (selection subset)
    WDEV void tcp_data(C pkt, int tcph, int base) {
        uint32_t sel = cfg.select;
        uint32_t sport = be16(tcph), dport = be16(tcph + 2);
        uint32_t msg = 0;
        if (clen(pkt) >= 4) {
            uint64_t w = clen(pkt) >= 8 ? le8(pkt.d) : 0;
            const uint64_t MT = LE8(0xff, 0xff, 0xfc, 0, 0, 0xff, 0, 0);
            if ((sel & SEL_TLS_CH) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x01, 0, 0), w)) msg = MFP_MSG_TLS_CH;
            else if ((sel & SEL_TLS_SH) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x02, 0, 0), w)) msg = MFP_MSG_TLS_SH;
            else if ((sel & SEL_TLS_CERT) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x0b, 0, 0), w)) msg = MFP_MSG_TLS_CERT;
            else if ((sel & (SEL_SSH_CLIENT | SEL_SSH_SERVER)) &&
                     m8(pkt, LE8(0xff, 0xff, 0xff, 0xff, 0, 0, 0, 0), LE8('S', 'S', 'H', '-', 0, 0, 0, 0), w))
                msg = MFP_MSG_SSH_INIT;
            else if ((sel & (SEL_SSH_CLIENT | SEL_SSH_SERVER)) &&
                     m8(pkt, LE8(0xff, 0xff, 0xf0, 0, 0, 0xff, 0, 0), LE8(0, 0, 0, 0, 0, 0x14, 0, 0), w))
                msg = MFP_MSG_SSH_KEX;
        }
        if (msg == 0) {
            if (clen(pkt) < 4) return;
            uint32_t kw = (ld(pkt.d) << 24) | (ld(pkt.d + 1) << 16) | (ld(pkt.d + 2) << 8) | ld(pkt.d + 3);
            if (sel & SEL_HTTP_REQ) {
                bool hit = false;
                for (int i = 0; i < 36; i++) hit |= (mfp::k_http_kw[i] == kw);
                if (hit) {
                    if constexpr (!(SPEC & SPEC_HTTP)) { punt = true; return; }
                    o.msg = MFP_MSG_HTTP_REQ;
                    if (http_msg(pkt, true, base)) { o.flags |= MFP_FLAG_EMIT; o.fp_type = 3; }
                    else o.msg = 0;
                    return;
                }
            }
            if ((sel & SEL_HTTP_RESP) && kw == 0x48545450u) {
                if constexpr (!(SPEC & SPEC_HTTP)) { punt = true; return; }
                o.msg = MFP_MSG_HTTP_RESP;
                if (http_msg(pkt, false, base)) { o.flags |= MFP_FLAG_EMIT; o.fp_type = 4; }
                else o.msg = 0;
            }
            return;
        }
        o.msg = msg;
        if constexpr (!(SPEC & SPEC_TLS)) {
            if (msg == MFP_MSG_TLS_CH || msg == MFP_MSG_TLS_SH || msg == MFP_MSG_TLS_CERT) { punt = true; return; }
        }
        if constexpr (!(SPEC & SPEC_SSH)) {
            if (msg == MFP_MSG_SSH_INIT || msg == MFP_MSG_SSH_KEX) { punt = true; return; }
        }
        switch (msg) {
        case MFP_MSG_TLS_CH: {
#ifdef MFP_PROBE_NOCH
            return;
#endif
            C p = pkt;
            C frag = tls_record_fragment(p);
            Hs hs = tls_hs_parse(frag);
            if (hs.more) o.flags |= MFP_FLAG_TRUNCATED;
            Ch ch = tls_ch_parse(hs.body);
            if (!cnotempty(ch.compression)) return;
            o.flags |= MFP_FLAG_EMIT; o.fp_type = 1;
            fp_type_prefix(1);
            tls_ch_fp(ch, (int)cfg.tls_format);
            tls_sni(ch.extensions, base);
            return;
        }
        case MFP_MSG_TLS_SH: {                           // tls.h:573
#ifdef MFP_PROBE_NOSH
            return;
#endif
            C p = pkt;
            Sh sh; cset_null(sh.version); cset_null(sh.cipher); cset_null(sh.extensions);
            Cert cert; cset_null(cert.list); cert.more = 0;
            C frag = tls_record_fragment(p);
            Hs hs = tls_hs_parse(frag);
            if (hs.msg_type == 2) {
                sh = tls_sh_parse(hs.body);
                if (cnotempty(frag)) { Hs h2 = tls_hs_parse(frag); tls_cert_parse(cert, h2.body); }
            } else if (hs.msg_type == 11) {
                tls_cert_parse(cert, hs.body);
            }
            C frag2 = tls_record_fragment(p);
            Hs hs2 = tls_hs_parse(frag2);
            if (hs2.msg_type == 11) tls_cert_parse(cert, hs2.body);
            cert_record(o, cert.list, base);            // tls.h:605-627 (the JSON writer's certs)
            if (cert.more) o.flags |= MFP_FLAG_TRUNCATED;
            bool hello = tls_sh_not_empty(sh);
            if (hello || cnotempty(cert.list)) o.flags |= MFP_FLAG_EMIT;
            if (hello) { o.fp_type = 2; fp_type_prefix(2); tls_sh_fp(sh); }
            return;
        }
        case MFP_MSG_TLS_CERT: {                         // tls.h:720
            C p = pkt;
            Cert cert; cset_null(cert.list); cert.more = 0;
            C frag = tls_record_fragment(p);
            Hs hs = tls_hs_parse(frag);
            if (hs.msg_type == 11) {
                tls_cert_parse(cert, hs.body);
                uint32_t t = 0;                              // entity, tls.h:728-744
                if (cnotempty(frag)) { Hs h = tls_hs_parse(frag); t = h.msg_type; }
                else if (cnotempty(p)) { C f2 = tls_record_fragment(p); Hs h = tls_hs_parse(f2); t = h.msg_type; }
                if (t == 16) o.flags |= MFP_FLAG_CERT_CLIENT; else if (t == 12) o.flags |= MFP_FLAG_CERT_SERVER;
            }
            cert_record(o, cert.list, base);
            if (cert.more) o.flags |= MFP_FLAG_TRUNCATED;
            if (cnotempty(cert.list)) o.flags |= MFP_FLAG_EMIT;
            return;
        }
        case MFP_MSG_SSH_INIT: {                         // ssh.h:342-430
#ifdef MFP_PROBE_NOSSH
            return;
#endif
            bool server = !(dport <= sport);
            if (!(sel & (server ? SEL_SSH_SERVER : SEL_SSH_CLIENT))) { o.msg = 0; return; }
            C p = pkt, proto, comment = cnul();
            uint32_t delim = cparse_to_delims(proto, p, '\n', ' ');
            if (delim != '\n') { cskip(p, 1); cparse_to_delim(comment, p, '\n'); }
            cskip(p, 1);
            bool kex = false;
            SshBin bin; cset_null(bin.payload); bin.more = 0;
            if (cnotempty(p)) {
                bin = ssh_bin_parse(p);
                if (cnotempty(bin.payload)) kex = ssh_kex_fp(false, bin.payload);
            }
            uint64_t more = kex ? bin.more : 8192;
            if (more) o.flags |= MFP_FLAG_TRUNCATED;
            if (!cnotempty(proto)) return;
            o.flags |= MFP_FLAG_EMIT;
            if (kex) {
                o.fp_type = server ? 18 : 5;
                fp_type_prefix(o.fp_type);
                ssh_kex_fp(true, bin.payload);
            } else {
                o.fp_type = server ? 20 : 17;
                fp_type_prefix(o.fp_type);
                putc('(');
                if (cnotempty(comment)) {
                    hex(proto.d, clen(proto));
                    put2('2', '0');
                    C t = comment; t.e -= 1; if (t.e < t.d) t.e = t.d;
                    hex(t.d, clen(t));
                } else {
                    C t = proto; t.e -= 1; if (t.e < t.d) t.e = t.d;
                    hex(t.d, clen(t));
                }
                putc(')');
            }
            o.ua_off = (uint32_t)(proto.d - base); o.ua_len = (uint32_t)clen(proto);   // ssh.h:480
            return;
        }
        case MFP_MSG_SSH_KEX: {                          // pkt_proc.cc:586-601
            bool server = !(dport <= sport);
            if (!(sel & (server ? SEL_SSH_SERVER : SEL_SSH_CLIENT))) { o.msg = 0; return; }
            C p = pkt;
            SshBin bin = ssh_bin_parse(p);
            if (bin.more) o.flags |= MFP_FLAG_TRUNCATED;
            if (!ssh_kex_fp(false, bin.payload)) return;
            o.flags |= MFP_FLAG_EMIT;
            o.fp_type = server ? 19 : 6;
            fp_type_prefix(o.fp_type);
            ssh_kex_fp(true, bin.payload);
            return;
        }
        }
    }
    // set_udp_protocol pkt_proc.cc:677 (DTLS, dtls.h)
    WDEV void udp_data(C pkt, int base) {
#ifdef MFP_PROBE_NOUDP
        return;
#endif
        if (!(cfg.select & SEL_DTLS) || clen(pkt) < 16) return;
        uint64_t w0 = le8(pkt.d), w1 = le8(pkt.d + 8);
        const uint64_t M0 = LE8(0xff, 0xff, 0xfd, 0, 0, 0, 0, 0), V0 = LE8(0x16, 0xfe, 0xfd, 0, 0, 0, 0, 0);
        const uint64_t M1 = LE8(0, 0, 0, 0, 0, 0xff, 0, 0);
        if ((w0 & M0) != V0) return;
        uint32_t hb = (uint32_t)((w1 & M1) >> 40);
        uint32_t msg = hb == 1 ? MFP_MSG_DTLS_CH : hb == 2 ? MFP_MSG_DTLS_SH : hb == 3 ? MFP_MSG_DTLS_HVR : 0;
        if (!msg) return;
        if constexpr (!(SPEC & SPEC_DTLS)) { punt = true; return; }
        o.msg = msg;
        C d = pkt, frag = cnul(), body = cnul();
        uint64_t t, len = 0, foff = 0, flen = 0, more = 0;
        if (clen(d) < 13) cset_null(d);
        else {
            rd_uint(d, 1, t); rd_uint(d, 2, t); rd_uint(d, 2, t); rd_uint(d, 6, t); rd_uint(d, 2, t);
            cparse(frag, d, (long)t);
        }
        if (clen(frag) < 12) cset_null(frag);
        else {
            rd_uint(frag, 1, t); rd_uint(frag, 3, len); rd_uint(frag, 2, t);
            rd_uint(frag, 3, foff); rd_uint(frag, 3, flen);
            cparse(body, frag, (long)flen);
            if (foff == 0) {
                long bl = clen(body);
                if (flen <= len && bl >= 0 && (uint64_t)bl <= len) more = len - (uint64_t)bl;
            }
        }
        if (msg == MFP_MSG_DTLS_CH) {
            if ((uint32_t)more) o.flags |= MFP_FLAG_TRUNCATED;
            Ch ch = tls_ch_parse(body);
            if (!cnotempty(ch.compression)) return;
            o.flags |= MFP_FLAG_EMIT; o.fp_type = 10;
            fp_type_prefix(10);
            tls_ch_fp(ch, (int)cfg.tls_format);
            tls_sni(ch.extensions, base);
        } else if (msg == MFP_MSG_DTLS_SH) {
            C b2 = body;
            Sh sh = tls_sh_parse(b2);
            if (!tls_sh_not_empty(sh)) return;
            o.flags |= MFP_FLAG_EMIT; o.fp_type = 11;
            fp_type_prefix(11);
            tls_sh_fp(sh);
        } else {
            C b2 = body; uint64_t cl; C ck;
            rd_uint(b2, 2, t); rd_uint(b2, 1, cl);
            cparse(ck, b2, (long)cl);
            if (!cnull(b2)) o.flags |= MFP_FLAG_EMIT;
        }
    }
    // IP header (ip.h:124, ip.h:448); returns transport protocol or 255
    WDEV uint32_t ip_parse(C &p, int &iph, int &ipv) {
        uint32_t v = look_u8(p);
        iph = -1; ipv = 0;
        if ((v & 0xf0) == 0x40) {
            int h = cget_ptr(p, 20);
            ipv = 4;
            if (h < 0) return 255;
            iph = h;
            long tl = (long)be16(h + 2);
            ctrim_to_length(p, tl - 20);
            return ld(h + 9);
        }
        if ((v & 0xf0) == 0x60) {
            int h = cget_ptr(p, 40);
            ipv = 6;
            if (h < 0) return 255;
            iph = h;
            ctrim_to_length(p, (long)be16(h + 4));
            uint32_t nh = ld(h + 6);
            while (clen(p) > 0) {
                bool ext = (nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135 || nh == 139 || nh == 140);
                if (!ext) break;
                uint32_t hdr = nh, nnh = rd_u8(p), hl; C dd;
                if (hdr == 44) cparse(dd, p, 7);
                else if (hdr == 51) { hl = rd_u8(p); cparse(dd, p, (long)hl * 4 + 6); }
                else { hl = rd_u8(p); cparse(dd, p, (long)hl * 8 + 6); }
                nh = nnh;
            }
            return nh;
        }
        return 255;
    }
    // TCP SYN fingerprint (tcpip.h:215-249, ip.h:141-163, 478-503)
    WDEV void tcp_syn_fp(int ipv, int iph, int tcph, C opts) {
        if (ipv == 4) {
            lit("(40)(");
            if (ld(iph + 4) == 0 && ld(iph + 5) == 0) put2('0', '0');
            put2(')', '(');
            hex8(ld(iph + 8) & 0xe0);
            putc(')');
        } else {
            lit("(60)(");
            if (ld(iph + 1) == 0 && ld(iph + 2) == 0 && ld(iph + 3) == 0) put2('0', '0');
            put2(')', '(');
            hex8(ld(iph + 7) & 0xe0);
            putc(')');
        }
        putc('('); hex(tcph + 14, 2); put2(')', '(');
        C tmp = opts;
        while (clen(tmp) > 0) {
            uint32_t kind = rd_u8(tmp), len = 0;
            C od = cnul();
            if (!(kind == 0 || kind == 1)) {
                len = rd_u8(tmp);
                if (len >= 2) cparse(od, tmp, (long)len - 2);
            }
            putc('(');
            hex8(kind);
            if (kind == 2 || kind == 3) { hex8(len); hex_c(od); }
            putc(')');
        }
        putc(')');
    }
    // IP layer: ip_write_json pkt_proc.cc:1063 / analyze_ip_packet pkt_proc.cc:1597
    WDEV void ip_path(C pkt, int base) {
        int iph, ipv;
        uint32_t proto = ip_parse(pkt, iph, ipv);
        uint32_t enc = 0;        // net bits 20-27 (see mfp_device.hpp ip_path)
        for (int k = 0; k < 4 && (proto == 4 || proto == 41); k++) {   // pkt_proc.cc:959
            const int oh = iph, ov = ipv;
            proto = ip_parse(pkt, iph, ipv);
            o.flags |= MFP_FLAG_ENCAP;
            if (ov == 6) enc |= 8u << k;
            if (oh < 0 || iph < 0 || iph - oh != (ov == 6 ? 40 : 20)) enc |= 128u;
            enc = (enc & ~7u) | (uint32_t)(k + 1);
        }
        if (iph >= 0) o.net = (uint32_t)(iph - base) | ((uint32_t)ipv << 16) | (enc << 20);
        if (proto == 6) {
            int tcph = cget_ptr(pkt, 20);
            if (tcph < 0) return;
            C opts = cnul();
            cparse(opts, pkt, (long)(ld(tcph + 12) >> 4) * 4 - 20);
            o.src_port = be16(tcph);
            o.dst_port = be16(tcph + 2);
            uint32_t fl = ld(tcph + 13);
            bool syn = fl & 0x02, ack = fl & 0x10;
            if (cfg.mode == MFP_MODE_WRITE_JSON) {
                if (syn && !ack) {
                    if (cfg.select & SEL_TCP_SYN) {
                        o.msg = MFP_MSG_TCP_SYN; o.flags |= MFP_FLAG_EMIT; o.fp_type = 7;
                        fp_type_prefix(7);
                        tcp_syn_fp(ipv, iph, tcph, opts);
                    }
                    return;
                }
                if (syn && ack) {
                    if ((cfg.select & SEL_TCP_SYN) && (cfg.select & SEL_TCP_SYNACK)) {
                        o.msg = MFP_MSG_TCP_SYNACK; o.flags |= MFP_FLAG_EMIT; o.fp_type = 13;
                        fp_type_prefix(13);
                        tcp_syn_fp(ipv, iph, tcph, opts);
                    }
                    return;
                }
                if (clen(pkt) == 0) return;
            }
            tcp_data(pkt, tcph, base);
        } else if (proto == 17) {
            int udph = cget_ptr(pkt, 8);
            if (udph >= 0) {
                o.src_port = be16(udph);
                o.dst_port = be16(udph + 2);
            }
            udp_data(pkt, base);
        }
    }
    WDEV bool ppp_is_ip(C &p) {                          // ppp::is_ip ppp.h:76
        uint32_t b = look_u8(p);
        if (b == 0x7e) {
            rd_u8(p);
            b = look_u8(p);
            if (b == 0xff) { rd_u8(p); rd_u8(p); }
        } else if (b == 0xff) {
            rd_u8(p); rd_u8(p);
        }
        uint32_t proto;
        b = look_u8(p);
        if (b & 1) { if (!(p.d >= 0 && p.e > p.d)) { cset_null(p); proto = 0; } else { proto = rd_u8(p); } }
        else { uint32_t v = 0; for (int i = 0; i < 2; i++) { v *= 256; v += rd_u8(p); } proto = v; }
        return proto == 0x21 || proto == 0x57;
    }
    // link layer: stateful_pkt_proc::write_json(..., linktype) pkt_proc.cc:1328
    // and analyze_packet pkt_proc.cc:1814.  `base` = buf offset of byte 0.
    WDEV void packet_walk(int base, uint32_t len, uint32_t linktype) {
        o.fp_type = 0; o.msg = 0; o.flags = 0;
        o.sni_off = o.ua_off = 0; o.sni_len = o.ua_len = 0xffff;
        o.src_port = o.dst_port = 0;
        o.net = 0;
        C p = cmk(base, base + (int)len);
        switch (linktype) {
        case 1: {                                        // eth::eth eth.h:137
            uint64_t et;
            cskip(p, 12);
            if (!rd_uint(p, 2, et)) return;
            if (et == 0x88a8) { cskip(p, 2); if (!rd_uint(p, 2, et)) return; }
            while (et == 0x8100) { cskip(p, 2); if (!rd_uint(p, 2, et)) return; }
            if (et == 0x8847) {
                uint64_t lbl = 0;
                while (!(lbl & 0x100)) { if (!rd_uint(p, 4, lbl)) return; }
                et = 0x0800;
            }
            if (et == 0x8909) { cskip(p, 6); if (!rd_uint(p, 2, et)) return; }
            if (et == 0x0800 || et == 0x86dd) break;
            if (et == 0x8864) {
                C t; cparse(t, p, 1); cparse(t, p, 1); cparse(t, p, 2); cparse(t, p, 2);
                if (!ppp_is_ip(p)) return;
                break;
            }
            return;
        }
        case 9:
            if (!ppp_is_ip(p)) return;
            break;
        case 101:
            break;
        case 113: {                                      // linux_sll.hpp
            uint64_t pt, ar, al, pr; C lla;
            rd_uint(p, 2, pt); rd_uint(p, 2, ar); rd_uint(p, 2, al); cparse(lla, p, 8); rd_uint(p, 2, pr);
            if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return;
            break;
        }
        case 276: {                                      // linux_sll2.hpp
            uint64_t pr, t, ar; C lla;
            rd_uint(p, 2, pr); rd_uint(p, 2, t); rd_uint(p, 4, t); rd_uint(p, 2, ar);
            rd_uint(p, 1, t); rd_uint(p, 1, t); cparse(lla, p, 8);
            if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return;
            break;
        }
        case 0: {                                        // loopback.hpp
            if (cfg.mode != MFP_MODE_WRITE_JSON) return;
            uint64_t v; rd_uint(p, 4, v);
            if (!cnull(p)) {
                if (!(v == 2 || v == 0x02000000 || v == 24 || v == 0x18000000 || v == 28 || v == 0x1c000000 ||
                      v == 30 || v == 0x1e000000))
                    return;
            }
            break;
        }
        default:
            return;
        }
        if (cnull(p)) return;
        ip_path(p, base);
    }

    // =======================================================================
    // cooperative expansion of the segment table into the fingerprint
    // string: lane l of round r writes characters [512 r + 8 l, +8)
    // =======================================================================
    // ... and the string hash (mfpc::str_hash) of the words, stored after the
    // string at round_up(T, 8) (include/mfp.h MFP_FLAG_HASHED)
    WDEV void expand(uint8_t *out) {
#ifdef MFP_PROBE_NOEXPAND
        return;
#endif
        const uint32_t T = n;
        uint64_t hacc = 0;
        for (uint32_t r0 = 0; r0 < T; r0 += 512) {
            uint32_t p0 = r0 + 8 * lane;
            if (p0 < T) {
                // lower_bound: first segment with end > p0
                int lo = 0, hi = nseg - 1;
                while (lo < hi) {
                    int mid = (lo + hi) >> 1;
                    if ((uint32_t)L.seg_end[mid] > p0) hi = mid; else lo = mid + 1;
                }
                int s = lo;
                uint32_t s_end = L.seg_end[s];
                uint32_t s_start = s ? L.seg_end[s - 1] : 0;
                uint32_t info = L.seg_info[s];
                uint64_t word = 0;
                for (int k = 0; k < 8; k++) {
                    uint32_t p = p0 + k;
                    if (p >= T) break;
                    if (p >= s_end) {
                        s++;
                        s_start = s_end;
                        s_end = L.seg_end[s];
                        info = L.seg_info[s];
                    }
                    uint32_t q = p - s_start, kind = info >> 16, src = info & 0xffff;
                    uint32_t c;
                    if (kind == K_RAW) {
                        c = L.buf[src + q];
                    } else if (kind == K_HEX) {
                        uint32_t b = L.buf[src + (q >> 1)];
                        c = hexc((q & 1) ? (b & 15) : (b >> 4));
                    } else {
                        uint32_t wsrc = src + ((q >> 2) << 1);
                        uint32_t hb = L.buf[wsrc], lb = L.buf[wsrc + 1];
                        uint32_t wv = mfp::degrease16((hb << 8) | lb);
                        uint32_t b = (q & 2) ? (wv & 0xff) : (wv >> 8);
                        c = hexc((q & 1) ? (b & 15) : (b >> 4));
                    }
                    word |= (uint64_t)c << (8 * k);
                }
                *(uint64_t *)(out + p0) = word;
                hacc ^= mfpc::word_term(word, p0 >> 3);
            }
        }
        hacc = wave_xor64(hacc);
        if (lane == 0) *(uint64_t *)(out + ((T + 7) & ~7u)) = mfpc::hash_final(hacc, T);
    }
};

}  // namespace mfpw
