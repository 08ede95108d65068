// mfp_device.hpp -- device-side (gfx950) packet walk and fingerprint
// construction for the MI355X-native mercury path.
//
// One lane owns one packet.  The same walker runs twice per tile:
//   pass 1 (EMIT=false): protocol identification + exact fingerprint length;
//   pass 2 (EMIT=true):  writes the fingerprint bytes with 8-byte
//                        write-combined stores into the tile's arena slice.
// Semantics follow the reference exactly (file:line cites are relative to
// /root/reference/src/libmerc/); the C oracle (oracle/mfp_oracle.c) restates
// the same rules on the CPU and the parity tests compare the two.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mfp.h"
#include "mfp_common.hpp"

namespace mfp {

#define DEV __device__ __forceinline__
#define DEV_HD_CONSTEXPR constexpr __host__ __device__

// ---------------------------------------------------------------------------
// cursor == struct datum (datum.h:220-850); null cursor has d == nullptr
// ---------------------------------------------------------------------------
struct Cur {
    const uint8_t *d, *e;
};

DEV long clen(Cur c) { return c.d ? (long)(c.e - c.d) : 0; }
DEV bool cnull(Cur c) { return c.d == nullptr; }
DEV bool cnotempty(Cur c) { return c.d != nullptr && c.d < c.e; }
DEV void cset_null(Cur &c) { c.d = c.e = nullptr; }
DEV Cur cmk(const uint8_t *d, const uint8_t *e) { Cur c; c.d = d; c.e = e; return c; }

DEV uint32_t ld(const uint8_t *p) { return *p; }

// Multi-byte reads from the aligned dwords that hold the bytes: a lane reads
// its own packet, so every load instruction touches 64 different lines and the
// texture-address unit, not HBM, sets the pace -- fewer, wider loads.
// Only dwords holding requested bytes are read (a packet's last aligned
// block is readable, include/mfp.h).
// big-endian value of n (1..4) bytes at p
DEV uint32_t ld_be32n(const uint8_t *p, int n) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t lo = q[0];
    const uint32_t hi = sh + (uint32_t)n > 4 ? q[1] : 0u;
    const uint32_t le = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh)) : lo;   // p[0] in bits 0..7
    return __builtin_bswap32(le) >> (32 - 8 * n);
}
DEV uint64_t ld_be(const uint8_t *p, int n) {          // n = 1..8
    if (n <= 4) return ld_be32n(p, n);
    return ((uint64_t)ld_be32n(p, 4) << (8 * (n - 4))) | ld_be32n(p + 4, n - 4);
}
// up to 32 bytes of p[0, len) as eight little-endian 4-byte groups, from the
// aligned 8-byte words that hold them (at most 5 loads per 32 bytes: the lane
// walkers are bound by their scattered accesses, round 6 r06/r06aa_*), all
// issued before any is used and realigned with static word indices; groups past
// len hold garbage the caller masks.  Only words holding requested bytes are
// read (within the 16-byte block of a packet's last byte, include/mfp.h).
struct LeBlock {
    uint32_t v[8];
    DEV void load(const uint8_t *p, long len) {
        const uintptr_t a = (uintptr_t)p;
        const uint64_t *q = (const uint64_t *)(a & ~(uintptr_t)7);
        const uint32_t sh = (uint32_t)(a & 7) * 8;
        const long nb = len < 32 ? len : 32;
        const int nqw = (int)(((long)(sh / 8) + nb + 7) / 8);   // 1..5
        uint64_t w[5];
#pragma unroll
        for (int k = 0; k < 5; k++) w[k] = k < nqw ? q[k] : 0ull;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t x = sh ? (w[j] >> sh) | (w[j + 1] << (64 - sh)) : w[j];
            v[2 * j] = (uint32_t)x;
            v[2 * j + 1] = (uint32_t)(x >> 32);
        }
    }
};
// 4 bytes (b0 lowest) -> 8 lowercase hex characters, little-endian (b0's high nibble first)
DEV uint64_t hex4(uint32_t le) {
    uint64_t x = le;
    x = (x | (x << 16)) & 0x0000ffff0000ffffull;
    x = (x | (x << 8)) & 0x00ff00ff00ff00ffull;
    const uint64_t nib = ((x >> 4) & 0x000f000f000f000full) | ((x & 0x000f000f000f000full) << 8);
    const uint64_t gt9 = ((nib + 0x7676767676767676ull) & 0x8080808080808080ull) >> 7;
    return nib + 0x3030303030303030ull + gt9 * 0x27;
}

DEV bool cskip(Cur &c, long n) {                       // datum::skip datum.h:365
    if (!c.d) return false;
    if (n > c.e - c.d) { c.d = c.e; return false; }
    c.d += n;
    return true;
}
DEV void cparse(Cur &dst, Cur &r, long n) {            // datum::parse datum.h:294
    if (clen(r) < n || n < 0) { cset_null(r); cset_null(dst); return; }
    dst.d = r.d; dst.e = r.d ? r.d + n : nullptr;
    if (r.d) r.d += n;
}
DEV void cparse_soft(Cur &dst, Cur &r, long n) {       // datum::parse_soft_fail datum.h:305
    long l = clen(r);
    if (l < n) n = l;
    dst.d = r.d; dst.e = r.d ? r.d + n : nullptr;
    if (r.d) r.d += n;
}
DEV bool rd_uint(Cur &c, int n, uint64_t &out) {      // datum::read_uint datum.h:795
    if (c.d && c.d + n <= c.e) {
        const uint64_t v = ld_be(c.d, n);
        c.d += n; out = v; return true;
    }
    cset_null(c); out = 0; return false;
}
DEV uint32_t rd_u8(Cur &c) {                           // datum::read_uint8 datum.h:749
    if (c.d && c.e > c.d) { uint32_t v = ld(c.d); c.d += 1; return v; }
    cset_null(c); return 0;
}
DEV uint32_t look_u8(Cur &c) {                         // datum::lookahead_uint8 datum.h:702
    if (c.d && c.e > c.d) return ld(c.d);
    cset_null(c); return 0;
}
DEV bool look_uint(Cur &c, int n, uint64_t &out) {    // datum::lookahead_uint datum.h:712
    if (c.d && c.d + n <= c.e) {
        out = ld_be(c.d, n); return true;
    }
    return false;
}
DEV void cinit_outer(Cur &dst, Cur &outer, uint64_t len) {  // datum::init_from_outer_parser datum.h:825
    if (!cnotempty(outer)) return;
    const uint8_t *end = (len > (uint64_t)(outer.e - outer.d)) ? outer.e : outer.d + len;
    dst.d = outer.d; dst.e = end; outer.d = end;
}
DEV const uint8_t *cget_ptr(Cur &c, long n) {          // datum::get_pointer datum.h:737
    if (c.d && c.d + n <= c.e) { const uint8_t *p = c.d; c.d += n; return p; }
    return nullptr;
}
DEV void ctrim_to_length(Cur &c, long len) {           // datum::trim_to_length datum.h:383
    if (c.d && len <= (long)(c.e - c.d)) c.e = c.d + len;
}
// ---- SWAR byte classes: bit 7 of each byte of the result flags the byte.
// Exact per byte (no borrow between bytes), so a masked-off byte cannot
// raise a flag next to it.
DEV uint64_t swar_zero(uint64_t x) {
    return ~(((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x) & 0x8080808080808080ull;
}
DEV uint64_t swar_eq(uint64_t w, uint32_t c) { return swar_zero(w ^ (0x0101010101010101ull * (c & 0xff))); }
DEV uint64_t swar_upper(uint64_t w) {                  // 'A'..'Z'
    const uint64_t x = w & 0x7f7f7f7f7f7f7f7full;
    return (x + 0x3f3f3f3f3f3f3f3full) & ~(x + 0x2525252525252525ull) & ~w & 0x8080808080808080ull;
}
DEV uint64_t swar_alpha(uint64_t w) {                  // isalpha (ASCII)
    const uint64_t x = (w | 0x2020202020202020ull) & 0x7f7f7f7f7f7f7f7full;
    return (x + 0x1f1f1f1f1f1f1f1full) & ~(x + 0x0505050505050505ull) & ~w & 0x8080808080808080ull;
}
// first byte of [p, e) whose class flag is set, or e.  A lane scanning its
// own packet: SWB aligned 8-byte loads issued together per memory round trip
// (words inside the range only), then the flags checked in order
#ifndef MFP_SWB
#define MFP_SWB 4
#endif
// (w0: when given, receives the first round's words, from p & ~7)
template <class F>
DEV const uint8_t *swar_find(const uint8_t *p, const uint8_t *e, F flag, uint64_t *w0 = nullptr) {
    if (!p || p >= e) return e;
    const uintptr_t ee = (uintptr_t)e;
    uintptr_t a = (uintptr_t)p & ~(uintptr_t)7;
    uint64_t m0 = ~0ull << (8 * ((uintptr_t)p & 7));   // bytes before p in the first word
    while (true) {
        uint64_t w[MFP_SWB];
#pragma unroll
        for (int k = 0; k < MFP_SWB; k++) w[k] = a + 8 * k < ee ? *(const uint64_t *)(a + 8 * k) : 0ull;
        if (w0) {
#pragma unroll
            for (int k = 0; k < MFP_SWB; k++) w0[k] = w[k];
            w0 = nullptr;
        }
#pragma unroll
        for (int k = 0; k < MFP_SWB; k++) {
            const uintptr_t ak = a + 8 * k;
            if (ak >= ee) return e;
            uint64_t m = flag(w[k]) & (k == 0 ? m0 : ~0ull);
            const uintptr_t in = ee - ak;                  // bytes of this word inside the range
            if (in < 8) m &= (1ull << (8 * in)) - 1;
            if (m) return (const uint8_t *)(ak + (__builtin_ctzll(m) >> 3));
        }
        a += 8 * MFP_SWB;
        m0 = ~0ull;
    }
}
DEV void cparse_to_delim(Cur &dst, Cur &r, uint8_t delim) {   // datum::parse_up_to_delim datum.h:313
    if (!cnotempty(r)) { cset_null(r); cset_null(dst); return; }
    dst.d = r.d;
    const uint8_t *q = swar_find(r.d, r.e, [=](uint64_t w) { return swar_eq(w, delim); });
    if (q < r.e) { dst.e = r.d = q; return; }
    dst.e = r.e;
}
DEV uint32_t cparse_to_delims(Cur &dst, Cur &r, uint8_t d1, uint8_t d2) {   // datum.h:328
    dst.d = r.d;
    if (r.d) {
        const uint8_t *q = swar_find(r.d, r.e, [=](uint64_t w) { return swar_eq(w, d1) | swar_eq(w, d2); });
        r.d = q;
        if (q < r.e) { dst.e = q; return ld(q); }
    }
    dst.e = r.e;
    return 0;
}
// A lane's last SWB loaded words (from a, words at or past the range end e
// left zero) kept across searches of one line: swar_find_w looks there first
// when p lies inside, and records the last round it loads (MFP_HTTP_WIN).
// Precondition: the later searches' ends do not pass the recorded e.
struct SWin {
    uint64_t w[MFP_SWB];
    uintptr_t a = 0, e = 0;
};
template <class F>
DEV const uint8_t *swar_find_w(const uint8_t *p, const uint8_t *e, F flag, SWin &W) {
    if (!p || p >= e) return e;
    const uintptr_t pp = (uintptr_t)p, ee = (uintptr_t)e;
    uintptr_t a;
    uint64_t m0;
    if (W.a && pp >= W.a && pp < W.a + 8 * MFP_SWB && ee <= W.e) {
#pragma unroll
        for (int k = 0; k < MFP_SWB; k++) {
            const uintptr_t ak = W.a + 8 * (uintptr_t)k;
            if (ak + 8 <= pp) continue;
            if (ak >= ee) return e;
            uint64_t m = flag(W.w[k]);
            if (ak < pp) m &= ~0ull << (8 * (pp - ak));
            const uintptr_t in = ee - ak;
            if (in < 8) m &= (1ull << (8 * in)) - 1;
            if (m) return (const uint8_t *)(ak + (__builtin_ctzll(m) >> 3));
        }
        a = W.a + 8 * MFP_SWB;
        m0 = ~0ull;
        if (a >= ee) return e;
    } else {
        a = pp & ~(uintptr_t)7;
        m0 = ~0ull << (8 * (pp & 7));
    }
    while (true) {
#pragma unroll
        for (int k = 0; k < MFP_SWB; k++) W.w[k] = a + 8 * k < ee ? *(const uint64_t *)(a + 8 * k) : 0ull;
        W.a = a;
        W.e = ee;
#pragma unroll
        for (int k = 0; k < MFP_SWB; k++) {
            const uintptr_t ak = a + 8 * k;
            if (ak >= ee) return e;
            uint64_t m = flag(W.w[k]) & (k == 0 ? m0 : ~0ull);
            const uintptr_t in = ee - ak;
            if (in < 8) m &= (1ull << (8 * in)) - 1;
            if (m) return (const uint8_t *)(ak + (__builtin_ctzll(m) >> 3));
        }
        a += 8 * MFP_SWB;
        m0 = ~0ull;
    }
}
// cparse_to_delim / cparse_to_delims through the window (the delimiter's value is not read)
DEV void cparse_to_delim_w(Cur &dst, Cur &r, uint8_t delim, SWin &W) {
    if (!cnotempty(r)) { cset_null(r); cset_null(dst); return; }
    dst.d = r.d;
    const uint8_t *q = swar_find_w(r.d, r.e, [=](uint64_t w) { return swar_eq(w, delim); }, W);
    if (q < r.e) { dst.e = r.d = q; return; }
    dst.e = r.e;
}
DEV void cparse_to_delims_w(Cur &dst, Cur &r, uint8_t d1, uint8_t d2, SWin &W) {
    dst.d = r.d;
    if (r.d) {
        const uint8_t *q = swar_find_w(r.d, r.e, [=](uint64_t w) { return swar_eq(w, d1) | swar_eq(w, d2); }, W);
        r.d = q;
        if (q < r.e) { dst.e = q; return; }
    }
    dst.e = r.e;
}
DEV bool ccompare_n(Cur c, const uint8_t *x, long n) {        // datum::compare_nbytes datum.h:873
    if (!(c.d && clen(c) >= n)) return false;
    for (long i = 0; i < n; i++) if (ld(c.d + i) != ld(x + i)) return false;
    return true;
}
DEV int ccmp(Cur a, Cur b) {                                   // datum::cmp datum.h:456
    if (cnull(a)) return cnull(b) ? 0 : -1;
    if (cnull(b)) return 1;
    long la = clen(a), lb = clen(b), m = la < lb ? la : lb;
    for (long i = 0; i < m; i++) {
        int x = (int)ld(a.d + i), y = (int)ld(b.d + i);
        if (x != y) return x - y;
    }
    return (int)(la - lb);
}
DEV bool c_isupper(uint32_t c) { return c >= 'A' && c <= 'Z'; }
DEV bool c_isalpha(uint32_t c) { return ((c | 0x20) >= 'a') && ((c | 0x20) <= 'z'); }
DEV uint32_t c_tolower(uint32_t c) { return c_isupper(c) ? c + 32 : c; }

// ---------------------------------------------------------------------------
// emitter: restates buffer_stream's truncation rule (buffer_stream.h:100-240)
// as a length count in pass 1; in pass 2 writes bytes with 8-byte stores
// ---------------------------------------------------------------------------
constexpr uint32_t FP_MAX = 8192;   // fingerprint::MAX_FP_STR_LEN fingerprint.h:15

struct TlsPlan;
// FAST >= 0 (k_fp_tls1, TLS format FAST): pass 1 records the ClientHello plan
// with the string's length by arithmetic (tls_ch_plan_fast), pass 2 emits it
// with tls_ch_emit_fast
template <bool EMIT, int FAST_FMT = -1, int LINEW = 8>
struct Em {
    uint32_t n = 0;          // bytes produced
    bool last_putc = false;
    bool punt = false;       // the message needs a parser family this walker lacks
    DEV void punt_pkt() { punt = true; }
    static constexpr int FAST = FAST_FMT;
    static constexpr bool PLAN = !EMIT;   // pass 1 records a ClientHello plan (TlsPlan) in *plan
    TlsPlan *plan = nullptr;              // set by every kernel that runs pass 1 on TLS/DTLS packets
    static constexpr bool SEG = false;
    static constexpr bool emit_pass() { return EMIT; }
    bool spans = false;      // an emitting walk that is the only walk: it also records the hello's spans
    // Pass-2 output.  The string starts 16-byte aligned and owns its slot
    // rounded up to 16 bytes.  Bytes gather in `acc`; whole 8-byte words go
    // to a per-lane line of LINEW words in LDS, and a full line leaves as
    // LINEW / 2 16-byte stores.  Lanes reach a word or line boundary at different
    // pushes, so a store is issued for the lanes that have one; staging the
    // line in LDS makes those (divergent) global stores 8x rarer than
    // storing every word.
    uint8_t *out = nullptr;  // next 64-byte line of the string
    uint8_t *out_end = nullptr; // (optional) end of the string's slot: lines past it are not stored
    uint64_t *line = nullptr;   // this lane's LDS line (8 words)
    uint64_t acc = 0;        // staged bytes of the current word
    uint32_t nacc = 0;       // bytes in acc
    uint32_t nw = 0;         // words in the LDS line
    uint32_t wi = 0;         // words completed (string hash position)
    uint64_t h = 0;          // mfpc::str_hash accumulator of the words so far

    DEV void begin(uint8_t *o, uint64_t *lds_line) {
        out = o;
        line = lds_line;
        acc = 0; nacc = 0; nw = 0; wi = 0; h = 0;
    }
    // the string's mfpc::str_hash (after finish()): the classifier's lookup
    // key, stored behind the string so k_analyze never re-reads it
    DEV uint64_t hash() const { return mfpc::hash_final(h, n); }
    DEV void flush_line(uint32_t words) {       // first `words` words of the line -> out
#ifdef MFP_PROBE_NOSTORE
        if (acc == 0x0123456789abcdefull) *(volatile uint8_t *)out = 0;   // keep the value live
        return;
#endif
        const uint4 *l4 = (const uint4 *)line;
        uint4 *o4 = (uint4 *)out;
        if (out_end && out + 8 * ((words + 1) & ~1u) > out_end) return;   // (an over-long string: dropped anyway)
        for (uint32_t k = 0; 2 * k < words; k++) o4[k] = l4[k];
    }
    DEV void put_word() {
        h ^= mfpc::word_term(acc, wi++);
        line[nw++] = acc;
        if (nw == (uint32_t)LINEW) { flush_line(LINEW); out += 8 * LINEW; nw = 0; }
    }
    DEV void push(uint64_t v, uint32_t k) {     // append k (1..8) bytes, little-endian in v (zero above)
        if (EMIT) {
            const uint32_t room = 8 - nacc;
            if (k < room) {
                acc |= v << (8 * nacc);
                nacc += k;
            } else {
                acc |= (room == 8) ? v : (v << (8 * nacc));
                put_word();
                const uint32_t rest = k - room;
                acc = rest ? (v >> (8 * room)) : 0;
                nacc = rest;
            }
        }
        n += k;
    }
    DEV void finish() {
        if (EMIT) {
            if (nacc) { h ^= mfpc::word_term(acc, wi++); line[nw++] = acc; nacc = 0; }
            if (nw) flush_line(nw);
        }
    }
    DEV void putc(uint32_t c) { push(c & 0xff, 1); last_putc = true; }
    DEV static uint64_t hex2(uint32_t b) {
        uint32_t hi = b >> 4, lo = b & 15;
        uint32_t ch = hi + (hi < 10 ? '0' : 'a' - 10);
        uint32_t cl = lo + (lo < 10 ? '0' : 'a' - 10);
        return (uint64_t)ch | ((uint64_t)cl << 8);
    }
    // raw_as_hex buffer_stream.h:1087 (NULL data -> nothing)
    DEV void hex(const uint8_t *p, long len) {
        if (!p || len <= 0) return;
        last_putc = false;
        if (!EMIT) { n += (uint32_t)(2 * len); return; }
#ifdef MFP_PROBE_NOHEXLOAD
        for (long i = 0; i < len; i++) push(hex2((uint32_t)i), 2);
        return;
#endif
        for (long i0 = 0; i0 < len; i0 += 32) {
            LeBlock blk;
            blk.load(p + i0, len - i0);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const long i = i0 + 4 * k;
                if (i + 4 <= len) {
                    push(hex4(blk.v[k]), 8);
                } else if (i < len) {
                    const uint64_t v = hex4(blk.v[k]);
                    const uint32_t c = (uint32_t)(len - i) * 2;   // 2, 4 or 6 characters
                    push(v & ((1ull << (8 * c)) - 1), c);
                }
            }
        }
    }
    DEV void hex16s(uint32_t m) { n += 4 * m; last_putc = false; }   // m hex16 appends (length only)
    DEV void hex16(uint32_t v) {                // append_uint16_hex buffer_stream.h:425
        last_putc = false;
        uint64_t w = hex2((v >> 8) & 0xff) | (hex2(v & 0xff) << 16);
        push(w, 4);
    }
    DEV void hex8(uint32_t v) { last_putc = false; push(hex2(v & 0xff), 2); }
    DEV void lit(const char *s) {               // puts (strncpy) of a literal
        last_putc = false;
        for (; *s; s++) push((uint8_t)*s, 1);
    }
    // valid iff no append truncated: end <= 8190, or 8191 reached by putc
    DEV bool valid() const { return n <= FP_MAX - 2 || (n == FP_MAX - 1 && last_putc); }
};

// ---------------------------------------------------------------------------
// segment emitter (k_fp_seg): records an HTTP fingerprint as a list of
// segments instead of bytes -- "(" hex(packet bytes) ")" is one segment, the
// type prefix and bare parentheses point into a literal pool -- so that the
// wave can expand the string afterwards with coalesced stores.  Anything an
// HTTP fingerprint does not contain (other literals, hex16/hex8, raw pushes),
// or a list longer than SEG_MAX, sets `ovf`: the packet goes to the fallback
// lane kernel.  A segment is one u32: end character (13 bits), kind (2),
// source offset in the packet or the pool (16).
// ---------------------------------------------------------------------------
constexpr int SEG_MAX = 24;
enum : uint32_t { SK_POOL = 0, SK_HEX = 1, SK_HEXP = 3 };   // SK_HEXP: '(' hex ')'
#define MFP_SEG_POOL "http_server/http/()20ssh_kex_server/ssh_kex/ssh_init_server/ssh_init/ssh_server/ssh/"
constexpr uint32_t POOL_HTTP_SERVER = 0, POOL_HTTP = 12, POOL_OPEN = 17, POOL_CLOSE = 18, POOL_2 = 19, POOL_0 = 20;
constexpr uint32_t SEG_POOL_BYTES = 96;
// a type prefix's place in the pool (fp_type_prefix's literals for HTTP and
// SSH, told apart by first character and length); ~0u: not in the pool
DEV uint32_t seg_pool_lit(uint32_t c0, uint32_t k) {
    if (c0 == 'h') return k == 12 ? 0u : k == 5 ? 12u : ~0u;
    if (c0 != 's') return ~0u;
    switch (k) {
    case 15: return 21;   // ssh_kex_server/
    case 8: return 36;    // ssh_kex/
    case 16: return 44;   // ssh_init_server/
    case 9: return 60;    // ssh_init/
    case 11: return 69;   // ssh_server/
    case 4: return 80;    // ssh/
    }
    return ~0u;
}
DEV uint32_t seg_end(uint32_t s) { return s & 0x1fff; }
DEV uint32_t seg_kind(uint32_t s) { return (s >> 13) & 3; }
DEV uint32_t seg_src(uint32_t s) { return s >> 15; }

struct HdrKey;
struct SegEm {
    static constexpr bool SEG = true;
    // (MFP_HTTP_NAMEWIN) LDS copies of the header-name tables, set by k_fp_seg
    const uint8_t *slots_req = nullptr, *slots_resp = nullptr;
    const HdrKey *keys_req = nullptr, *keys_resp = nullptr;
    static constexpr bool PLAN = false;
    static constexpr bool emit_pass() { return false; }
    static constexpr bool spans = false;
    uint32_t n = 0;                     // characters produced
    bool last_putc = false;
    bool ovf = false;
    const uint8_t *base;                // packet start: hex sources are offsets from it
    uint32_t *seg;                      // this lane's list (LDS)
    uint32_t nseg = 0;
    bool open = false;                  // '(' produced, not yet stored
    uint32_t sp_src = 0, sp_len = 0;    // hex bytes right after the open '(' (0 = none)

    DEV SegEm(const uint8_t *b, uint32_t *s) : base(b), seg(s) {}
    DEV void punt_pkt() { ovf = true; }
    DEV void store(uint32_t kind, uint32_t src, uint32_t end) {
        if (nseg >= (uint32_t)SEG_MAX) { ovf = true; return; }
        seg[nseg++] = (end & 0x1fff) | (kind << 13) | (src << 15);
    }
    DEV void flush_open() {
        if (!open) return;
        if (sp_len) {
            store(SK_POOL, POOL_OPEN, n - 2 * sp_len);
            store(SK_HEX, sp_src, n);
        } else {
            store(SK_POOL, POOL_OPEN, n);
        }
        open = false; sp_len = 0;
    }
    DEV void putc(uint32_t c) {
        c &= 0xff;
        if (c == ')' && open) {                           // "(hex)" or "()"
            if (sp_len) store(SK_HEXP, sp_src, n + 1);
            else store(SK_POOL, POOL_OPEN, n + 1);
            open = false; sp_len = 0;
        } else {
            flush_open();
            if (c == '(') open = true;
            else if (c == ')') store(SK_POOL, POOL_CLOSE, n + 1);
            else if (c == '2') store(SK_POOL, POOL_2, n + 1);     // the SSH protocol/comment delimiter "20"
            else if (c == '0') store(SK_POOL, POOL_0, n + 1);
            else ovf = true;
        }
        n += 1;
        last_putc = true;
    }
    DEV void hex(const uint8_t *p, long len) {
        if (!p || len <= 0) return;
        last_putc = false;
        const uint32_t src = (uint32_t)(p - base);
        if (open && !sp_len) { sp_src = src; sp_len = (uint32_t)len; }
        else { flush_open(); store(SK_HEX, src, n + 2 * (uint32_t)len); }
        n += 2 * (uint32_t)len;
    }
    DEV void lit(const char *s) {
        flush_open();
        last_putc = false;
        uint32_t k = 0;
        while (s[k]) k++;
        const uint32_t at = seg_pool_lit((uint8_t)s[0], k);
        if (at != ~0u) store(SK_POOL, at, n + k);
        else ovf = true;
        n += k;
    }
    DEV void hex16(uint32_t) { ovf = true; n += 4; last_putc = false; }
    DEV void hex16s(uint32_t m) { ovf = true; n += 4 * m; last_putc = false; }
    DEV void hex8(uint32_t) { ovf = true; n += 2; last_putc = false; }
    DEV void push(uint64_t, uint32_t k) { ovf = true; n += k; }
    DEV void finish() { flush_open(); }
    DEV bool valid() const { return n <= FP_MAX - 2 || (n == FP_MAX - 1 && last_putc); }
};

DEV uint32_t hexch(uint32_t nib) { return nib + (nib < 10 ? '0' : 'a' - 10); }

// XOR over the 64 lanes of a wave (every lane gets the result; all lanes active)
DEV uint64_t wave_xor64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        lo ^= (uint32_t)__shfl_xor((int)lo, d, 64);
        hi ^= (uint32_t)__shfl_xor((int)hi, d, 64);
    }
    return ((uint64_t)hi << 32) | lo;
}

// Wave-cooperative expansion of one segment list (k_fp_seg): lane l writes
// characters [512 r + 8 l, +8) of round r with one 8-byte store, and folds
// its words into the string hash (mfpc::str_hash); returns this lane's part
// of the hash accumulator (XOR over the wave gives the whole).  A lane whose
// 8 characters are hex digits of one segment converts 4-5 source bytes with
// one SWAR step; other lanes go character by character.
DEV uint64_t seg_expand(const uint32_t *sg, uint32_t nseg, const uint8_t *pkt, uint32_t T, uint8_t *out,
                        const uint8_t *pool, uint32_t lane) {
    uint64_t h = 0;
    for (uint32_t r0 = 0; r0 < T; r0 += 512) {
        const uint32_t p0 = r0 + 8 * lane;
        if (p0 >= T) continue;
        uint32_t lo = 0, hi = nseg - 1;               // first segment ending after p0
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (seg_end(sg[mid]) > p0) hi = mid; else lo = mid + 1;
        }
        uint32_t s = lo, info = sg[s];
        uint32_t s_end = seg_end(info), s_start = s ? seg_end(sg[s - 1]) : 0;
        const uint32_t kind = seg_kind(info), q0 = p0 - s_start;
        const uint32_t hq = kind == SK_HEXP ? q0 - 1 : q0;           // hex digit index
        const uint32_t hend = kind == SK_HEXP ? s_end - 1 : s_end;    // end of the hex digits
        uint64_t word = 0;
        if (kind != SK_POOL && (kind != SK_HEXP || q0 >= 1) && p0 + 8 <= hend) {
            const uintptr_t a = (uintptr_t)(pkt + seg_src(info) + (hq >> 1));
            const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)(a & 3), nb = 4 + (hq & 1);
            const uint32_t w0 = q[0];
            const uint32_t w1 = sh + nb > 4 ? q[1] : 0u;
            const uint64_t v = (((uint64_t)w1 << 32) | w0) >> (8 * sh);
            const uint64_t x = hex4((uint32_t)v);
            word = (hq & 1) ? (x >> 8) | (hex4((uint32_t)(v >> 32)) << 56) : x;
        } else {
            uintptr_t wa = ~(uintptr_t)0;
            uint32_t wv = 0;
            for (uint32_t k = 0; k < 8; k++) {
                const uint32_t p = p0 + k;
                if (p >= T) break;
                if (p >= s_end) { s++; s_start = s_end; info = sg[s]; s_end = seg_end(info); }
                const uint32_t kd = seg_kind(info), q = p - s_start;
                uint32_t c;
                if (kd == SK_POOL) {
                    c = pool[seg_src(info) + q];
                } else if (kd == SK_HEXP && q == 0) {
                    c = '(';
                } else if (kd == SK_HEXP && p == s_end - 1) {
                    c = ')';
                } else {
                    const uint32_t hd = kd == SK_HEXP ? q - 1 : q;
                    const uintptr_t a = (uintptr_t)(pkt + seg_src(info) + (hd >> 1));
                    if ((a >> 2) != wa) { wa = a >> 2; wv = *(const uint32_t *)(a & ~(uintptr_t)3); }
                    const uint32_t by = (wv >> (8 * (a & 3))) & 0xff;
                    c = hexch((hd & 1) ? (by & 15) : (by >> 4));
                }
                word |= (uint64_t)c << (8 * k);
            }
        }
        *(uint64_t *)(out + p0) = word;
        h ^= mfpc::word_term(word, p0 >> 3);
    }
    return h;
}

// degrease_uint16 (tls.h:776) of the two byte pairs of a little-endian word
// (pair = bytes 0,1 and 2,3, the first byte the high one)
DEV uint32_t degrease_pairs(uint32_t le) {
    const uint32_t b0 = le & 0xff, b1 = (le >> 8) & 0xff, b2 = (le >> 16) & 0xff, b3 = le >> 24;
    const uint32_t lo = (b0 == b1 && (b0 & 15) == 10) ? 0x0a0au : (le & 0xffff);
    const uint32_t hi = (b2 == b3 && (b2 & 15) == 10) ? 0x0a0au : (le >> 16);
    return lo | (hi << 16);
}
DEV uint64_t low_chars(uint64_t v, uint32_t k) { return k >= 8 ? v : (v & ((1ull << (8 * k)) - 1)); }
// raw_as_hex (buffer_stream.h:1087) / raw_as_hex_degrease (tls.h:802, len
// even) of p[0, len), 4 bytes -> 8 characters per push
template <bool DEGREASE, class E>
DEV void hex_run(E &b, const uint8_t *p, uint32_t len) {
    // 32 bytes per round trip: the block's dword loads are all issued before
    // the first is used (LeBlock), then 8 characters per push
    for (uint32_t i0 = 0; i0 < len; i0 += 32) {
        LeBlock blk;
#ifdef MFP_PROBE_HEXRUN_NOLOAD   // (profiling probe only: the value loads' cost)
#pragma unroll
        for (int k = 0; k < 8; k++) blk.v[k] = (uint32_t)(uintptr_t)p + i0 + k;
#else
        blk.load(p + i0, (long)(len - i0));
#endif
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t i = i0 + 4 * (uint32_t)k;
            if (i < len) {
                uint32_t w = blk.v[k];
                if (DEGREASE) w = degrease_pairs(w);
                const uint32_t c = len - i >= 4 ? 8u : 2 * (len - i);
                b.push(low_chars(hex4(w), c), c);
            }
        }
    }
}
// Lane emission of one segment list (k_fp_seg): the lane writes its own
// string, 4 packet bytes -> 8 hex characters per push, so the 64 lanes of a
// wave write 64 strings at once (the wave-cooperative expansion above writes
// one string at a time).  Every segment takes the same instructions whatever
// its kind; `pool` is the literal pool in LDS.
template <class E>
DEV void seg_emit_lane(E &b, const uint32_t *sg, uint32_t nseg, const uint8_t *pkt, const uint8_t *pool) {
    uint32_t start = 0;
    for (uint32_t s = 0; s < nseg; s++) {
        const uint32_t info = sg[s], end = seg_end(info), kind = seg_kind(info), src = seg_src(info);
        const uint32_t k = end - start;
        start = end;
        if (kind == SK_POOL) {                            // at most 12 characters ("http_server/")
            uint64_t w0 = 0, w1 = 0;
            for (uint32_t i = 0; i < k; i++) {
                const uint64_t c = pool[src + i];
                if (i < 8) w0 |= c << (8 * i); else w1 |= c << (8 * (i - 8));
            }
            b.push(w0, k < 8 ? k : 8);
            b.push(w1, k > 8 ? k - 8 : 0);
        } else {
            const bool paren = kind == SK_HEXP;
            b.push(paren ? '(' : 0u, paren ? 1u : 0u);
            hex_run<false>(b, pkt + src, (k - (paren ? 2u : 0u)) / 2);
            b.push(paren ? ')' : 0u, paren ? 1u : 0u);
        }
    }
}

// ---------------------------------------------------------------------------
// TLS (tls.h)
// ---------------------------------------------------------------------------
DEV uint32_t degrease16(uint32_t x) {                   // degrease_uint16 tls.h:776
    if ((x & 0x0f0f) == 0x0a0a && ((x >> 12) == ((x >> 4) & 15))) return 0x0a0a;
    return x;
}
template <class E>
DEV void hex_degrease(E &b, const uint8_t *p, long len) {   // raw_as_hex_degrease tls.h:802
    if (len % 2) len--;
    if (!E::emit_pass()) {                       // pass 1: lengths only
        if (len >= 2) b.hex16s((uint32_t)(len / 2));
        return;
    }
    for (long i0 = 0; i0 < len; i0 += 32) {
        LeBlock blk;
        blk.load(p + i0, len - i0);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const long i = i0 + 4 * k;               // bytes i..i+3, little-endian in v[k]
            if (i < len) {
                const uint32_t v = blk.v[k];
                b.hex16(degrease16(((v & 0xff) << 8) | ((v >> 8) & 0xff)));
                if (i + 2 < len) b.hex16(degrease16((((v >> 16) & 0xff) << 8) | (v >> 24)));
            }
        }
    }
}
DEV bool is_static_ext(uint32_t t) {                    // static_extension_types tls.h:1000
    switch (t) {
    case 1: case 5: case 7: case 8: case 9: case 10: case 11: case 13: case 15: case 16: case 17:
    case 24: case 27: case 28: case 0x39: case 43: case 45: case 50: case 21760: case 0xffa5:
        return true;
    }
    return false;
}
struct Ext {
    uint32_t type, length, encoded_type;
    const uint8_t *type_ptr, *length_ptr;
    Cur value;
    bool ok;
};
DEV Ext ext_parse(Cur &p) {                             // tls_extension ctor tls.h:1383
    Ext x;
    x.type = x.length = x.encoded_type = 0;
    x.type_ptr = p.d; x.length_ptr = nullptr; x.ok = false; cset_null(x.value);
    uint64_t v;
    if (!rd_uint(p, 2, v)) return x;
    x.type = (uint32_t)v;
    x.length_ptr = p.d;
    if (!rd_uint(p, 2, v)) return x;
    x.length = (uint32_t)v;
    if ((long)x.length <= clen(p)) {
        x.value.d = p.d; x.value.e = p.d + x.length; p.d += x.length; x.ok = true;
    }
    x.encoded_type = ((x.type & 0x0f0f) == 0x0a0a) ? 0x0a0a : x.type;
    return x;
}
DEV bool ext_is_grease(uint32_t t) { return (t & 0x0f0f) == 0x0a0a; }

template <class E>
DEV void ext_degreased_value(E &b, const Ext &x, long ungreased) {   // tls.h:1513
    if (!cnotempty(x.value)) return;
    long vl = clen(x.value), skip, gl;
    if (ungreased < vl) { skip = ungreased; gl = vl - ungreased; } else { skip = vl; gl = 0; }
    b.hex(x.value.d, skip);
    hex_degrease(b, x.value.d + skip, gl);
}

// QUIC transport parameters inside a TLS extension (tls.h:1237-1262,
// quic_vli.hpp:30-113)
DEV int vli_len(uint32_t b) { return (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1; }
DEV uint64_t vli_value(Cur c) {
    uint32_t b = rd_u8(c);
    int len = vli_len(b);
    uint64_t v = b & 0x3f;
    for (int i = 1; i < len; i++) v = v * 256 + rd_u8(c);
    return v;
}
DEV bool qtp_parse(Cur &d, Cur &id) {                   // quic_transport_parameter ctor tls.h:1247
    uint32_t b = look_u8(d);
    cparse(id, d, vli_len(b));
    uint32_t bb = rd_u8(d);
    int l2 = vli_len(bb);
    uint64_t v = bb & 0x3f;
    for (int i = 1; i < l2; i++) v = v * 256 + rd_u8(d);
    Cur val;
    long vlen = (v > 0x7fffffffffffffffULL) ? -1 : (long)v;
    cparse(val, d, vlen);
    return !cnull(val);
}
DEV bool qtp_is_grease(Cur id) { return vli_value(id) % 31 == 27; }
// variable_length_integer (quic_vli.hpp): a failed read yields 0 and a null cursor
DEV uint64_t vli_rd(Cur &c) {
    const uint32_t b = rd_u8(c);
    const int len = vli_len(b);
    uint64_t v = b & 0x3f;
    for (int i = 1; i < len; i++) v = v * 256 + rd_u8(c);
    return v;
}
template <class E>
DEV void qtp_write_id(E &b, Cur id) {
    if (!qtp_is_grease(id)) b.hex(id.d, clen(id));
    else { b.putc('1'); b.putc('b'); }
}
DEV bool qtp_less(Cur a, Cur b) {                       // fmt-1 id comparator tls.h:1453
    bool ga = qtp_is_grease(a), gb = qtp_is_grease(b);
    if (ga) { if (gb) return false; return 0x1b < vli_value(b); }
    if (gb) return vli_value(a) < 0x1b;
    return ccmp(a, b) < 0;
}

// The sorted transport parameter ids of a 0x39 / 0xffa5 extension
// (fingerprint_format1 tls.h:1440-1470) from one parse: each id's sort key in
// a register list (insertion by max/min), then written in order.  The key:
// GREASE ids as 0x1b, the others by value -- the comparator's byte order
// (datum::cmp) for minimally encoded ids -- then the wire offset.  Returns
// false, having written nothing, for more than QTP_MAX ids, a non-minimal
// encoding or a value past 2^46 (the caller's selection handles those).
constexpr int QTP_MAX = 16;
template <class E>
DEV bool qtp_sorted_fp(E &b, const Ext &x) {
    uint64_t K[QTP_MAX];
#pragma unroll
    for (int k = 0; k < QTP_MAX; k++) K[k] = ~0ull;
    uint32_t cnt = 0;
    Cur v = x.value;
    while (!cnull(v)) {
        Cur id;
        if (!qtp_parse(v, id)) continue;
        if (cnt >= (uint32_t)QTP_MAX) return false;
        const uint32_t L = (uint32_t)clen(id);
        const uint64_t val = vli_value(id);
        const bool minimal = L == 1 || (L == 2 && val >= 64) || (L == 4 && val >= 16384) || (L == 8 && val >= (1ull << 30));
        if (!minimal || val >= (1ull << 46)) return false;
        const uint64_t key = ((val % 31 == 27 ? 0x1bull : val) << 17) | (uint64_t)(id.d - x.value.d);
        uint64_t prev = 0;
#pragma unroll
        for (int k = 0; k < QTP_MAX; k++) {
            const uint64_t old = K[k];
            const uint64_t hi = prev > key ? prev : key;
            K[k] = hi < old ? hi : old;
            prev = old;
        }
        cnt++;
    }
    for (uint32_t j = 0; j < cnt; j++) {
        const uint64_t e = K[0];
#pragma unroll
        for (int k = 0; k + 1 < QTP_MAX; k++) K[k] = K[k + 1];
        Cur id;
        id.d = x.value.d + (e & 0x1ffff);
        id.e = id.d + vli_len(ld(id.d));
        b.putc('('); qtp_write_id(b, id); b.putc(')');
    }
    return true;
}

// fmt-1 output of one extension: tls_extension::fingerprint_format1 tls.h:1413
template <class E>
DEV void ext_fp1(E &b, Ext &x, int role) {
    if (is_static_ext(x.type)) {
        if (x.type == 0x000a || x.type == 0x002b) {
            b.putc('('); b.hex16(x.encoded_type);
            if (x.length_ptr) hex_degrease(b, x.length_ptr, 2);
            ext_degreased_value(b, x, x.type == 0x000a ? 2 : (role == 0 ? 1 : 0));
            b.putc(')');
        } else if (x.type == 0x39 || x.type == 0xffa5) {
            b.putc('('); b.putc('('); b.hex16(x.encoded_type); b.putc(')');
            b.putc('[');
            // selection order == std::sort order for the (consistent) comparator
            Cur prev; cset_null(prev);
            bool have_prev = false;
            long prev_pos = -1;
            const bool sorted = qtp_sorted_fp(b, x);
            while (!sorted) {
                Cur best; cset_null(best); long best_pos = -1;
                Cur v = x.value; long pos = 0;
                while (!cnull(v)) {
                    Cur id;
                    bool ok = qtp_parse(v, id);
                    if (ok) {
                        bool after = !have_prev || qtp_less(prev, id) ||
                                     (!qtp_less(id, prev) && pos > prev_pos);
                        if (after) {
                            bool better = best_pos < 0 || qtp_less(id, best) ||
                                          (!qtp_less(best, id) && pos < best_pos);
                            if (better) { best = id; best_pos = pos; }
                        }
                        pos++;
                    }
                }
                if (best_pos < 0) break;
                b.putc('('); qtp_write_id(b, best); b.putc(')');
                prev = best; prev_pos = best_pos; have_prev = true;
            }
            b.putc(']');
            b.putc(')');
        } else {
            b.putc('('); b.hex16(x.encoded_type);
            if (x.length_ptr) hex_degrease(b, x.length_ptr, 2);
            if (cnotempty(x.value)) b.hex(x.value.d, clen(x.value));
            b.putc(')');
        }
    } else {
        b.putc('('); b.hex16(x.encoded_type); b.putc(')');
    }
}

// format 0 output of one extension (the loop body of tls_extensions::fingerprint, tls.h:1553-1613)
template <class E>
DEV void ext_fp0(E &b, const Ext &x, int role) {
    if (is_static_ext(x.type)) {
        if (x.type == 0x000a || x.type == 0x002b) {
            b.putc('(');
            if (x.type_ptr) hex_degrease(b, x.type_ptr, 2);
            if (x.length_ptr) hex_degrease(b, x.length_ptr, 2);
            ext_degreased_value(b, x, x.type == 0x000a ? 2 : (role == 0 ? 1 : 0));
            b.putc(')');
        } else if (x.type == 0x39 || x.type == 0xffa5) {
            b.putc('('); b.putc('(');
            if (x.type_ptr) hex_degrease(b, x.type_ptr, 2);
            b.putc(')');
            b.putc('(');
            Cur v = x.value;
            while (!cnull(v)) {
                Cur id;
                if (qtp_parse(v, id)) { b.putc('('); qtp_write_id(b, id); b.putc(')'); }
            }
            b.putc(')'); b.putc(')');
        } else {
            b.putc('(');
            if (x.type_ptr) hex_degrease(b, x.type_ptr, 2);
            if (x.length_ptr) hex_degrease(b, x.length_ptr, 2);
            if (cnotempty(x.value)) b.hex(x.value.d, clen(x.value));
            b.putc(')');
        }
    } else {
        b.putc('(');
        if (x.type_ptr) hex_degrease(b, x.type_ptr, 2);
        b.putc(')');
    }
}

// format 0: tls_extensions::fingerprint tls.h:1549
template <class E>
DEV void exts_fp0(E &b, Cur exts, int role) {
    Cur p = exts;
    b.putc('(');
    while (clen(p) > 0) {
        Ext x = ext_parse(p);
        if (!x.ok) break;
        ext_fp0(b, x, role);
    }
    b.putc(')');
}

// tls_extensions_assign::get_index tls_extensions.h:15-110
DEV int fmt2_index(uint32_t t) {
    if (t <= 20) return (int)t;
    if (t >= 22 && t <= 34) return (int)t - 1;
    if (t >= 36 && t <= 40) return (int)t - 2;
    if (t >= 43 && t <= 62) return (int)t - 4;
    switch (t) {
    case 2570: return 59; case 13172: return 60; case 21760: return 61; case 30031: return 62;
    case 30032: return 63; case 64768: return 64; case 65037: return 65; case 65280: return 66;
    case 65281: return 67; case 65283: return 68; case 65445: return 69; case 65486: return 70;
    }
    return -1;
}
// fmt-2 bucket after the private/unassigned remap (tls.h:1680-1693)
DEV int fmt2_bucket_t(uint32_t type, uint32_t &encoded_type) {
    int idx = fmt2_index(type);
    if (idx == -1) {
        if (type == 65280 || type >= 65282) encoded_type = 65280;
        else if (type >= 62 && type <= 65279 && !ext_is_grease(type)) encoded_type = 62;
        idx = fmt2_index(encoded_type);
    }
    return idx;
}
DEV int fmt2_bucket(Ext &x) { return fmt2_bucket_t(x.type, x.encoded_type); }

// ordering key of an extension for formats 1 and 2.  Returns a 32-bit
// primary key; ties (same primary) are broken by ext_tie_less.
//   fmt 1 (tls.h:1637): grease == type 0x0a0a, then type, length, value
//   fmt 2 (tls.h:1709): bucket, then (grease first...) length, value
DEV uint32_t ext_key(const Ext &x, int fmt, int bucket) {
    if (fmt == 1) {
        bool g = ext_is_grease(x.type);
        return g ? (0x0a0aU << 16) : ((x.type << 16) | x.length);
    }
    bool g = ext_is_grease(x.type);
    return ((uint32_t)bucket << 24) | (g ? 0 : (1u << 23)) | (g ? 0 : x.length);
}
// strict "less" on full comparator given equal primary keys
DEV bool ext_tie_less(const Ext &a, const Ext &b) {
    if (ext_is_grease(a.type) || ext_is_grease(b.type)) return false;
    return ccmp(a.value, b.value) < 0;
}

// Formats 1 and 2 keep the extensions they emit as a sorted list in
// registers: (primary key << 32 | wire offset), insertion-sorted as they are
// parsed, so equal keys stay in wire order.  No LDS scratch per lane (the
// previous 192-byte per-lane list halved the lane kernel's occupancy).  Equal
// non-GREASE primary keys (a repeated extension type and length) need the
// reference's value comparison, and more than REG_EXT kept extensions do not
// fit: both take the selection over the wire list below (same total order).
#ifndef MFP_REG_EXT
#define MFP_REG_EXT 24
#endif
constexpr int REG_EXT = MFP_REG_EXT;
DEV bool key_is_grease(uint32_t key, int fmt) {
    return fmt == 1 ? (key >> 16) == 0x0a0a : !(key & (1u << 23));
}

// formats 1 and 2: sort kept extensions, then emit fingerprint_format1 each
template <class E>
DEV void exts_fp12(E &b, Cur exts, int role, int fmt) {
    b.putc('[');
    uint64_t V[REG_EXT];
#pragma unroll
    for (int k = 0; k < REG_EXT; k++) V[k] = ~0ull;
    int n = 0;
    bool rare = false;
    {
        Cur p = exts;
        while (clen(p) > 0) {
            const uint8_t *start = p.d;
            Ext x = ext_parse(p);
            if (!x.ok) break;
            int bucket = 0;
            if (fmt == 2) {
                bucket = fmt2_bucket(x);
                if (bucket < 0) continue;
                // keep the first three per bucket (tls.h:1695-1701)
                int cnt = 0;
#pragma unroll
                for (int k = 0; k < REG_EXT; k++) cnt += (V[k] != ~0ull && (uint32_t)(V[k] >> 56) == (uint32_t)bucket);
                if (cnt >= 3) continue;
            }
            if (n >= REG_EXT) { rare = true; break; }
            const uint32_t key = ext_key(x, fmt, bucket);
            const uint64_t v = ((uint64_t)key << 32) | (uint32_t)(start - exts.d);
            uint32_t pos = 0;
            bool tie = false;
#pragma unroll
            for (int k = 0; k < REG_EXT; k++) {
                pos += V[k] < v ? 1u : 0u;
                tie |= (uint32_t)(V[k] >> 32) == key;
            }
            if (tie && !key_is_grease(key, fmt)) rare = true;
#pragma unroll
            for (int k = REG_EXT - 1; k > 0; k--) V[k] = (uint32_t)k > pos ? V[k - 1] : ((uint32_t)k == pos ? v : V[k]);
            if (pos == 0) V[0] = v;
            n++;
        }
    }
    if (!rare) {
        // emit in key order (pass 1 only counts; the order does not change the length)
        for (int j = 0; j < n; j++) {
            const uint32_t off = (uint32_t)V[0];
#pragma unroll
            for (int k = 0; k < REG_EXT - 1; k++) V[k] = V[k + 1];
            Cur q = cmk(exts.d + off, exts.e);
            Ext x = ext_parse(q);
            if (fmt == 2) fmt2_bucket(x);
            ext_fp1(b, x, role);
        }
    } else {
        // selection over the wire list, O(n^2), the reference's comparator
        // (key, then value bytes, then wire position)
        uint32_t prev_key = 0; long prev_pos = -1; bool have_prev = false;
        Ext prev_x; prev_x.type = 0; prev_x.length = 0; cset_null(prev_x.value);
        while (true) {
            long best_pos = -1; uint32_t best_key = 0; Ext best_x; best_x.type = 0; cset_null(best_x.value);
            Cur p = exts; long pos = 0;
            while (clen(p) > 0) {
                Ext x = ext_parse(p);
                if (!x.ok) break;
                long mypos = pos++;
                int bucket = 0;
                if (fmt == 2) {
                    bucket = fmt2_bucket(x);
                    if (bucket < 0) continue;
                    // count earlier kept in bucket
                    Cur q = exts; int cnt = 0; long qp = 0;
                    while (qp < mypos && clen(q) > 0) {
                        Ext y = ext_parse(q);
                        if (!y.ok) break;
                        qp++;
                        if (fmt2_bucket(y) == bucket) cnt++;
                    }
                    if (cnt >= 3) continue;
                }
                uint32_t k = ext_key(x, fmt, bucket);
                auto lt = [&](uint32_t ka, const Ext &xa, long pa, uint32_t kb, const Ext &xb, long pb) {
                    if (ka != kb) return ka < kb;
                    if (ext_tie_less(xa, xb)) return true;
                    if (ext_tie_less(xb, xa)) return false;
                    return pa < pb;
                };
                bool after = !have_prev || lt(prev_key, prev_x, prev_pos, k, x, mypos);
                if (!after) continue;
                if (best_pos < 0 || lt(k, x, mypos, best_key, best_x, best_pos)) {
                    best_pos = mypos; best_key = k; best_x = x;
                }
            }
            if (best_pos < 0) break;
            ext_fp1(b, best_x, role);
            prev_key = best_key; prev_pos = best_pos; prev_x = best_x; have_prev = true;
        }
    }
    b.putc(']');
}

}  // namespace mfp

namespace mfp {

// ---------------------------------------------------------------------------
// TLS handshake containers (tls.h:145-262), ClientHello/ServerHello/Cert
// ---------------------------------------------------------------------------
DEV Cur tls_record_fragment(Cur &d) {                   // tls_record::parse tls.h:153
    Cur f; cset_null(f);
    if (clen(d) < 5) return f;
    uint64_t t, len;
    rd_uint(d, 1, t); rd_uint(d, 2, t); rd_uint(d, 2, len);
    cinit_outer(f, d, len);
    return f;
}
struct Hs { uint32_t msg_type; uint64_t length; Cur body; uint64_t more; };
DEV Hs tls_hs_parse(Cur &d) {                           // tls_handshake::parse tls.h:244
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
struct Ch { Cur version, ciphers, compression, extensions; };
DEV Ch tls_ch_parse(Cur p) {                            // tls_client_hello::parse tls.h:1811
    Ch ch; cset_null(ch.version); cset_null(ch.ciphers); cset_null(ch.compression); cset_null(ch.extensions);
    uint64_t l;
    Cur t;
    cparse(ch.version, p, 2);
    if (!cnotempty(ch.version)) return ch;
    bool dtls = ld(ch.version.d) == 0xfe;
    cparse(t, p, 32);
    if (!rd_uint(p, 1, l)) return ch;
    cparse(t, p, (long)l);
    if (dtls) {
        if (!look_uint(p, 1, l)) return ch;
        if (!cskip(p, (long)l + 1)) return ch;
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
template <class E>
DEV void tls_ch_fp(E &b, const Ch &ch, int fmt) {   // tls.h:1928
    if (fmt >= 1 && fmt <= 2) { b.putc('0' + fmt); b.putc('/'); }
    b.putc('('); b.hex(ch.version.d, clen(ch.version)); b.putc(')');
    b.putc('('); hex_degrease(b, ch.ciphers.d, clen(ch.ciphers)); b.putc(')');
    if (fmt == 0) exts_fp0(b, ch.extensions, 0);
    else exts_fp12(b, ch.extensions, 0, fmt);
}
// tls_extensions::set_meta_data tls.h:1316 (server_name; last one wins)
// the ALPN extension's protocol_name_list (tls.h:1357-1362, protocol_name_list
// tls.h:1172-1176: a 16-bit length, then that many bytes; short: none)
DEV void tls_alpn(const uint8_t *start, const uint8_t *end, const uint8_t *base, uint32_t &off, uint32_t &len) {
    Cur e = cmk(start, end);
    cskip(e, 4);
    uint64_t l;
    if (rd_uint(e, 2, l) && (uint64_t)clen(e) >= l) { off = (uint32_t)(e.d - base); len = (uint32_t)l; }
    else { off = 0; len = 0xffff; }
}
// the user agent of a quic_transport_parameters_draft extension [start, end)
// (tls_extensions::set_meta_data tls.h:1346-1355: transport parameter 0x3129,
// quic_transport_parameter tls.h:1244; the last one wins and a value that does
// not parse is a null -- empty -- user agent).  It takes the record's ua span,
// which otherwise holds the ALPN list, and sets MFP_XF_TLS_UA; the ALPN list is
// then re-read from the packet by the host outputs.
DEV void tls_draft_ua(const uint8_t *start, const uint8_t *end, const uint8_t *base, uint32_t &off, uint32_t &len,
                      uint32_t &xf) {
    Cur e = cmk(start, end);
    cskip(e, 4);
    while (clen(e) > 0) {
        Cur id; cparse(id, e, vli_len(look_u8(e)));
        const uint64_t vl = vli_rd(e);
        Cur val; cparse(val, e, (long)vl);
        if (vli_value(id) == 0x3129) {
            off = cnull(val) ? 0u : (uint32_t)(val.d - base);
            len = cnull(val) ? 0u : (uint32_t)clen(val);
            xf |= MFP_XF_TLS_UA;
        }
    }
}
// server name (tls_extensions::set_meta_data tls.h:1316-1366; the last one
// wins) and ALPN list of a ClientHello's extensions
DEV void tls_sni(Cur exts, const uint8_t *base, uint32_t &off, uint32_t &len, uint32_t &aoff, uint32_t &alen,
                 uint32_t &xf) {
    Cur p = exts;
    while (clen(p) > 0) {
        const uint8_t *start = p.d;
        uint64_t t, l;
        if (!rd_uint(p, 2, t)) break;
        if (!rd_uint(p, 2, l)) break;
        if (!cskip(p, (long)l)) break;
        if (t == 0) {
            Cur e = cmk(start, p.d);
            cskip(e, 9);
            off = (uint32_t)(e.d - base); len = (uint32_t)clen(e);
        }
        if (t == 16 && !(xf & MFP_XF_TLS_UA)) tls_alpn(start, p.d, base, aoff, alen);
        if (t == 0xffa5) tls_draft_ua(start, p.d, base, aoff, alen, xf);
    }
}
// ClientHello plan: pass 1 of the lane kernels records what pass 2 needs to
// write the fingerprint -- the ClientHello's version and cipher datums and its
// extensions in emission order (format 0: wire order; formats 1/2: the sorted
// list, key << 32 | offset) -- so pass 2 writes the string without walking the
// link, IP, TCP and TLS headers and the extension list again.  More than
// REG_EXT extensions, or a tie that needs value comparison, leaves the plan
// unset and pass 2 walks the packet as before.
struct TlsPlan {
    uint32_t O[REG_EXT / 2];   // extension offsets in emission order, two 16-bit offsets per word
    Cur version, ciphers, exts;
    uint32_t n, type, fmt;
    bool ok;
    // the fast plan (k_fp_tls1): the lane's rows in LDS -- the kept
    // extensions by wire index (ext_row: header and offset), and the emission
    // order as wire indices
    uint32_t *off_row = nullptr;   // ext_row entries (below)
    uint8_t *ord_row = nullptr;
    uint8_t *win = nullptr;    // (k_fp_tls1) the extension-header window in LDS (ExtWin::wv)
    uint8_t *win2 = nullptr;   // (k_fp_tls1, MFP_EXT_WIN_BLOCKS > 4) its blocks from the fifth on
    uint32_t win_lane = 0;
};

// pass 1 of a TLS/DTLS ClientHello: fingerprint length (through the counting
// emitter), the server name (tls_extensions::set_meta_data tls.h:1316, last
// one wins) and the plan -- one walk over the extension list
template <class E>
DEV void tls_ch_plan(E &b, TlsPlan &pl, const Ch &ch, int fmt, uint32_t type, const uint8_t *base,
                     uint32_t &sni_off, uint32_t &sni_len, uint32_t &alpn_off, uint32_t &alpn_len, uint32_t &xf) {
    pl.ok = false;
    fp_type_prefix(b, type);
    if (fmt >= 1 && fmt <= 2) { b.putc('0' + fmt); b.putc('/'); }
    b.putc('('); b.hex(ch.version.d, clen(ch.version)); b.putc(')');
    b.putc('('); hex_degrease(b, ch.ciphers.d, clen(ch.ciphers)); b.putc(')');
    const uint32_t n0 = b.n;
    b.putc(fmt == 0 ? '(' : '[');
    uint64_t V[REG_EXT];                         // key << 32 | offset, in emission order
#pragma unroll
    for (int k = 0; k < REG_EXT; k++) V[k] = ~0ull;
    int n = 0;
    bool rare = false;
    Cur p = ch.extensions;
    while (clen(p) > 0) {
        const uint8_t *start = p.d;
        Ext x = ext_parse(p);
        if (!x.ok) break;
        if (x.type == 0) {                       // server_name: bytes after the 9-byte header (tls.h:1342)
            Cur e = cmk(start, p.d);
            cskip(e, 9);
            sni_off = (uint32_t)(e.d - base); sni_len = (uint32_t)clen(e);
        }
        if (x.type == 16 && !(xf & MFP_XF_TLS_UA)) tls_alpn(start, p.d, base, alpn_off, alpn_len);
        if (x.type == 0xffa5) tls_draft_ua(start, p.d, base, alpn_off, alpn_len, xf);
        if (rare) continue;
        int bucket = 0;
        if (fmt == 2) {
            bucket = fmt2_bucket(x);
            if (bucket < 0) continue;
            int cnt = 0;                         // first three per bucket (tls.h:1695-1701)
#pragma unroll
            for (int k = 0; k < REG_EXT; k++) cnt += (V[k] != ~0ull && (uint32_t)(V[k] >> 56) == (uint32_t)bucket);
            if (cnt >= 3) continue;
        }
        if (n >= REG_EXT) { rare = true; continue; }
        const uint32_t off = (uint32_t)(start - ch.extensions.d);
        if (fmt == 0) {
#pragma unroll
            for (int k = 0; k < REG_EXT; k++) if (k == n) V[k] = off;
            ext_fp0(b, x, 0);
        } else {
            const uint32_t key = ext_key(x, fmt, bucket);
            const uint64_t v = ((uint64_t)key << 32) | off;
            uint32_t pos = 0;
            bool tie = false;
#pragma unroll
            for (int k = 0; k < REG_EXT; k++) {
                pos += V[k] < v ? 1u : 0u;
                tie |= (uint32_t)(V[k] >> 32) == key;
            }
            if (tie && !key_is_grease(key, fmt)) rare = true;
#pragma unroll
            for (int k = REG_EXT - 1; k > 0; k--)
                V[k] = (uint32_t)k > pos ? V[k - 1] : ((uint32_t)k == pos ? v : V[k]);
            if (pos == 0) V[0] = v;
            ext_fp1(b, x, 0);
        }
        n++;
    }
    if (rare) {                                  // length by the general walk; pass 2 re-walks
        b.n = n0;
        if (fmt == 0) exts_fp0(b, ch.extensions, 0);
        else exts_fp12(b, ch.extensions, 0, fmt);
        return;
    }
    b.putc(fmt == 0 ? ')' : ']');
#pragma unroll
    for (int k = 0; k < REG_EXT / 2; k++) pl.O[k] = ((uint32_t)V[2 * k] & 0xffff) | ((uint32_t)V[2 * k + 1] << 16);
    pl.version = ch.version; pl.ciphers = ch.ciphers; pl.exts = ch.extensions;
    pl.n = (uint32_t)n; pl.type = type; pl.fmt = (uint32_t)fmt;
    pl.ok = true;
}

// pass 2 from the plan: the same bytes tls_client_hello::fingerprint writes
// (tls.h:1928-1964)
template <class E>
DEV void tls_ch_emit(E &b, TlsPlan &pl) {
    fp_type_prefix(b, pl.type);
    const int fmt = (int)pl.fmt;
    if (fmt >= 1) { b.putc('0' + fmt); b.putc('/'); }
    b.putc('('); b.hex(pl.version.d, clen(pl.version)); b.putc(')');
    b.putc('('); hex_degrease(b, pl.ciphers.d, clen(pl.ciphers)); b.putc(')');
    b.putc(fmt == 0 ? '(' : '[');
    for (uint32_t j = 0; j < pl.n; j++) {
        const uint32_t off = pl.O[0] & 0xffff;
#pragma unroll
        for (int k = 0; k < REG_EXT / 2; k++)             // pop the front offset
            pl.O[k] = (pl.O[k] >> 16) | (k + 1 < REG_EXT / 2 ? pl.O[k + 1] << 16 : 0u);
        Cur q = cmk(pl.exts.d + off, pl.exts.e);
        Ext x = ext_parse(q);
        if (fmt == 0) {
            ext_fp0(b, x, 0);
        } else {
            if (fmt == 2) fmt2_bucket(x);
            ext_fp1(b, x, 0);
        }
    }
    b.putc(fmt == 0 ? ')' : ']');
}

// ---------------------------------------------------------------------------
// The ClientHello plan with the length by arithmetic, and a uniform emitter
// (k_fp_tls1).  The lanes of a wave hold different ClientHellos: the general
// emitter's per-type branches (ext_fp0 / ext_fp1) run for the union of the
// wave's extension types, byte pushes at a time.  Here every extension takes
// the same instructions -- one 4-byte header load, a head word of up to 9
// characters made branch-free, then the value as runs of 4 bytes -> 8 hex
// characters -- so a wave's cost follows its longest string, not the union of
// its paths.  The characters are tls_client_hello::fingerprint's (tls.h:1928-
// 1964; extensions: tls_extensions::fingerprint tls.h:1549-1613 for format 0,
// fingerprint_format1 tls.h:1413-1470 for formats 1/2).  QUIC transport
// parameters (0x39, 0xffa5) leave the plan unset: the fallback lane writes them.
// ---------------------------------------------------------------------------
DEV bool static_ext_bit(uint32_t t) {                   // static_extension_types tls.h:1000
    constexpr uint64_t M = (1ull << 1) | (1ull << 5) | (1ull << 7) | (1ull << 8) | (1ull << 9) | (1ull << 10) |
                           (1ull << 11) | (1ull << 13) | (1ull << 15) | (1ull << 16) | (1ull << 17) | (1ull << 24) |
                           (1ull << 27) | (1ull << 28) | (1ull << 43) | (1ull << 45) | (1ull << 50) | (1ull << 57);
    return t < 64 ? ((M >> t) & 1) != 0 : (t == 21760 || t == 0xffa5);
}
// characters an extension adds (ext_fp0 / ext_fp1 agree on every length)
DEV uint32_t ext_fp_len(uint32_t t, uint32_t vl) {
    if (!static_ext_bit(t)) return 6;                   // "(" type ")"
    if (t == 0x000a || t == 0x002b) {                   // ext_degreased_value tls.h:1513 (client role)
        const uint32_t ung = t == 0x000a ? 2u : 1u;
        const uint32_t skip = vl < ung ? vl : ung;
        return 10 + 2 * skip + 2 * ((vl - skip) & ~1u);
    }
    return 10 + 2 * vl;                                  // "(" type length value ")"
}
// At most FAST_EXT kept extensions (MFP_FAST_EXT; more leave the plan unset).
#ifndef MFP_FAST_EXT
#define MFP_FAST_EXT 24
#endif
constexpr int FAST_EXT = MFP_FAST_EXT;
// Formats 1/2 order the kept extensions by a 32-bit key (ext_key32): the
// field the reference's comparator looks at first, then the length, then the
// wire index (so equal keys keep wire order); the sorted list lives in 24
// registers and an insertion is a max and a min per entry (inserting v into a
// sorted list: new[k] = min(max(old[k-1], v), old[k]), no position search).  Equal keys that need the
// reference's value comparison, lengths past the key's field and more than
// FAST_EXT kept extensions leave the plan unset (the fallback lane writes them).
DEV uint32_t ext_key32(const Ext &x, int fmt, int bucket, uint32_t idx, bool &fits) {
    const bool g = ext_is_grease(x.type);
    if (fmt == 1) {                              // tls.h:1637: GREASE as 0x0a0a, then type, length
        fits = g || x.length < 2048;
        return g ? ((0x0a0au << 16) | idx) : ((x.type << 16) | ((x.length & 2047) << 5) | idx);
    }
    fits = true;                                 // tls.h:1709: bucket, GREASE first, length
    return ((uint32_t)bucket << 24) | (g ? 0u : (1u << 23)) | (g ? 0u : (x.length << 5)) | idx;
}
DEV bool key32_grease(uint32_t k, int fmt) { return fmt == 1 ? (k >> 16) == 0x0a0a : !(k & (1u << 23)); }

// The extension headers of a ClientHello through a per-lane 64-byte LDS
// window filled by four independent 16-byte loads (k_fp_tls1): a run of short
// extensions costs one memory round trip instead of one per header (each
// header's address depends on the previous length, tls.h:1383).  Only the
// blocks that hold bytes before `end` are loaded (the 16-byte block holding a
// packet's last byte is readable, include/mfp.h); bytes past `end` in the
// window are never used.
#ifndef MFP_EXT_WIN
#define MFP_EXT_WIN 2
#endif
// 16-byte blocks in the window (MFP_EXT_WIN 2): 4 = 64 bytes per lane
#ifndef MFP_EXT_WIN_BLOCKS
#define MFP_EXT_WIN_BLOCKS 4
#endif
// MFP_EXT_WIN 2: the blocks go straight to LDS (global_load_lds_dwordx4, no
// VGPRs); the wave's window area is 4 x 1 KiB, block k of lane l at
// wv + 1024 k + 16 l (the instruction writes lane l's 16 bytes at the
// wave-uniform base + 16 l).  MFP_EXT_WIN 1: through VGPRs into a per-lane
// 64-byte row.
struct ExtWin {
    uint8_t *wv;                 // the wave's window area in LDS (4 KiB; MFP_EXT_WIN 1: the lane's 64-byte row)
    uint32_t lane;
    const uint8_t *base;         // the window's first byte (16-byte aligned); nullptr: empty
    uint8_t *wv2;                // blocks 4.. of the window (MFP_EXT_WIN_BLOCKS > 4)
    DEV uint8_t *blk(uint32_t b) const { return b < 4 ? wv + 1024 * b : wv2 + 1024 * (b - 4); }
    DEV const uint32_t *dw(uint32_t k) const {
        return MFP_EXT_WIN == 2 ? (const uint32_t *)(blk(k >> 2) + 16 * lane + 4 * (k & 3))
                                : (const uint32_t *)wv + k;
    }
};
// the 4 bytes at a, big-endian (a < end; bytes at or past end are garbage)
DEV uint32_t win_be32(ExtWin &wn, const uint8_t *a, const uint8_t *end) {
    uint64_t o = (uint64_t)(a - wn.base);
    constexpr uint32_t NB = MFP_EXT_WIN == 2 ? MFP_EXT_WIN_BLOCKS : 4;
    if (wn.base == nullptr || a < wn.base || o > 16 * NB - 8) {
        const uint8_t *b = (const uint8_t *)((uintptr_t)a & ~(uintptr_t)15);
        const uint4 *s = (const uint4 *)b;
        if (MFP_EXT_WIN == 2) {
#pragma unroll
            for (uint32_t k = 0; k < NB; k++)
                if (k == 0 || b + 16 * k < end)
                    __builtin_amdgcn_global_load_lds((const void *)(s + k),
                                                     (void __attribute__((address_space(3))) *)(wn.blk(k)),
                                                     16, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            const uint4 z = make_uint4(0, 0, 0, 0);
            const uint4 v0 = s[0];
            const uint4 v1 = b + 16 < end ? s[1] : z;
            const uint4 v2 = b + 32 < end ? s[2] : z;
            const uint4 v3 = b + 48 < end ? s[3] : z;
            uint4 *w4 = (uint4 *)wn.wv;
            w4[0] = v0; w4[1] = v1; w4[2] = v2; w4[3] = v3;
        }
        wn.base = b;
        o = (uint64_t)(a - b);
    }
    const uint32_t k = (uint32_t)o >> 2, sh = (uint32_t)o & 3;
    const uint32_t lo = *wn.dw(k), hi = *wn.dw(k + 1);
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, sh));
}
// ext_parse (tls_extension ctor tls.h:1383) with the header from the window
DEV Ext ext_parse_win(Cur &p, ExtWin &wn) {
    if (!MFP_EXT_WIN || !wn.wv || !p.d || p.e - p.d < 4) return ext_parse(p);
    Ext x;
    const uint32_t th = win_be32(wn, p.d, p.e);
    x.type = th >> 16; x.length = th & 0xffff;
    x.type_ptr = p.d; x.length_ptr = p.d + 2;
    x.encoded_type = ((x.type & 0x0f0f) == 0x0a0a) ? 0x0a0a : x.type;
    p.d += 4;
    x.ok = (long)x.length <= p.e - p.d;
    if (x.ok) { x.value.d = p.d; x.value.e = p.d + x.length; p.d += x.length; }
    else cset_null(x.value);
    return x;
}

// A kept extension in the plan's LDS row (k_fp_tls1), so the emission reads
// no extension header again: a static extension (its value is printed) as
// 1 << 31 | type code << 22 | length << 11 | offset in the extension block
// (type code: the type, below 64, or 63 for 21760; length and offset at most
// 2047, else the plan is left unset); any other as its 16-bit type (only the
// type is printed)
DEV uint32_t ext_row(uint32_t t, uint32_t vl, uint32_t off, bool st) {
    return st ? (1u << 31) | ((t < 64 ? t : 63u) << 22) | (vl << 11) | off : t;
}
DEV uint32_t ext_row_type(uint32_t er) {
    if (!(er >> 31)) return er & 0xffff;
    const uint32_t tc = (er >> 22) & 63u;
    return tc == 63 ? 21760u : tc;
}
template <int FMT, class E>
DEV void tls_ch_plan_fast(E &b, TlsPlan &pl, const Ch &ch, uint32_t type, const uint8_t *base,
                          uint32_t &sni_off, uint32_t &sni_len, uint32_t &alpn_off, uint32_t &alpn_len) {
    pl.ok = false;
    // type prefix, "1/" or "2/", "(" version ")" "(" degreased ciphers ")", "(" or "[", ... ")" or "]"
    uint32_t n = (type == 10 ? 5u : 4u) + (FMT ? 2u : 0u) + 2 + 2 * (uint32_t)clen(ch.version) + 2 +
                 2 * ((uint32_t)clen(ch.ciphers) & ~1u) + 2;
    uint32_t V[FAST_EXT];                         // formats 1/2: sorted ext_key32 values
#pragma unroll
    for (int k = 0; k < FAST_EXT; k++) V[k] = ~0u;
    uint32_t cnt = 0;
    bool rare = false;
    Cur p = ch.extensions;
    ExtWin wn{pl.win, pl.win_lane, nullptr, pl.win2};
    while (clen(p) > 0) {
        const uint8_t *start = p.d;
        Ext x = ext_parse_win(p, wn);
        if (!x.ok) break;
        if (x.type == 0) {                       // server_name: bytes after the 9-byte header (tls.h:1342)
            Cur e = cmk(start, p.d);
            cskip(e, 9);
            sni_off = (uint32_t)(e.d - base); sni_len = (uint32_t)clen(e);
        }
        if (x.type == 16) {                      // tls_alpn: protocol_name_list tls.h:1172-1176
            if (MFP_EXT_WIN && wn.wv) {
                const uint32_t l = x.length >= 2 ? win_be32(wn, start + 4, p.e) >> 16 : 0u;
                if (x.length >= 2 && x.length - 2 >= l) { alpn_off = (uint32_t)(start + 6 - base); alpn_len = l; }
                else { alpn_off = 0; alpn_len = 0xffff; }
            } else {
                tls_alpn(start, p.d, base, alpn_off, alpn_len);
            }
        }
        // a draft transport-parameter extension may carry the user agent
        // (tls_draft_ua): the fallback lane writes such a hello's record
        if (x.type == 0xffa5) rare = true;
        if (rare) continue;
        int bucket = 0;
        if (FMT == 2) {
            bucket = fmt2_bucket(x);
            if (bucket < 0) continue;
            uint32_t c3 = 0;                     // first three per bucket (tls.h:1695-1701)
#pragma unroll
            for (int k = 0; k < FAST_EXT; k++) c3 += (V[k] >> 24) == (uint32_t)bucket ? 1u : 0u;
            if (c3 >= 3) continue;
        }
        if (cnt >= (uint32_t)FAST_EXT || x.type == 0x39 || x.type == 0xffa5) { rare = true; continue; }
        {
            const uint32_t off = (uint32_t)(start - ch.extensions.d);
            const bool st = static_ext_bit(x.type);
            if (st && (off > 2047 || x.length > 2047)) { rare = true; continue; }
            pl.off_row[cnt] = ext_row(x.type, x.length, off, st);
        }
        if (FMT != 0) {
            bool fits;
            const uint32_t v = ext_key32(x, FMT, bucket, cnt, fits);
            rare |= !fits;
#ifdef MFP_PROBE_NOSORT   // (profiling probe only: the insertion's cost; wrong order for formats 1/2)
#pragma unroll
            for (int k = 0; k < FAST_EXT; k++) if ((uint32_t)k == cnt) V[k] = v;
#else
            uint32_t prev = 0;
#pragma unroll
            for (int k = 0; k < FAST_EXT; k++) {  // insert v into the sorted list
                const uint32_t old = V[k];
                const uint32_t hi = prev > v ? prev : v;
                V[k] = hi < old ? hi : old;
                prev = old;
            }
#endif
        }
        n += ext_fp_len(x.type, (uint32_t)clen(x.value));
        cnt++;
    }
    if (FMT != 0 && !rare) {                     // equal keys the reference orders by value
#pragma unroll
        for (int k = 0; k + 1 < FAST_EXT; k++)
            rare |= V[k + 1] != ~0u && (V[k] >> 5) == (V[k + 1] >> 5) && !key32_grease(V[k], FMT);
    }
    b.n = n;
    b.last_putc = true;                          // the string ends with ")" or "]"
    if (rare) return;
    if (FMT != 0) {
#pragma unroll
        for (int k = 0; k < FAST_EXT; k++) if ((uint32_t)k < cnt) pl.ord_row[k] = (uint8_t)(V[k] & 31);
    }
    pl.version = ch.version; pl.ciphers = ch.ciphers; pl.exts = ch.extensions;
    pl.n = cnt; pl.type = type; pl.fmt = (uint32_t)FMT;
    pl.ok = true;
}
template <int FMT, class E>
DEV void tls_ch_emit_fast(E &b, TlsPlan &pl) {
    if (pl.type == 10) b.push(0x2f736c7464ull, 5);                         // "dtls/"
    else b.push(0x2f736c74ull, 4);                                          // "tls/"
    if (FMT) b.push((uint64_t)('0' + FMT) | ((uint64_t)'/' << 8), 2);
    {   // "(" version ")(": the version is 2 bytes (tls_ch_parse parsed it whole)
        const uint32_t v = ld_be32n(pl.version.d, 2);
        const uint64_t hx = hex4(__builtin_bswap32(v << 16));
        b.push('(' | ((hx & 0xffffffffull) << 8) | ((uint64_t)')' << 40) | ((uint64_t)'(' << 48), 7);
    }
    hex_run<true>(b, pl.ciphers.d, (uint32_t)clen(pl.ciphers) & ~1u);
    b.push(')' | ((FMT ? '[' : '(') << 8), 2);
    // the extension headers come from the plan's rows (no packet loads)
    for (uint32_t j = 0; j < pl.n; j++) {
        const uint32_t er = pl.off_row[FMT == 0 ? j : pl.ord_row[j]];
        const bool st = er >> 31;
        const uint32_t t = ext_row_type(er), vl = st ? (er >> 11) & 2047u : 0u;
        const uint8_t *h = pl.exts.d + (er & 2047u);
        const uint32_t th = (t << 16) | vl;                // type << 16 | length (the plan kept whole extensions)
        uint32_t w;                                        // head: type, length as a little-endian word
        if (FMT == 0) {
            w = degrease_pairs(__builtin_bswap32(th));     // hex_degrease of type and length (tls.h:1560-1600)
        } else {
            uint32_t enc = ext_is_grease(t) ? 0x0a0au : t;  // tls_extension::encoded_type (tls.h:1390)
            if (FMT == 2) fmt2_bucket_t(t, enc);
            w = ((enc >> 8) & 0xff) | ((enc & 0xff) << 8) | (degrease_pairs(__builtin_bswap32(th)) & 0xffff0000u);
        }
        const uint64_t hx = hex4(w);
        // static: "(" + 8 head characters (+ value + ")"); other: "(" type ")"
        b.push(st ? ('(' | (hx << 8)) : ('(' | ((hx & 0xffffffffull) << 8) | ((uint64_t)')' << 40)), st ? 8u : 6u);
        if (st) {
            b.push(hx >> 56, 1);
            uint32_t skip = vl, gl = 0;
            if (t == 0x000a || t == 0x002b) {              // ext_degreased_value tls.h:1513
                const uint32_t ung = t == 0x000a ? 2u : 1u;
                skip = vl < ung ? vl : ung;
                gl = (vl - skip) & ~1u;
            }
            hex_run<false>(b, h + 4, skip);
            hex_run<true>(b, h + 4 + skip, gl);
            b.push(')', 1);
        }
    }
    b.push(FMT ? ']' : ')', 1);
    b.last_putc = true;
}

struct Sh { Cur version, cipher, extensions; };
DEV Sh tls_sh_parse(Cur &rec) {                         // parse_tls_server_hello tls.h:2097
    Sh s; cset_null(s.version); cset_null(s.cipher); cset_null(s.extensions);
    uint64_t l; Cur t;
    cparse(s.version, rec, 2);
    cparse(t, rec, 32);
    if (!look_uint(rec, 1, l)) return s;
    if (!cskip(rec, (long)l + 1)) return s;
    cparse(s.cipher, rec, 2);
    cparse(t, rec, 1);
    if (!rd_uint(rec, 2, l)) return s;
    cparse(s.extensions, rec, (long)l);
    return s;
}
DEV bool tls_sh_not_empty(const Sh &s) {                // tls_server_hello::is_not_empty tls.h:513
    Cur t = s.version; uint64_t v;
    rd_uint(t, 2, v);
    if (!(v == 0x0303 || v == 0x0302 || v == 0x0301 || v == 0x0300 || v == 0xfeff || v == 0xfefd)) return false;
    return cnotempty(s.cipher);
}
template <class E>
DEV void tls_sh_fp(E &b, const Sh &s) {                 // tls_server_hello::fingerprint tls.h:2126
    b.putc('('); b.hex(s.version.d, clen(s.version)); b.putc(')');
    b.putc('('); b.hex(s.cipher.d, clen(s.cipher)); b.putc(')');
    exts_fp0(b, s.extensions, 1);
}
struct Cert { Cur list; uint64_t more; };
DEV void tls_cert_parse(Cert &c, Cur &d) {              // tls_server_certificate::parse tls.h:281
    uint64_t t = 0;
    if (!rd_uint(d, 3, t)) return;
    if (t > 65536) { cset_null(d); return; }
    cinit_outer(c.list, d, t);
    c.more = t - (uint64_t)clen(c.list);
}

// ---------------------------------------------------------------------------
// SSH (ssh.h)
// ---------------------------------------------------------------------------
struct SshBin { Cur payload; uint64_t more; };
DEV SshBin ssh_bin_parse(Cur &p) {                      // ssh_binary_packet ssh.h:56
    SshBin b; cset_null(b.payload); b.more = 0;
    uint64_t plen, pad;
    rd_uint(p, 4, plen);
    rd_uint(p, 1, pad);
    if (plen > 16384 || plen < 1) { if (p.d) p.d = p.e; return b; }
    if (!cnotempty(p)) return b;
    long left = (long)plen - 1;
    if (left > clen(p)) b.more = left - clen(p);
    cparse_soft(b.payload, p, left);
    return b;
}
// ssh_kex_init::parse ssh.h:190; returns the kex_algorithms name-list and
// leaves the 10 name-lists' extents retrievable by re-walking
DEV void name_list_parse(Cur &nl, Cur &p) {             // name_list::parse ssh.h:110
    uint64_t l;
    rd_uint(p, 4, l);
    if (l > 2048) { if (p.d) p.d = p.e; return; }
    cparse(nl, p, (long)l);
}
// The 10 name-lists of a KEXINIT, parsed once for the check and the
// fingerprint: each as offset << 16 | length from the payload's start, ~0u
// when null (ssh_kex_init::parse ssh.h:190; a payload is at most 16 KiB, a
// list at most 2048 bytes)
struct SshKex {
    uint32_t nl[10];
    bool ok;                                            // the kex_algorithms list is not empty
};
DEV SshKex ssh_kex_parse(Cur payload) {
    SshKex k;
    Cur p = payload, t;
    cparse(t, p, 1);
    cparse(t, p, 16);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        Cur l;
        cset_null(l);
        name_list_parse(l, p);
        k.nl[i] = cnull(l) ? ~0u : ((uint32_t)(l.d - payload.d) << 16) | (uint32_t)clen(l);
    }
    k.ok = k.nl[0] != ~0u && (k.nl[0] & 0xffff) != 0;
    return k;
}
template <class E>
DEV void ssh_kex_fp(E &b, Cur payload, const SshKex &k) {   // ssh_kex_init::fingerprint ssh.h:240
#pragma unroll
    for (int i = 0; i < 10; i++) {
        b.putc('(');
        if (k.nl[i] != ~0u && (k.nl[i] & 0xffff)) b.hex(payload.d + (k.nl[i] >> 16), (long)(k.nl[i] & 0xffff));
        b.putc(')');
    }
}

// ---------------------------------------------------------------------------
// HTTP (http.h, http.cc) -- header-name tables in constant memory
// ---------------------------------------------------------------------------
// (len, include_value, capture, name): http.cc:426-445 (request) and
// :487-536 (response); capture: 1 host, 2 user-agent
#define MFP_REQ_NAMES(X)                                                                                          \
    X(6, 1, 0, "accept") X(15, 1, 0, "accept-encoding") X(10, 1, 0, "connection") X(3, 1, 0, "dnt")              \
    X(3, 1, 0, "dpr") X(25, 1, 0, "upgrade-insecure-requests") X(16, 1, 0, "x-requested-with")                    \
    X(14, 0, 0, "accept-charset") X(15, 0, 0, "accept-language") X(13, 0, 0, "authorization")                     \
    X(13, 0, 0, "cache-control") X(4, 0, 1, "host") X(17, 0, 0, "if-modified-since") X(10, 0, 0, "keep-alive")    \
    X(10, 0, 2, "user-agent") X(15, 0, 0, "x-flash-version") X(14, 0, 0, "x-p2p-peerdist")
#define MFP_RESP_NAMES(X)                                                                                         \
    X(32, 1, 0, "access-control-allow-credentials") X(28, 1, 0, "access-control-allow-headers")                   \
    X(28, 1, 0, "access-control-allow-methods") X(29, 1, 0, "access-control-expose-headers")                      \
    X(13, 1, 0, "cache-control") X(4, 1, 0, "code") X(10, 1, 0, "connection") X(16, 1, 0, "content-language")     \
    X(25, 1, 0, "content-transfer-encoding") X(3, 1, 0, "p3p") X(6, 1, 0, "pragma") X(6, 1, 0, "reason")          \
    X(6, 1, 0, "server") X(25, 1, 0, "strict-transport-security") X(7, 1, 0, "version")                           \
    X(19, 1, 0, "x-aspnetmvc-version") X(16, 1, 0, "x-aspnet-version") X(5, 1, 0, "x-cid")                        \
    X(12, 1, 0, "x-ms-version") X(16, 1, 0, "x-xss-protection")                                                   \
    X(17, 0, 0, "appex-activity-id") X(7, 0, 0, "cdnuuid") X(6, 0, 0, "cf-ray") X(13, 0, 0, "content-range")      \
    X(12, 0, 0, "content-type") X(4, 0, 0, "date") X(4, 0, 0, "etag") X(7, 0, 0, "expires")                       \
    X(12, 0, 0, "flow_context") X(5, 0, 0, "ms-cv") X(8, 0, 0, "msregion") X(12, 0, 0, "ms-requestid")            \
    X(10, 0, 0, "request-id") X(4, 0, 0, "vary") X(12, 0, 0, "x-amz-cf-pop") X(16, 0, 0, "x-amz-request-id")      \
    X(24, 0, 0, "x-azure-ref-originshield") X(7, 0, 0, "x-cache") X(12, 0, 0, "x-cache-hits")                     \
    X(5, 0, 0, "x-ccc") X(14, 0, 0, "x-diagnostic-s") X(10, 0, 0, "x-feserver") X(4, 0, 0, "x-hw")                \
    X(12, 0, 0, "x-msedge-ref") X(19, 0, 0, "x-ocsp-responder-id") X(11, 0, 0, "x-requestid")                     \
    X(11, 0, 0, "x-served-by") X(7, 0, 0, "x-timer") X(15, 0, 0, "x-trace-context")

// the names as lowercase text packed into four little-endian words (zero
// past the name) for word-at-a-time comparison
struct HdrKey { uint64_t w[4]; uint32_t len, info; };   // info: incl_value | capture << 8
constexpr uint64_t pack_name(const char *s, int len, int k) {
    uint64_t w = 0;
    for (int i = 0; i < 8; i++)
        if (8 * k + i < len) w |= (uint64_t)(uint8_t)s[8 * k + i] << (8 * i);
    return w;
}
#define MFP_HK(len, incl, cap, str) \
    HdrKey{{pack_name(str, len, 0), pack_name(str, len, 1), pack_name(str, len, 2), pack_name(str, len, 3)}, \
           len, (incl) | ((cap) << 8)},
__constant__ HdrKey k_req_keys[] = {MFP_REQ_NAMES(MFP_HK)};
__constant__ HdrKey k_resp_keys[] = {MFP_RESP_NAMES(MFP_HK)};
constexpr HdrKey kReqKeys[] = {MFP_REQ_NAMES(MFP_HK)};
constexpr HdrKey kRespKeys[] = {MFP_RESP_NAMES(MFP_HK)};
#undef MFP_HK
constexpr int N_REQ_NAMES = sizeof(kReqKeys) / sizeof(kReqKeys[0]);
constexpr int N_RESP_NAMES = sizeof(kRespKeys) / sizeof(kRespKeys[0]);
static_assert(N_REQ_NAMES == 17 && N_RESP_NAMES == 49, "http.cc header lists");

// perfect_hash::lookup (perfect_hash.h:256) as a collision-free
// multiplicative hash of the packed lowercase name: slot -> table index + 1;
// the candidate is then compared word for word (exact, any input)
DEV_HD_CONSTEXPR uint64_t name_key(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint64_t len) {
    return w0 + 3 * w1 + 5 * w2 + 7 * w3 + len;
}
constexpr uint64_t REQ_MUL = 0x9531985d5d9dc9f9ull, RESP_MUL = 0xad514947c1ae3f7bull;
constexpr int REQ_BITS = 6, RESP_BITS = 7;
template <int BITS>
struct HdrSlots { uint8_t s[1 << BITS]; bool perfect; };
template <int BITS, int N>
constexpr HdrSlots<BITS> make_slots(const HdrKey (&t)[N], uint64_t mul) {
    HdrSlots<BITS> r{};
    r.perfect = true;
    for (int i = 0; i < N; i++) {
        const uint32_t h = (uint32_t)((name_key(t[i].w[0], t[i].w[1], t[i].w[2], t[i].w[3], t[i].len) * mul) >> (64 - BITS));
        if (r.s[h]) r.perfect = false;
        r.s[h] = (uint8_t)(i + 1);
    }
    return r;
}
constexpr HdrSlots<REQ_BITS> kReqSlots = make_slots<REQ_BITS>(kReqKeys, REQ_MUL);
constexpr HdrSlots<RESP_BITS> kRespSlots = make_slots<RESP_BITS>(kRespKeys, RESP_MUL);
static_assert(kReqSlots.perfect && kRespSlots.perfect, "header name hash must be collision-free");
__constant__ HdrSlots<REQ_BITS> k_req_slots = kReqSlots;
__constant__ HdrSlots<RESP_BITS> k_resp_slots = kRespSlots;

// ASCII A-Z -> a-z in each byte of w (bytes >= 0x80 unchanged)
DEV uint64_t swar_tolower(uint64_t w) {
    const uint64_t x = w & 0x7f7f7f7f7f7f7f7full;
    const uint64_t ge_a = x + 0x3f3f3f3f3f3f3f3full, gt_z = x + 0x2525252525252525ull;
    const uint64_t upper = ge_a & ~gt_z & ~w & 0x8080808080808080ull;
    return w | (upper >> 2);
}

// perfect_hash::lookup perfect_hash.h:256: exact ASCII-case-insensitive
// match -- the lowercased name as four packed words (aligned 8-byte loads of
// the name's bytes), one hashed slot, one word-wise comparison; returns the
// table index and the entry's incl_value | capture << 8
// the table lookup of a name whose aligned words aw[0..4] (from n.d & ~7) are
// loaded; the tables may be the __constant__ ones or LDS copies
DEV int name_match(bool req, Cur n, const uint64_t (&aw)[5], const uint8_t *slots_req, const uint8_t *slots_resp,
                   const HdrKey *keys_req, const HdrKey *keys_resp, uint32_t &info) {
    const long l = clen(n);
    const uint32_t sh = (uint32_t)((uintptr_t)n.d & 7) * 8;
    uint64_t nw[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint64_t w = sh ? (aw[k] >> sh) | (aw[k + 1] << (64 - sh)) : aw[k];
        const long rem = l - 8 * k;
        if (rem <= 0) w = 0;
        else if (rem < 8) w &= (1ull << (8 * rem)) - 1;
        nw[k] = swar_tolower(w);
    }
    const uint64_t key = name_key(nw[0], nw[1], nw[2], nw[3], (uint64_t)l);
    const int c = req ? (int)slots_req[(key * REQ_MUL) >> (64 - REQ_BITS)] - 1
                      : (int)slots_resp[(key * RESP_MUL) >> (64 - RESP_BITS)] - 1;
    if (c < 0) return -1;
    const HdrKey &k = req ? keys_req[c] : keys_resp[c];
    if (k.len == (uint32_t)l && k.w[0] == nw[0] && k.w[1] == nw[1] && k.w[2] == nw[2] && k.w[3] == nw[3]) {
        info = k.info;
        return c;
    }
    return -1;
}
DEV int name_lookup(bool req, Cur n, uint32_t &info) {
    const long l = clen(n);
    if (l <= 0 || l > 32) return -1;
    const uintptr_t a = (uintptr_t)n.d & ~(uintptr_t)7;
    const uint32_t sh = (uint32_t)((uintptr_t)n.d & 7) * 8;
    const uintptr_t end = (uintptr_t)n.e;
    uint64_t aw[5];
#pragma unroll
    for (int k = 0; k < 5; k++) aw[k] = a + 8 * k < end ? *(const uint64_t *)(a + 8 * k) : 0ull;
    uint64_t nw[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint64_t w = sh ? (aw[k] >> sh) | (aw[k + 1] << (64 - sh)) : aw[k];
        const long rem = l - 8 * k;
        if (rem <= 0) w = 0;
        else if (rem < 8) w &= (1ull << (8 * rem)) - 1;
        nw[k] = swar_tolower(w);
    }
    const uint64_t key = name_key(nw[0], nw[1], nw[2], nw[3], (uint64_t)l);
    const int c = req ? (int)k_req_slots.s[(key * REQ_MUL) >> (64 - REQ_BITS)] - 1
                      : (int)k_resp_slots.s[(key * RESP_MUL) >> (64 - RESP_BITS)] - 1;
    if (c < 0) return -1;
    const HdrKey &k = req ? k_req_keys[c] : k_resp_keys[c];
    if (k.len == (uint32_t)l && k.w[0] == nw[0] && k.w[1] == nw[1] && k.w[2] == nw[2] && k.w[3] == nw[3]) {
        info = k.info;
        return c;
    }
    return -1;
}
DEV bool http_delim(Cur &p, Cur del) {                  // delimiter(datum&, const datum&) http.h:113
    Cur dl; cset_null(dl);
    static const uint8_t crlf[2] = {'\r', '\n'};
    if (ccompare_n(p, del.d, clen(del))) cparse(dl, p, clen(del));
    else if (p.d && clen(p) >= 2 && ld(p.d) == '\r' && ld(p.d + 1) == '\n') cparse(dl, p, 2);
    else if (p.d && clen(p) >= 1 && ld(p.d) == '\n') cparse(dl, p, 1);
    (void)crlf;
    return cnotempty(dl);
}
// MFP_HTTP_FAST: the header loop's delimiter checks and the ':' / whitespace
// step read the bytes they test with one block load each (the delimiter
// packed once per message, up to 4 bytes) instead of one dependent byte load
// per comparison
// (A/B on MI355X, profiles/r04w_ab_*, r04x_ab_*: http_req 13.8 -> 11.4 ms and
// http_resp 4.2 -> 3.1 ms with 1; 2 takes http_resp to 2.95 ms)
#ifndef MFP_HTTP_FAST
#define MFP_HTTP_FAST 2
#endif
// p[0, n) (n = 1..4) little-endian, bytes above n zero: from the aligned
// 16-byte block holding p (and the next one when the bytes cross into it)
DEV uint32_t ld_le4n(const uint8_t *p, long n) {
    const uintptr_t a = (uintptr_t)p;
    const uint4 *q = (const uint4 *)(a & ~(uintptr_t)15);
    const uint32_t off = (uint32_t)(a & 15);
    const uint4 x0 = q[0];
    const uint32_t x1 = off + (uint32_t)n > 16 ? q[1].x : 0u;
    const uint32_t i = off >> 2;
    const uint32_t lo = i == 0 ? x0.x : i == 1 ? x0.y : i == 2 ? x0.z : x0.w;
    const uint32_t hi = i == 0 ? x0.y : i == 1 ? x0.z : i == 2 ? x0.w : x1;
    const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, off & 3);
    return n >= 4 ? v : v & ((1u << (8 * n)) - 1);
}
// http_delim with the delimiter packed (dl <= 4 bytes, value dv)
DEV bool http_delim4(Cur &p, uint32_t dv, long dl) {
    if (!p.d) return false;
    const long L = p.e - p.d;
    if (L <= 0) return false;                         // (dl = 0 matches but consumes nothing: false too)
    const uint32_t w = ld_le4n(p.d, L < 4 ? L : 4);
    if (dl <= L && (dl == 0 || (w & (dl >= 4 ? ~0u : (1u << (8 * dl)) - 1)) == dv)) {
        p.d += dl;
        return dl != 0;
    }
    if (L >= 2 && (w & 0xffff) == 0x0a0d) { p.d += 2; return true; }
    if ((w & 0xff) == 0x0a) { p.d += 1; return true; }
    return false;
}
// p[0, n) (n = 1..8) little-endian, bytes above n zero (as ld_le4n)
DEV uint64_t ld_le8n(const uint8_t *p, long n) {
    const uintptr_t a = (uintptr_t)p;
    const uint4 *q = (const uint4 *)(a & ~(uintptr_t)15);
    const uint32_t off = (uint32_t)(a & 15);
    const uint4 x0 = q[0];
    const uint2 x1 = off + (uint32_t)n > 16 ? *(const uint2 *)(q + 1) : make_uint2(0, 0);
    const uint32_t i = off >> 2, sb = off & 3;
    const uint32_t d0 = i == 0 ? x0.x : i == 1 ? x0.y : i == 2 ? x0.z : x0.w;
    const uint32_t d1 = i == 0 ? x0.y : i == 1 ? x0.z : i == 2 ? x0.w : x1.x;
    const uint32_t d2 = i == 0 ? x0.z : i == 1 ? x0.w : i == 2 ? x1.x : x1.y;
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sb) |
                       (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sb) << 32;
    return n >= 8 ? v : v & ((1ull << (8 * n)) - 1);
}
// http_delim4 on bytes already loaded: w holds p[0, min(4, len)) (bytes past
// the cursor's end are never tested)
DEV bool http_delim4w(Cur &p, uint32_t dv, long dl, uint32_t w) {
    if (!p.d) return false;
    const long L = p.e - p.d;
    if (L <= 0) return false;
    if (dl <= L && (dl == 0 || (w & (dl >= 4 ? ~0u : (1u << (8 * dl)) - 1)) == dv)) {
        p.d += dl;
        return dl != 0;
    }
    if (L >= 2 && (w & 0xffff) == 0x0a0d) { p.d += 2; return true; }
    if ((w & 0xff) == 0x0a) { p.d += 1; return true; }
    return false;
}
// the 8 bytes at x (wa <= x, x + 8 <= wa + 32) from four words loaded from wa
DEV uint64_t win_get8(const uint64_t (&w)[4], uintptr_t wa, uintptr_t x) {
    const uint32_t o = (uint32_t)(x - wa), k = o >> 3, sh = (o & 7) * 8;
    const uint64_t lo = k == 0 ? w[0] : k == 1 ? w[1] : k == 2 ? w[2] : w[3];
    const uint64_t hi = k == 0 ? w[1] : k == 1 ? w[2] : k == 2 ? w[3] : 0ull;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}
// MFP_HTTP_WIN (segment walker): a header line's whitespace, value end and
// delimiter come from the ':' search's 32 bytes when they lie in them (most
// header lines), instead of three more memory round trips (round 6:
// http_resp 2.74 -> 2.37 ms, http_req 10.28 -> 10.37, r06/r06r_ab_http_win.txt)
#ifndef MFP_HTTP_WIN
#define MFP_HTTP_WIN 1
#endif
// new_http_headers::fingerprint http.h:335 + httpheader http.h:146
// MFP_HTTP_NAMEWIN (segment walker): the header name's lookup right after the
// ':' search, from that search's words and LDS copies of the tables
// (http_req 11.1 -> 10.0 ms, http_resp 2.9 -> 2.7 at config 4, profiles/r04y_ab_*)
#ifndef MFP_HTTP_NAMEWIN
#define MFP_HTTP_NAMEWIN 1
#endif
template <class E>
DEV void http_headers_fp(E &b, Cur body, Cur delim, bool req, Cur &host, Cur &ua) {
    Cur tmp = body;
    constexpr bool NW = E::SEG && MFP_HTTP_NAMEWIN && MFP_HTTP_FAST >= 1;
#if MFP_HTTP_FAST
    const long dl = clen(delim);
    const uint32_t dv = dl > 0 && dl <= 4 ? ld_le4n(delim.d, dl) : 0u;
    const bool d4 = dl <= 4;
    // (the segment walker leaves longer delimiters to the fallback lane)
    if (E::SEG && !d4) { b.punt_pkt(); return; }
#define MFP_HDELIM(c) ((E::SEG || d4) ? http_delim4(c, dv, dl) : http_delim(c, delim))
    // MFP_HTTP_FAST >= 2 (segment walker): the delimiter after a value is
    // tested from an 8-byte window that also holds the next header's first
    // bytes (the loop-top test reads no memory), and the value's end is
    // searched from the ':' while the whitespace after it is loaded: one
    // memory round trip for both
    constexpr bool F2 = E::SEG && MFP_HTTP_FAST >= 2;
    static_assert(MFP_SWB == 4, "the name window is the ':' search's first four words");
    uint32_t wnext = 0;
    bool have_next = false;
#define MFP_HTOP(c) (F2 && have_next ? http_delim4w(c, dv, dl, wnext) : MFP_HDELIM(c))
#else
#define MFP_HDELIM(c) http_delim(c, delim)
#define MFP_HTOP(c) http_delim(c, delim)
#endif
    while (true) {
        if (MFP_HTOP(tmp)) break;
        Cur hdr_body = tmp, name; cset_null(name);
#if MFP_HTTP_FAST
        // the ':' found is the byte the reference tests next; none found leaves
        // the name's first byte, which is not ':'
        int early_idx = -1;
        uint32_t early_info = 0;
        // (MFP_HTTP_WIN) the ':' search's first 32 bytes, from wa, also serve the
        // whitespace, the value's end and the delimiter when they lie in them
        uint64_t w0[MFP_SWB] = {0, 0, 0, 0};
        uintptr_t wa = 0;
        if (!cnotempty(tmp)) { cset_null(tmp); }
        else {
            name.d = tmp.d; name.e = tmp.e;
            wa = (uintptr_t)tmp.d & ~(uintptr_t)7;
            const uint8_t *q = swar_find(tmp.d, tmp.e, [](uint64_t w) { return swar_eq(w, ':'); }, NW ? w0 : nullptr);
            if (q < tmp.e) {
                name.e = q; tmp.d = q + 1;
                if constexpr (NW) {
                    // the name's table lookup now, from the search's first 32
                    // bytes when they hold the name, and from the LDS tables
                    const long l = q - name.d;
                    const uintptr_t a = (uintptr_t)name.d & ~(uintptr_t)7;
                    if (l > 0 && l <= 32 && (uintptr_t)q <= a + 8 * MFP_SWB) {
                        const uint64_t aw[5] = {w0[0], w0[1], w0[2], w0[3], 0ull};
                        early_idx = name_match(req, name, aw, b.slots_req, b.slots_resp, b.keys_req, b.keys_resp, early_info);
                    } else {
                        early_idx = name_lookup(req, name, early_info);
                    }
                }
            } else cset_null(tmp);
        }
        Cur value;
        if constexpr (F2) {
            // whitespace (up to 4 bytes from one load) and the value's end: the
            // first CR or LF after the ':' is the first after the whitespace,
            // which holds neither
            long L = 0;
            uint32_t w = 0;
            constexpr bool WIN = NW && MFP_HTTP_WIN;
            if (tmp.d && tmp.d < tmp.e) {
                L = tmp.e - tmp.d;
                const long n4 = L < 4 ? L : 4;
                if (WIN && (uintptr_t)tmp.d + 8 <= wa + 8 * MFP_SWB) {
                    const uint32_t x = (uint32_t)win_get8(w0, wa, (uintptr_t)tmp.d);
                    w = n4 >= 4 ? x : x & ((1u << (8 * n4)) - 1);
                } else {
                    w = ld_le4n(tmp.d, n4);
                }
            }
            const uint8_t *q2 = nullptr;
            if (tmp.d) {
                auto crlf = [](uint64_t x) { return swar_eq(x, '\r') | swar_eq(x, '\n'); };
                const uintptr_t s0 = (uintptr_t)tmp.d, ee = (uintptr_t)tmp.e;
                uintptr_t from = s0;
                if constexpr (WIN) {   // the first CR or LF from s0: in the window first
                    bool found = false;
#pragma unroll
                    for (int k = 0; k < MFP_SWB; k++) {
                        const uintptr_t ak = wa + 8 * (uintptr_t)k;
                        if (!found && ak + 8 > s0 && ak < ee) {
                            uint64_t m = crlf(w0[k]);
                            if (ak < s0) m &= ~0ull << (8 * (s0 - ak));
                            const uintptr_t in = ee - ak;
                            if (in < 8) m &= (1ull << (8 * in)) - 1;
                            if (m) { q2 = (const uint8_t *)(ak + (__builtin_ctzll(m) >> 3)); found = true; }
                        }
                    }
                    if (!found) {
                        const uintptr_t wend = wa + 8 * MFP_SWB;
                        from = s0 > wend ? s0 : wend;
                        if (from >= ee) q2 = tmp.e;
                    }
                    if (!found && from < ee) q2 = swar_find((const uint8_t *)from, tmp.e, crlf);
                } else {
                    q2 = swar_find(tmp.d, tmp.e, crlf);
                }
            }
            if (L > 0) {
                int k = 0;
                while (k < 4 && k < L && (((w >> (8 * k)) & 0xff) == '\t' || ((w >> (8 * k)) & 0xff) == ' ')) k++;
                tmp.d += k;
                if (k == 4)
                    while (tmp.d < tmp.e && (ld(tmp.d) == '\t' || ld(tmp.d) == ' ')) tmp.d++;
            }
            // cparse_to_delims(value, tmp, '\r', '\n')
            value.d = tmp.d;
            if (tmp.d) { tmp.d = q2; value.e = q2; } else value.e = tmp.e;
            // the delimiter, and the next header's first bytes, from one window
            uint64_t w8 = 0;
            if (tmp.d && tmp.d < tmp.e) {
                const long L8 = tmp.e - tmp.d, n8 = L8 < 8 ? L8 : 8;
                if (WIN && (uintptr_t)tmp.d + 8 <= wa + 8 * MFP_SWB) {
                    w8 = win_get8(w0, wa, (uintptr_t)tmp.d);
                    if (n8 < 8) w8 &= (1ull << (8 * n8)) - 1;
                } else {
                    w8 = ld_le8n(tmp.d, n8);
                }
            }
            const uint8_t *at = tmp.d;
            http_delim4w(tmp, dv, dl, (uint32_t)w8);
            wnext = (uint32_t)(w8 >> (8 * (uint32_t)(tmp.d - at)));
            have_next = true;
        } else {
        bool more_ws = false;
        if (tmp.d && tmp.d < tmp.e) {                    // up to 4 bytes of whitespace from one load
            const long L = tmp.e - tmp.d;
            const uint32_t w = ld_le4n(tmp.d, L < 4 ? L : 4);
            int k = 0;
            while (k < 4 && k < L && (((w >> (8 * k)) & 0xff) == '\t' || ((w >> (8 * k)) & 0xff) == ' ')) k++;
            tmp.d += k;
            more_ws = k == 4;
        }
        if (more_ws)
            while (tmp.d && tmp.d < tmp.e && (ld(tmp.d) == '\t' || ld(tmp.d) == ' ')) tmp.d++;
        cparse_to_delims(value, tmp, '\r', '\n');
        MFP_HDELIM(tmp);
        }
#else
        const int early_idx = -1;
        const uint32_t early_info = 0;
        if (!cnotempty(tmp)) { cset_null(tmp); }
        else {
            name.d = tmp.d; name.e = tmp.e;
            const uint8_t *q = swar_find(tmp.d, tmp.e, [](uint64_t w) { return swar_eq(w, ':'); });
            if (q < tmp.e) { name.e = q; tmp.d = q; }
        }
        if (tmp.d && tmp.e > tmp.d && ld(tmp.d) == ':') tmp.d++; else cset_null(tmp);
        while (tmp.d && tmp.d < tmp.e && (ld(tmp.d) == '\t' || ld(tmp.d) == ' ')) tmp.d++;
        Cur value;
        cparse_to_delims(value, tmp, '\r', '\n');
        MFP_HDELIM(tmp);
#endif
        hdr_body.e = value.e;
        if (cnull(tmp)) break;
        uint32_t info = early_info;
        const int idx = NW ? early_idx : name_lookup(req, name, info);
        if (idx >= 0) {
#ifndef MFP_PROBE_LNOEMIT
            b.putc('(');
            if (info & 0xff) b.hex(hdr_body.d, clen(hdr_body)); else b.hex(name.d, clen(name));
            b.putc(')');
#endif
            if (req) {
                if ((info >> 8) == 1 && cnull(host)) host = value;
                if ((info >> 8) == 2 && cnull(ua)) ua = value;
            }
        }
    }
#undef MFP_HDELIM
#undef MFP_HTOP
}

// ---------------------------------------------------------------------------
// per-packet walk
// ---------------------------------------------------------------------------
struct Out {
    uint32_t fp_type, msg, flags;
    uint32_t xflags;     // MFP_XF_* (mfp_record.xflags)
    uint32_t sni_off, sni_len, ua_off, ua_len;
    uint32_t src_port, dst_port;
    uint32_t net;        // innermost IP header offset | version << 16 (flow key, flow_key.h:71)
    uint32_t pay_off, pay_len;   // QUIC: the UDP payload (k_quic takes it from here); TCP: the data
    // TCP reassembly inputs (tcp_packet tcpip.h:137-173): sequence number,
    // additional_bytes_needed of the message parsed from this segment, and
    // MFP_SEG_* kind bits (a data segment, supplementary, SSH-type reassembly)
    uint32_t seq, more, seg_kind;
};
// the certificate_list datum in the record's server-name slot (TLS server
// messages have no server name): the JSON writer's certs array (tls.h:2183)
DEV void cert_record(Out &o, Cur l, const uint8_t *base) {
    if (cnotempty(l)) { o.sni_off = (uint32_t)(l.d - base); o.sni_len = (uint32_t)clen(l); }
}
struct Cfg {
    uint32_t select, tls_format, mode;
    uint32_t classify;   // stop after protocol identification (o.msg), emit nothing
    uint32_t seg;        // the caller wants the reassembly inputs (KParams::seg)
    uint32_t block;      // BLK_*: selected protocols outside this path that are identified first
    uint32_t spread;     // k_fp_lds over a small batch: one packet per wave (lane 0), the packets'
                         // walks side by side on separate SIMDs instead of divergent lanes of one wave
};
// Protocols the selection may name ("all" names every one) that this path does
// not parse, but whose matchers or ports the reference consults before one of
// this path's (traffic_selector proto_identify.h:620-895; get_tcp_msg_type
// :936-942, get_udp_msg_type :944-968, the port tables :970-1075): a packet
// they claim writes no record here (MFP_MSG_OTHER), whatever this path would
// have made of it.  Mirrored in mfp_host.cpp (parse_select).
enum : uint32_t {
    BLK_SMTP = 1u << 0, BLK_DNS_TCP = 1u << 1, BLK_DNS_UDP = 1u << 2, BLK_SMB = 1u << 3, BLK_BT = 1u << 4,
    BLK_MYSQL = 1u << 5, BLK_SOCKS = 1u << 6, BLK_IEC = 1u << 7, BLK_DNP3 = 1u << 8, BLK_LDAP = 1u << 9,
    BLK_NBSS = 1u << 10, BLK_FTP_RESP = 1u << 11, BLK_TACACS = 1u << 12, BLK_RDP = 1u << 13, BLK_KRB5 = 1u << 14,
    BLK_REDIS_REQ = 1u << 15, BLK_REDIS_RESP = 1u << 16, BLK_IMAP_REQ = 1u << 17, BLK_IMAP_RESP = 1u << 18,
    BLK_TELNET = 1u << 19, BLK_IPSEC = 1u << 20, BLK_WIREGUARD = 1u << 21, BLK_SSDP = 1u << 22, BLK_NBDS = 1u << 23,
    BLK_TFTP = 1u << 24, BLK_SNMP = 1u << 25, BLK_SYSLOG = 1u << 26,
    BLK_TCP = BLK_SMTP | BLK_DNS_TCP | BLK_SMB | BLK_BT | BLK_MYSQL | BLK_SOCKS | BLK_IEC | BLK_DNP3 | BLK_LDAP |
              BLK_NBSS | BLK_FTP_RESP | BLK_TACACS | BLK_RDP | BLK_KRB5 | BLK_REDIS_REQ | BLK_REDIS_RESP |
              BLK_IMAP_REQ | BLK_IMAP_RESP | BLK_TELNET,
    BLK_UDP_PORTS = BLK_IPSEC | BLK_NBDS | BLK_TFTP | BLK_KRB5 | BLK_SNMP | BLK_SYSLOG,
    BLK_UDP = BLK_DNS_UDP | BLK_BT | BLK_WIREGUARD | BLK_SSDP | BLK_UDP_PORTS,
};
// parser families compiled into a walker instance (template argument FAM):
// a bin kernel carries only its protocol's parser, so its code and register
// footprint are the parser's, not the union of all of them; a packet whose
// message needs a family that is compiled out is punted (Em::punt /
// SegEm::ovf) to the fallback lane, which carries every family
enum : uint32_t {
    FAM_TLS = 1, FAM_SSH = 2, FAM_HTTP = 4, FAM_TCP = 8, FAM_DTLS = 16, FAM_STUN = 32,
    FAM_ALL = 63,
};
enum : uint32_t {
    SEL_TLS_CH = 1u << 0, SEL_TLS_SH = 1u << 1, SEL_TLS_CERT = 1u << 2, SEL_SSH_CLIENT = 1u << 3,
    SEL_SSH_SERVER = 1u << 4, SEL_HTTP_REQ = 1u << 5, SEL_HTTP_RESP = 1u << 6, SEL_TCP_SYN = 1u << 7,
    SEL_TCP_SYNACK = 1u << 8, SEL_DTLS = 1u << 9, SEL_QUIC = 1u << 10,
    SEL_GRE = 1u << 11, SEL_VXLAN = 1u << 12, SEL_GENEVE = 1u << 13,   // decapsulations (proto_identify.h:812-886)
    SEL_STUN = 1u << 14, SEL_OPENVPN = 1u << 15,                       // "stun", "openvpn_tcp" (proto_identify.h:834,868)
};

// masked 8/16-byte matchers (match.h:64-103)
DEV bool m8(Cur p, uint64_t mask, uint64_t val) {
    if (!p.d || clen(p) < 8) return false;
    uint64_t w = 0;
    for (int i = 0; i < 8; i++) w |= (uint64_t)ld(p.d + i) << (8 * i);
    return (w & mask) == val;
}
#define LE8(a, b, c, d, e, f, g, h)                                                                    \
    ((uint64_t)(a) | ((uint64_t)(b) << 8) | ((uint64_t)(c) << 16) | ((uint64_t)(d) << 24) |           \
     ((uint64_t)(e) << 32) | ((uint64_t)(f) << 40) | ((uint64_t)(g) << 48) | ((uint64_t)(h) << 56))

// HTTP request keywords that map to http_request (proto_identify.h:200-236)
__constant__ uint32_t k_http_kw[] = {
    0x41434c20, 0x42415345, 0x42494e44, 0x43484543, 0x434f4e4e, 0x434f5059, 0x44454c45, 0x47455420,
    0x48454144, 0x4c414245, 0x4c494e4b, 0x4c4f434b, 0x4d455247, 0x4d4b4143, 0x4d4b4341, 0x4d4b434f,
    0x4d4b5245, 0x4d4b574f, 0x4d4f5645, 0x4f505449, 0x4f524445, 0x50415443, 0x504f5354, 0x50524920,
    0x50524f50, 0x50555420, 0x52454249, 0x5245504f, 0x53454152, 0x54524143, 0x554e4249, 0x554e4348,
    0x554e4c49, 0x554e4c4f, 0x55504441, 0x56455253,
};

template <class E>
DEV void fp_type_prefix(E &b, uint32_t t) {             // fingerprint::set_type fingerprint.h:44
    switch (t) {
    case 1: b.lit("tls/"); break;
    case 2: b.lit("tls_server/"); break;
    case 3: b.lit("http/"); break;
    case 4: b.lit("http_server/"); break;
    case 5: b.lit("ssh/"); break;
    case 6: b.lit("ssh_kex/"); break;
    case 7: b.lit("tcp/"); break;
    case 10: b.lit("dtls/"); break;
    case 11: b.lit("dtls_server/"); break;
    case 12: b.lit("quic/"); break;
    case 13: b.lit("tcp_server/"); break;
    case 14: b.lit("openvpn/"); break;
    case 16: b.lit("stun/"); break;
    case 17: b.lit("ssh_init/"); break;
    case 18: b.lit("ssh_server/"); break;
    case 19: b.lit("ssh_kex_server/"); break;
    case 20: b.lit("ssh_init_server/"); break;
    }
    b.last_putc = true;   // set_type ends with write_char('/')
}

// HTTP request/response parse + fingerprint (http.cc:105-128, 369-383,
// 426-553); returns false when the message is empty (no record)
template <class E>
DEV bool http_msg(E &b, Cur p, bool req, Out &o, const uint8_t *base) {
    Cur f1, f2, f3;   // req: method, protocol ; resp: version, status, reason
    cset_null(f1); cset_null(f2); cset_null(f3);
    // (MFP_HTTP_WIN, segment walker) the line's searches share their loaded words
    constexpr bool LW = E::SEG && MFP_HTTP_WIN && MFP_HTTP_FAST < 3;
    SWin W;
    if (req) {
        Cur uri;
        if (LW) cparse_to_delim_w(f1, p, ' ', W);
        else cparse_to_delim(f1, p, ' ');
        long ml = clen(f1);
        if (ml < 3 || ml > 16) return false;
#if MFP_HTTP_FAST >= 3
        // the method's bytes (<= 16) loaded with the URI search, "HTTP/" with
        // the search for the line's end: one memory round trip each
        const uint64_t m0 = ld_le8n(f1.d, ml < 8 ? ml : 8);
        const uint64_t m1 = ml > 8 ? ld_le8n(f1.d + 8, ml - 8) : 0ull;
        cskip(p, 1);
        cparse_to_delim(uri, p, ' ');
        {   // every byte of the method 'A'..'Z'
            const uint64_t k0 = ml >= 8 ? 0x8080808080808080ull : 0x8080808080808080ull & ((1ull << (8 * ml)) - 1);
            const long r1 = ml - 8;
            const uint64_t k1 = r1 <= 0 ? 0ull : r1 >= 8 ? 0x8080808080808080ull : 0x8080808080808080ull & ((1ull << (8 * r1)) - 1);
            if ((swar_upper(m0) & k0) != k0 || (swar_upper(m1) & k1) != k1) return false;
        }
        cskip(p, 1);
        const long pl = clen(p);
        const uint64_t h5 = p.d && pl > 0 ? ld_le8n(p.d, pl < 5 ? pl : 5) : 0ull;
        cparse_to_delims(f2, p, '\r', '\n');
        if (!(f2.d && clen(f2) >= 5 && h5 == 0x2f50545448ull)) return false;   // "HTTP/"
#else
        if constexpr (LW) {
            if (swar_find_w(f1.d, f1.e, [](uint64_t w) { return ~swar_upper(w) & 0x8080808080808080ull; }, W) < f1.e)
                return false;
            cskip(p, 1);
            cparse_to_delim_w(uri, p, ' ', W);
            cskip(p, 1);
            cparse_to_delims_w(f2, p, '\r', '\n', W);
            if (!(f2.d && clen(f2) >= 5)) return false;
            const uintptr_t fa = (uintptr_t)f2.d;
            const uint64_t h5 = W.a && fa >= W.a && fa + 8 <= W.a + 8 * MFP_SWB ? win_get8(W.w, W.a, fa)
                                                                               : ld_le8n(f2.d, 5);
            if ((h5 & 0xffffffffffull) != 0x2f50545448ull) return false;   // "HTTP/" (f2 holds 5 bytes)
        } else {
        if (swar_find(f1.d, f1.e, [](uint64_t w) { return ~swar_upper(w) & 0x8080808080808080ull; }) < f1.e) return false;
        cskip(p, 1);
        cparse_to_delim(uri, p, ' ');
        cskip(p, 1);
        cparse_to_delims(f2, p, '\r', '\n');
        if (!(f2.d && clen(f2) >= 5 && ld(f2.d) == 'H' && ld(f2.d + 1) == 'T' && ld(f2.d + 2) == 'T' &&
              ld(f2.d + 3) == 'P' && ld(f2.d + 4) == '/'))
            return false;
        }
#endif
    } else if constexpr (LW) {
        cparse_to_delim_w(f1, p, ' ', W);
        cskip(p, 1);
        cparse_to_delim_w(f2, p, ' ', W);
        cskip(p, 1);
        cparse_to_delims_w(f3, p, '\r', '\n', W);
        if (!cnotempty(f2)) return false;
    } else {
        cparse_to_delim(f1, p, ' ');
        cskip(p, 1);
        cparse_to_delim(f2, p, ' ');
        cskip(p, 1);
        cparse_to_delims(f3, p, '\r', '\n');
        if (!cnotempty(f2)) return false;
    }
    Cur delim; delim.d = p.d;
    if (p.d) p.d = LW ? swar_find_w(p.d, p.e, [](uint64_t w) { return swar_alpha(w); }, W)
                      : swar_find(p.d, p.e, [](uint64_t w) { return swar_alpha(w); });
    delim.e = p.d;
    fp_type_prefix(b, req ? 3 : 4);
    b.putc('('); b.hex(f1.d, clen(f1)); b.putc(')');
    b.putc('('); b.hex(f2.d, clen(f2)); b.putc(')');
    if (!req) { b.putc('('); b.hex(f3.d, clen(f3)); b.putc(')'); }
    b.putc('(');
    Cur host, ua; cset_null(host); cset_null(ua);
    http_headers_fp(b, p, delim, req, host, ua);
    b.putc(')');
    if (req) {
        if (!cnull(host)) { o.sni_off = (uint32_t)(host.d - base); o.sni_len = (uint32_t)clen(host); }
        if (!cnull(ua)) { o.ua_off = (uint32_t)(ua.d - base); o.ua_len = (uint32_t)clen(ua); }
    }
    return true;
}

// the TCP matchers of selected protocols outside this path, consulted only
// when this path's matchers found nothing (they come after them in the tcp
// table; the 4-byte ones, with their length checks, are the tcp4 table that
// follows it): smtp_server "250-" (smtp.h:282), dns_packet::tcp_matcher
// (dns.h:1152), smb1 / smb2 (smb1.h:311, smb2.h:856), bittorrent_handshake
// (bittorrent.h:422), mysql_server_greet at offset 3 (mysql.hpp:577; the
// reference's bound check, (length + offset) < 8, lets it read past a short
// payload: read here as zero bytes), iec60870_5_104 (iec60870_5_104.h:538-549),
// dnp3 (dnp3.h:501-512), socks4_req / socks5_hello / socks5_req_resp
// (socks.h:90-110, 219-229, 490-505)
DEV bool tcp_other_matcher(Cur p, uint32_t blk) {
    const long n = clen(p);
    if (!p.d || n < 4) return false;                                  // protocol_identifier::get_msg_type
    if (n >= 8) {
        if ((blk & BLK_SMTP) && m8(p, LE8(0xff, 0xff, 0xff, 0xff, 0, 0, 0, 0), LE8('2', '5', '0', '-', 0, 0, 0, 0)))
            return true;
        if ((blk & BLK_DNS_TCP) && m8(p, LE8(0, 0, 0, 0, 0x10, 0x48, 0xff, 0), 0)) return true;
        if ((blk & BLK_SMB) && (m8(p, LE8(0, 0, 0, 0, 0xff, 0xff, 0xff, 0xff), LE8(0, 0, 0, 0, 0xff, 'S', 'M', 'B')) ||
                                m8(p, LE8(0, 0, 0, 0, 0xff, 0xff, 0xff, 0xff), LE8(0, 0, 0, 0, 0xfe, 'S', 'M', 'B'))))
            return true;
        if ((blk & BLK_BT) && m8(p, ~0ull, LE8(0x13, 'B', 'i', 't', 'T', 'o', 'r', 'r'))) return true;
    }
    if (blk & BLK_MYSQL) {
        uint64_t w = 0;
        for (int i = 0; i < 8; i++) w |= (uint64_t)(3 + i < n ? ld(p.d + 3 + i) : 0u) << (8 * i);
        if ((w & LE8(0xf8, 0xff, 0xf0, 0xff, 0xf0, 0xe0, 0xe0, 0)) == LE8(0, 0x0a, 0x30, 0x2e, 0x30, 0x20, 0x20, 0))
            return true;
    }
    const uint32_t b0 = ld(p.d), b1 = ld(p.d + 1), b2 = ld(p.d + 2), b3 = ld(p.d + 3);
    if ((blk & BLK_IEC) && b0 == 0x68 && (long)(b1 + 2) == n) return true;
    if ((blk & BLK_DNP3) && b0 == 0x05 && b1 == 0x64 &&
        (long)(3 + b2 + 2 + (b2 % 16 ? b2 / 16 + 1 : b2 / 16) * 2) == n)
        return true;
    if (blk & BLK_SOCKS) {
        if (b0 == 0x04 && (b1 & 0xfc) == 0 && n > 8) {
            const uint32_t f = ld(p.d + 8);
            if ((n == 9 && f == 0) || ((f >= 32 || f == 0) && ld(p.e - 2) >= 32 && ld(p.e - 1) == 0)) return true;
        }
        if (b0 == 0x05 && (b1 & 0xf0) == 0 && (long)(2 + b1) == n) return true;
        if (b0 == 0x05 && (b1 & 0xf0) == 0 && b2 == 0 && (b3 & 0xf8) == 0) {
            const long dom = n > 4 ? (long)ld(p.d + 4) : 0;
            if (n == 10 || n == 22 || n == 7 + dom) return true;
        }
    }
    return false;
}
// get_tcp_msg_type_from_ports (proto_identify.h:1015-1075): the ports checked
// before OpenVPN's 1194 (ldap, nbss) and after it (the rest), all before the
// keyword matchers that find HTTP
DEV bool tcp_other_port_first(uint32_t sp, uint32_t dp, uint32_t blk) {
    return ((blk & BLK_LDAP) && (sp == 389 || dp == 389)) || ((blk & BLK_NBSS) && (sp == 139 || dp == 139));
}
DEV bool tcp_other_port(uint32_t sp, uint32_t dp, uint32_t blk) {
    return ((blk & BLK_FTP_RESP) && sp == 21) || ((blk & BLK_TACACS) && (sp == 49 || dp == 49)) ||
           ((blk & BLK_RDP) && (sp == 3389 || dp == 3389)) || ((blk & BLK_MYSQL) && (sp == 3306 || dp == 3306)) ||
           ((blk & BLK_KRB5) && (sp == 88 || dp == 88)) || ((blk & BLK_REDIS_REQ) && dp == 6379) ||
           ((blk & BLK_REDIS_RESP) && sp == 6379) || ((blk & BLK_IMAP_REQ) && dp == 143) ||
           ((blk & BLK_IMAP_RESP) && sp == 143) || ((blk & BLK_TELNET) && (sp == 23 || dp == 23));
}
// the UDP matchers of the udp table that precede QUIC's (and so every 16- and
// 4-byte matcher): dns_packet::matcher (dns.h:1141; also for nbns / mdns),
// wireguard (wireguard.h:52), ssdp (ssdp.h:153), bittorrent DHT and LSD
// (bittorrent.h:66, 257); ESP/IKE on port 4500 before any of them (:946-953)
DEV bool udp_other_first(Cur p, uint32_t sp, uint32_t dp, uint32_t blk) {
    if ((blk & BLK_IPSEC) && (sp == 4500 || dp == 4500)) return true;
    if (!p.d || clen(p) < 8) return false;
    return ((blk & BLK_DNS_UDP) && m8(p, LE8(0, 0, 0x10, 0x48, 0xff, 0, 0xff, 0x80), 0)) ||
           ((blk & BLK_WIREGUARD) && m8(p, LE8(0xff, 0xff, 0xff, 0xff, 0, 0, 0, 0), LE8(1, 0, 0, 0, 0, 0, 0, 0))) ||
           ((blk & BLK_SSDP) && m8(p, LE8(0xe8, 0x84, 0xf0, 0xe0, 0, 0x90, 0, 0), LE8(0x48, 0x04, 0x50, 0x40, 0, 0x10, 0, 0))) ||
           ((blk & BLK_BT) && (m8(p, LE8(0xff, 0xff, 0xff, 0x8c, 0xff, 0xff, 0xff, 0xff), LE8('d', '1', ':', 0, 'd', '2', ':', 'i')) ||
                               m8(p, ~0ull, LE8('B', 'T', '-', 'S', 'E', 'A', 'R', 'C'))));
}
// get_udp_msg_type_from_ports (proto_identify.h:970-1013): the ports checked
// before VXLAN / Geneve / GRE over UDP (the encapsulation walk uses the same
// table, pkt_proc.cc:1000-1018)
DEV bool udp_other_port(uint32_t sp, uint32_t dp, uint32_t blk) {
    return ((blk & BLK_IPSEC) && (sp == 500 || dp == 500)) || ((blk & BLK_NBDS) && sp == 138 && dp == 138) ||
           ((blk & BLK_TFTP) && (sp == 69 || dp == 69)) || ((blk & BLK_KRB5) && (sp == 88 || dp == 88)) ||
           ((blk & BLK_SNMP) && (sp == 161 || sp == 162 || dp == 161 || dp == 162)) || ((blk & BLK_SYSLOG) && dp == 514);
}

// set_tcp_protocol pkt_proc.cc:488 (selection subset)
template <uint32_t FAM, class E>
DEV void tcp_data(E &b, const Cfg &cfg, Out &o, Cur pkt, const uint8_t *tcph, const uint8_t *base) {
    uint32_t sel = cfg.select;
    uint32_t sport = (ld(tcph) << 8) | ld(tcph + 1), dport = (ld(tcph + 2) << 8) | ld(tcph + 3);
    uint32_t msg = 0;
    if (clen(pkt) >= 4) {
        const uint64_t MT = LE8(0xff, 0xff, 0xfc, 0, 0, 0xff, 0, 0);
        if ((sel & SEL_TLS_CH) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x01, 0, 0))) msg = MFP_MSG_TLS_CH;
        else if ((sel & SEL_TLS_SH) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x02, 0, 0))) msg = MFP_MSG_TLS_SH;
        else if ((sel & SEL_TLS_CERT) && m8(pkt, MT, LE8(0x16, 0x03, 0, 0, 0, 0x0b, 0, 0))) msg = MFP_MSG_TLS_CERT;
        else if ((sel & (SEL_SSH_CLIENT | SEL_SSH_SERVER)) &&
                 m8(pkt, LE8(0xff, 0xff, 0xff, 0xff, 0, 0, 0, 0), LE8('S', 'S', 'H', '-', 0, 0, 0, 0)))
            msg = MFP_MSG_SSH_INIT;
        else if ((sel & (SEL_SSH_CLIENT | SEL_SSH_SERVER)) &&
                 m8(pkt, LE8(0xff, 0xff, 0xf0, 0, 0, 0xff, 0, 0), LE8(0, 0, 0, 0, 0, 0x14, 0, 0)))
            msg = MFP_MSG_SSH_KEX;
    }
    // a selected protocol outside this path claims the payload first: the
    // walkers that parse HTTP decide it (they carry the checks), the others
    // hand the packet to the fallback lane, which does
    const bool blk = msg == 0 && (cfg.block & BLK_TCP) && !cfg.classify;
    if (blk) {
        if constexpr (!(FAM & FAM_HTTP)) {
            b.punt_pkt();
            return;
        } else if (tcp_other_matcher(pkt, cfg.block) || tcp_other_port_first(sport, dport, cfg.block)) {
            o.msg = MFP_MSG_OTHER;
            return;
        }
    }
    // tcp_msg_type_from_ports (proto_identify.h:1028-1030): OpenVPN over TCP
    // on port 1194, before the keyword matchers.  k_quic parses it (the
    // ClientHello may span several control records, openvpn.h:388-403).
    if (msg == 0 && (sel & SEL_OPENVPN) && (sport == 1194 || dport == 1194)) {
        o.msg = MFP_MSG_OPENVPN;
        o.pay_off = (uint32_t)(pkt.d - base);
        o.pay_len = (uint32_t)clen(pkt);
        if (!cfg.classify) b.punt_pkt();
        return;
    }
    if (blk && tcp_other_port(sport, dport, cfg.block)) {
        o.msg = MFP_MSG_OTHER;
        return;
    }
    if (msg == 0) {
        if (clen(pkt) < 4) return;
        uint32_t kw = (ld(pkt.d) << 24) | (ld(pkt.d + 1) << 16) | (ld(pkt.d + 2) << 8) | ld(pkt.d + 3);
        if (sel & SEL_HTTP_REQ) {
            bool hit = false;
            for (int i = 0; i < 36; i++) hit |= (k_http_kw[i] == kw);
            if (hit) {
                o.msg = MFP_MSG_HTTP_REQ;
                if (cfg.classify) return;
                if constexpr (!(FAM & FAM_HTTP)) { b.punt_pkt(); return; }
                else {
                    if (http_msg(b, pkt, true, o, base)) { o.flags |= MFP_FLAG_EMIT; o.fp_type = 3; }
                    else o.msg = 0;
                }
                return;
            }
        }
        if ((sel & SEL_HTTP_RESP) && kw == 0x48545450u) {
            o.msg = MFP_MSG_HTTP_RESP;
            if (cfg.classify) return;
            if constexpr (!(FAM & FAM_HTTP)) { b.punt_pkt(); return; }
            else {
                if (http_msg(b, pkt, false, o, base)) { o.flags |= MFP_FLAG_EMIT; o.fp_type = 4; }
                else o.msg = 0;
            }
        }
        return;
    }
    o.msg = msg;
    if (cfg.classify) return;
    const bool tls_msg = msg == MFP_MSG_TLS_CH || msg == MFP_MSG_TLS_SH || msg == MFP_MSG_TLS_CERT;
    if ((E::SEG && (FAM & FAM_TLS)) || (tls_msg && !(FAM & FAM_TLS)) || (!tls_msg && !(FAM & FAM_SSH))) {
        b.punt_pkt();          // a parser this walker lacks: the fallback lane fingerprints it
        return;
    }
    if constexpr (!E::SEG || !(FAM & FAM_TLS)) {
    switch (msg) {
    case MFP_MSG_TLS_CH: {
        if constexpr (!(FAM & FAM_TLS)) return; else {
        Cur p = pkt;
        Cur frag = tls_record_fragment(p);
        Hs hs = tls_hs_parse(frag);
        if (hs.more) o.flags |= MFP_FLAG_TRUNCATED;
        o.more = (uint32_t)hs.more;                    // pkt_proc.cc:527-531
        Ch ch = tls_ch_parse(hs.body);
        if (!cnotempty(ch.compression)) return;
        o.flags |= MFP_FLAG_EMIT; o.fp_type = 1;
        if (clen(ch.ciphers) <= 0) o.flags |= MFP_FLAG_NO_CIPHERS;   // no "tls" object (tls.h:1882-1885)
        if constexpr (E::PLAN) {
#ifdef MFP_PROBE_NOPLAN   // (profiling probe only: the walk up to the ClientHello; everything punted)
            if constexpr (E::FAST >= 0) { o.fp_type = 0; return; }
#endif
            if constexpr (E::FAST >= 0)
                tls_ch_plan_fast<E::FAST>(b, *b.plan, ch, 1, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len);
            else
                tls_ch_plan(b, *b.plan, ch, (int)cfg.tls_format, 1, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len, o.xflags);
        } else {
            fp_type_prefix(b, 1);
            tls_ch_fp(b, ch, (int)cfg.tls_format);
            if (!E::emit_pass() || b.spans) tls_sni(ch.extensions, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len, o.xflags);
        }
        return;
        }
    }
    case MFP_MSG_TLS_SH: {                              // tls.h:573
        if constexpr (!(FAM & FAM_TLS)) return; else {
        Cur p = pkt;
        Sh sh; cset_null(sh.version); cset_null(sh.cipher); cset_null(sh.extensions);
        Cert cert; cset_null(cert.list); cert.more = 0;
        Cur frag = tls_record_fragment(p);
        Hs hs = tls_hs_parse(frag);
        if (hs.msg_type == 2) {
            sh = tls_sh_parse(hs.body);
            if (cnotempty(frag)) { Hs h2 = tls_hs_parse(frag); tls_cert_parse(cert, h2.body); }
        } else if (hs.msg_type == 11) {
            tls_cert_parse(cert, hs.body);
        }
        Cur frag2 = tls_record_fragment(p);
        Hs hs2 = tls_hs_parse(frag2);
        if (hs2.msg_type == 11) tls_cert_parse(cert, hs2.body);
        cert_record(o, cert.list, base);            // tls.h:605-627 (the JSON writer's certs)
        if (cert.more) o.flags |= MFP_FLAG_TRUNCATED;
        o.more = (uint32_t)cert.more;                  // tls.h:596-598
        bool hello = tls_sh_not_empty(sh);
        if (hello || cnotempty(cert.list)) o.flags |= MFP_FLAG_EMIT;
        if (hello) { o.fp_type = 2; fp_type_prefix(b, 2); tls_sh_fp(b, sh); }
        return;
        }
    }
    case MFP_MSG_TLS_CERT: {                            // tls.h:720
        if constexpr (!(FAM & FAM_TLS)) return; else {
        Cur p = pkt;
        Cert cert; cset_null(cert.list); cert.more = 0;
        Cur frag = tls_record_fragment(p);
        Hs hs = tls_hs_parse(frag);
        if (hs.msg_type == 11) {
            tls_cert_parse(cert, hs.body);
            uint32_t t = 0;                              // entity, tls.h:728-744
            if (cnotempty(frag)) { Hs h = tls_hs_parse(frag); t = h.msg_type; }
            else if (cnotempty(p)) { Cur f2 = tls_record_fragment(p); Hs h = tls_hs_parse(f2); t = h.msg_type; }
            if (t == 16) o.flags |= MFP_FLAG_CERT_CLIENT; else if (t == 12) o.flags |= MFP_FLAG_CERT_SERVER;
        }
        cert_record(o, cert.list, base);
        if (cert.more) o.flags |= MFP_FLAG_TRUNCATED;
        o.more = (uint32_t)cert.more;                  // tls.h:735-737
        if (cnotempty(cert.list)) o.flags |= MFP_FLAG_EMIT;
        return;
        }
    }
    case MFP_MSG_SSH_INIT: {                            // ssh.h:342-430
        if constexpr (!(FAM & FAM_SSH)) return; else {
        bool server = !(dport <= sport);
        if (!(sel & (server ? SEL_SSH_SERVER : SEL_SSH_CLIENT))) { o.msg = 0; return; }
        Cur p = pkt, proto, comment; cset_null(comment);
        uint32_t delim = cparse_to_delims(proto, p, '\n', ' ');
        if (delim != '\n') { cskip(p, 1); cparse_to_delim(comment, p, '\n'); }
        cskip(p, 1);
        bool kex = false;
        SshBin bin; cset_null(bin.payload); bin.more = 0;
        SshKex kx;
        kx.ok = false;
        if (cnotempty(p)) {
            bin = ssh_bin_parse(p);
            if (cnotempty(bin.payload)) { kx = ssh_kex_parse(bin.payload); kex = kx.ok; }
        }
        uint64_t more = kex ? bin.more : 8192;
        if (more) o.flags |= MFP_FLAG_TRUNCATED;
        if (more) { o.more = (uint32_t)more; o.seg_kind |= MFP_SEG_SSH; }   // pkt_proc.cc:550-553
        if (!cnotempty(proto)) return;
        o.flags |= MFP_FLAG_EMIT;
        if (kex) {
            o.fp_type = server ? 18 : 5;
            fp_type_prefix(b, o.fp_type);
            ssh_kex_fp(b, bin.payload, kx);
        } else {
            o.fp_type = server ? 20 : 17;
            fp_type_prefix(b, o.fp_type);
            b.putc('(');
            if (cnotempty(comment)) {
                b.hex(proto.d, clen(proto));
                b.putc('2'); b.putc('0');
                Cur t = comment; t.e -= 1; if (t.e < t.d) t.e = t.d;
                b.hex(t.d, clen(t));
            } else {
                Cur t = proto; t.e -= 1; if (t.e < t.d) t.e = t.d;
                b.hex(t.d, clen(t));
            }
            b.putc(')');
        }
        // analysis: user agent = protocol + comment strings (do_analysis
        // ssh.h:480-487: a data_buffer<512> that a null comment nulls).  The
        // span runs from the protocol string to the comment's end; its first
        // space is the delimiter, which the classifier drops (k_analyze_wave).
        if (!cnull(comment)) { o.ua_off = (uint32_t)(proto.d - base); o.ua_len = (uint32_t)(comment.e - proto.d); }
        return;
        }
    }
    case MFP_MSG_SSH_KEX: {                             // pkt_proc.cc:586-601
        if constexpr (!(FAM & FAM_SSH)) return; else {
        bool server = !(dport <= sport);
        if (!(sel & (server ? SEL_SSH_SERVER : SEL_SSH_CLIENT))) { o.msg = 0; return; }
        Cur p = pkt;
        SshBin bin = ssh_bin_parse(p);
        if (bin.more) o.flags |= MFP_FLAG_TRUNCATED;
        if (bin.more) o.more = (uint32_t)bin.more;     // pkt_proc.cc:563-569
        else o.seg_kind |= MFP_SEG_SUPPLEMENTARY;
        const SshKex kx = ssh_kex_parse(bin.payload);
        if (!kx.ok) return;
        o.flags |= MFP_FLAG_EMIT;
        o.fp_type = server ? 19 : 6;
        fp_type_prefix(b, o.fp_type);
        ssh_kex_fp(b, bin.payload, kx);
        return;
        }
    }
    }
    }
}

// STUN attribute (stun::attribute stun.h:323-338): type, length, value and
// padding to a 4-byte boundary; false (cursor null) when any part is missing
DEV bool stun_attr(Cur &d, uint32_t &type, Cur &value) {
    uint64_t t, l;
    rd_uint(d, 2, t);
    rd_uint(d, 2, l);
    cparse(value, d, cnull(d) ? 0 : (long)l);
    const long pad = (4 - (long)(l & 3)) & 3;             // pad_len datum.h:2344
    if (!cnull(d)) { if (clen(d) < pad) cset_null(d); else d.d += pad; }
    type = (uint32_t)t;
    return !cnull(d);
}

// STUN message (stun::message stun.h:783-1013), reached through udp4's
// length matcher: the header's length field + 20 equals the UDP payload
// length (protocol_identifier<4>, proto_identify.h:387-390).  The record
// exists when is_not_empty() holds (stun.h:902-916); responses set the
// fingerprint buffer's truncated bit, so they carry no fingerprint
// (stun.h:932-941).  The record's server-name span holds the message (for the
// JSON writer's "stun" object), its user-agent span the last SOFTWARE value
// (do_analysis stun.h:1021-1036).
template <uint32_t FAM, class E>
DEV void stun_msg(E &b, const Cfg &cfg, Out &o, Cur pkt, const uint8_t *base) {
    o.msg = MFP_MSG_STUN;
    if (cfg.classify) return;
    if constexpr (E::SEG || !(FAM & FAM_STUN)) {
        b.punt_pkt();
        return;
    } else {
    const uint8_t *h = pkt.d;
    const uint32_t mtf = (ld(h) << 8) | ld(h + 1);
    const bool cookie = ld(h + 4) == 0x21 && ld(h + 5) == 0x12 && ld(h + 6) == 0xa4 && ld(h + 7) == 0x42;
    Cur body = cmk(h + 20, pkt.e);
    bool present = cookie;
    if (!present) {
        const bool classic = mtf == 0x0001 || mtf == 0x0101 || mtf == 0x0111 || mtf == 0x0002 || mtf == 0x0102 ||
                             mtf == 0x0112;                          // message_type_is_valid_for_classic_stun
        if (classic) {
            if (clen(body) == 0) {
                uint32_t z = 0;
                for (int k = 4; k < 20; k++) z += ld(h + k) == 0;     // tid_zero_count
                present = z < 2;
            } else {
                Cur t = body, v; uint32_t ty;
                present = stun_attr(t, ty, v);                    // lookahead<stun::attribute>
            }
        }
    }
    if (!present) return;
    o.flags |= MFP_FLAG_EMIT;
    o.sni_off = (uint32_t)(h - base); o.sni_len = (uint32_t)clen(pkt);
    // SOFTWARE (the last one) for the classifier, recorded while fingerprinting
    Cur sw; cset_null(sw);
    if (mtf & 0x100) {                                          // is_response(): no fingerprint
        Cur t = body, v; uint32_t ty;
        while (clen(t) > 0 && stun_attr(t, ty, v)) if (ty == 0x8022) sw = v;
    } else {
        o.fp_type = 16;
        fp_type_prefix(b, 16);
        b.putc('1'); b.putc('/');                               // set_type(stun, 1) fingerprint.h:48-51
        const uint32_t cls = ((mtf & 0x100) >> 7) | ((mtf & 0x10) >> 4);
        const uint32_t method = (mtf & 0x0f) | ((mtf & 0xe0) >> 1) | ((mtf & 0x3e00) >> 2);
        b.putc('('); b.hex8(cls); b.putc(')');
        b.putc('('); b.hex16(method); b.putc(')');
        b.putc('('); b.hex8(cookie ? 1u : 0u); b.putc(')');
        b.putc('(');
        Cur t = body, v; uint32_t ty;
        while (clen(t) > 0 && stun_attr(t, ty, v)) {
            // attr_fp_type (stun.h:957-970): type only, or type + length + value
            const bool tlv = ty == 0x8037 || ty == 0x8070;
            const bool only = ty == 0x0006 || ty == 0x0008 || ty == 0x0020 || ty == 0x8007 || ty == 0x8008 ||
                              ty == 0x8022 || ty == 0x8028 || ty == 0xc003 || ty == 0xc057 || ty == 0xdaba;
            if (tlv || only) {
                b.putc('(');
                b.hex16(ty);
                if (tlv) { b.hex16((uint32_t)clen(v)); b.hex(v.d, clen(v)); }
                b.putc(')');
            }
            if (ty == 0x8022) sw = v;
        }
        b.putc(')');
    }
    if (!cnull(sw)) { o.ua_off = (uint32_t)(sw.d - base); o.ua_len = (uint32_t)clen(sw); }
    }
}

// set_udp_protocol pkt_proc.cc:677 (selection subset: QUIC, DTLS, STUN)
template <uint32_t FAM, class E>
DEV void udp_data(E &b, const Cfg &cfg, Out &o, Cur pkt, const uint8_t *base) {
    // a selected protocol outside this path claims the datagram first: only
    // the fallback lane (every family) carries the checks
    if ((cfg.block & BLK_UDP) && !cfg.classify) {
        if constexpr (FAM != FAM_ALL) {
            b.punt_pkt();
            return;
        } else {
            if (udp_other_first(pkt, o.src_port, o.dst_port, cfg.block)) { o.msg = MFP_MSG_OTHER; return; }
        }
    }
    // 8-byte matchers before 16-byte ones (get_udp_msg_type proto_identify.h:955-960):
    // the QUIC long header (quic_initial_packet::matcher quic.h:544).  Only
    // k_quic (mfp_quic.hip) parses QUIC; every other walker hands it over.
    if ((cfg.select & SEL_QUIC) && clen(pkt) >= 8 && (ld(pkt.d) & 0x80) && !(ld(pkt.d + 5) & 0xe0)) {
        o.msg = MFP_MSG_QUIC;
        o.pay_off = (uint32_t)(pkt.d - base);
        o.pay_len = (uint32_t)clen(pkt);
        if (!cfg.classify) b.punt_pkt();
        return;
    }
    if (clen(pkt) < 16) return;
    uint32_t msg = 0;
    if (cfg.select & SEL_DTLS) {                       // udp16 matchers
        uint64_t w0 = 0, w1 = 0;
        for (int i = 0; i < 8; i++) { w0 |= (uint64_t)ld(pkt.d + i) << (8 * i); w1 |= (uint64_t)ld(pkt.d + 8 + i) << (8 * i); }
        const uint64_t M0 = LE8(0xff, 0xff, 0xfd, 0, 0, 0, 0, 0), V0 = LE8(0x16, 0xfe, 0xfd, 0, 0, 0, 0, 0);
        const uint64_t M1 = LE8(0, 0, 0, 0, 0, 0xff, 0, 0);
        if ((w0 & M0) == V0) {
            uint32_t hb = (uint32_t)((w1 & M1) >> 40);
            msg = hb == 1 ? MFP_MSG_DTLS_CH : hb == 2 ? MFP_MSG_DTLS_SH : hb == 3 ? MFP_MSG_DTLS_HVR : 0;
        }
    }
    if (!msg) {                                        // udp4: STUN's length matcher
        if ((cfg.select & SEL_STUN) && 20 + ((ld(pkt.d + 2) << 8) | ld(pkt.d + 3)) == (uint32_t)clen(pkt))
            stun_msg<FAM>(b, cfg, o, pkt, base);
        else if ((cfg.block & BLK_UDP_PORTS) && !cfg.classify && udp_other_port(o.src_port, o.dst_port, cfg.block))
            o.msg = MFP_MSG_OTHER;
        return;
    }
    o.msg = msg;
    if (cfg.classify) return;
    if constexpr (E::SEG || !(FAM & FAM_DTLS)) {
        b.punt_pkt();
        return;
    } else {
    Cur d = pkt, frag, body; cset_null(frag); cset_null(body);
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
    if (msg == MFP_MSG_DTLS_CH && cfg.seg && cnotempty(body)) {
        // offset-reassembly inputs of the fragment (dtls_client_hello
        // dtls.h:155-175, process_udp_offset_reassembly reassembly.hpp:1036)
        o.seg_kind |= MFP_SEG_DTLS;
        o.seq = (uint32_t)foff; o.more = (uint32_t)more;
        o.pay_off = (uint32_t)(body.d - base); o.pay_len = (uint32_t)clen(body);
    }
    if (msg == MFP_MSG_DTLS_CH) {
        if ((uint32_t)more) o.flags |= MFP_FLAG_TRUNCATED;
        Ch ch = tls_ch_parse(body);
        if (!cnotempty(ch.compression)) return;
        o.flags |= MFP_FLAG_EMIT; o.fp_type = 10;
        if (clen(ch.ciphers) <= 0) o.flags |= MFP_FLAG_NO_CIPHERS;   // no "dtls" object (tls.h:1882-1885)
        if constexpr (E::PLAN) {
            if constexpr (E::FAST >= 0)
                tls_ch_plan_fast<E::FAST>(b, *b.plan, ch, 10, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len);
            else
                tls_ch_plan(b, *b.plan, ch, (int)cfg.tls_format, 10, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len, o.xflags);
        } else {
            fp_type_prefix(b, 10);
            tls_ch_fp(b, ch, (int)cfg.tls_format);
            if (!E::emit_pass() || b.spans) tls_sni(ch.extensions, base, o.sni_off, o.sni_len, o.ua_off, o.ua_len, o.xflags);
        }
    } else if (msg == MFP_MSG_DTLS_SH) {
        Cur b2 = body;
        Sh sh = tls_sh_parse(b2);
        if (!tls_sh_not_empty(sh)) return;
        o.flags |= MFP_FLAG_EMIT; o.fp_type = 11;
        fp_type_prefix(b, 11);
        tls_sh_fp(b, sh);
    } else {
        Cur b2 = body; uint64_t cl; Cur ck;
        rd_uint(b2, 2, t); rd_uint(b2, 1, cl);
        cparse(ck, b2, (long)cl);
        if (!cnull(b2)) o.flags |= MFP_FLAG_EMIT;
    }
    }
}

// IP header (ip.h:124, ip.h:448); returns transport protocol or 255
DEV uint32_t ip_parse(Cur &p, const uint8_t *&iph, int &ipv) {
    uint32_t v = look_u8(p);
    iph = nullptr; ipv = 0;
    if ((v & 0xf0) == 0x40) {
        const uint8_t *h = cget_ptr(p, 20);
        ipv = 4;
        if (!h) return 255;
        iph = h;
        long tl = ((long)ld(h + 2) << 8) | ld(h + 3);
        ctrim_to_length(p, tl - 20);
        return ld(h + 9);
    }
    if ((v & 0xf0) == 0x60) {
        const uint8_t *h = cget_ptr(p, 40);
        ipv = 6;
        if (!h) return 255;
        iph = h;
        ctrim_to_length(p, ((long)ld(h + 4) << 8) | ld(h + 5));
        uint32_t nh = ld(h + 6);
        while (clen(p) > 0) {
            bool ext = (nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135 || nh == 139 || nh == 140);
            if (!ext) break;
            uint32_t hdr = nh, nnh = rd_u8(p), hl; Cur dd;
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
template <class E>
DEV void tcp_syn_fp(E &b, int ipv, const uint8_t *iph, const uint8_t *tcph, Cur opts) {
    if (ipv == 4) {
        b.lit("(40)");
        b.putc('(');
        if (ld(iph + 4) == 0 && ld(iph + 5) == 0) { b.putc('0'); b.putc('0'); }
        b.putc(')');
        b.putc('('); b.hex8(ld(iph + 8) & 0xe0); b.putc(')');
    } else {
        b.lit("(60)");
        b.putc('(');
        if (ld(iph + 1) == 0 && ld(iph + 2) == 0 && ld(iph + 3) == 0) { b.putc('0'); b.putc('0'); }
        b.putc(')');
        b.putc('('); b.hex8(ld(iph + 7) & 0xe0); b.putc(')');
    }
    b.putc('('); b.hex(tcph + 14, 2); b.putc(')');
    b.putc('(');
    Cur tmp = opts;
    while (clen(tmp) > 0) {
        uint32_t kind = rd_u8(tmp), len = 0;
        Cur od; cset_null(od);
        if (!(kind == 0 || kind == 1)) {
            len = rd_u8(tmp);
            if (len >= 2) cparse(od, tmp, (long)len - 2);
        }
        b.putc('(');
        b.hex8(kind);
        if (kind == 2 || kind == 3) { b.hex8(len); b.hex(od.d, clen(od)); }
        b.putc(')');
    }
    b.putc(')');
}

DEV bool ppp_is_ip(Cur &p) {                            // ppp::is_ip ppp.h:76
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
    if (b & 1) { uint32_t x; if (!(p.d && p.e > p.d)) { cset_null(p); proto = 0; } else { x = rd_u8(p); proto = x; } }
    else { uint32_t v = 0; for (int i = 0; i < 2; i++) { v *= 256; v += rd_u8(p); } proto = v; }
    return proto == 0x21 || proto == 0x57;
}

// eth::get_ip (eth.h:114-133 over the eth ctor eth.h:137-187): Ethernet
// (802.1ad, 802.1Q, MPLS, Cisco metadata) down to IP, or PPPoE -> PPP -> IP
DEV bool eth_get_ip(Cur &p) {
    uint64_t et;
    cskip(p, 12);
    if (!rd_uint(p, 2, et)) return false;
    if (et == 0x88a8) { cskip(p, 2); if (!rd_uint(p, 2, et)) return false; }
    while (et == 0x8100) { cskip(p, 2); if (!rd_uint(p, 2, et)) return false; }
    if (et == 0x8847) {
        uint64_t lbl = 0;
        while (!(lbl & 0x100)) { if (!rd_uint(p, 4, lbl)) return false; }
        et = 0x0800;
    }
    if (et == 0x8909) { cskip(p, 6); if (!rd_uint(p, 2, et)) return false; }
    if (et == 0x0800 || et == 0x86dd) return true;
    if (et == 0x8864) {
        Cur t; cparse(t, p, 1); cparse(t, p, 1); cparse(t, p, 2); cparse(t, p, 2);
        return ppp_is_ip(p);
    }
    return false;
}

// GRE header (gre_header gre.h): flags/version, protocol type, the checksum
// word when C is set; an inner IP packet follows for IPv4 / IPv6
DEV bool gre_next(Cur &p) {
    uint64_t crv, pt;
    rd_uint(p, 2, crv);
    rd_uint(p, 2, pt);
    if (crv & 0x8000) cskip(p, 4);
    if (cnull(p)) pt = 0;
    return pt == 0x0800 || pt == 0x86dd;
}

// IP layer: ip_write_json pkt_proc.cc:1063 / analyze_ip_packet pkt_proc.cc:1597
template <uint32_t FAM, class E>
DEV void ip_path(E &b, const Cfg &cfg, Out &o, Cur pkt, const uint8_t *base) {
    if (cfg.seg) o.seg_kind = MFP_SEG_IP;   // analyze_ip_packet runs: analysis.reinit() (pkt_proc.cc:1609)
    const uint8_t *iph; int ipv;
    uint32_t proto = ip_parse(pkt, iph, ipv);
    uint32_t enc = 0;            // net bits 20-27: levels, v6 mask, irregular (include/mfp.h)
    // encapsulations::process_encapsulations (pkt_proc.cc:972-1028): up to
    // four levels of IP-in-IP, GRE (IP protocol 47 or UDP port 4754), VXLAN
    // (UDP 4789) and Geneve (UDP 6081), each re-parsing the inner IP header.
    // A tunnel header whose payload is not IP ends the walk with the cursor
    // past it, as in the reference.  Only IP-in-IP levels are described in the
    // record (the JSON writer rebuilds their "encapsulations" entries); any
    // other tunnel marks the chain irregular.
    for (int n = 0; n < 4; n++) {
        const uint8_t *oh = iph; const int ov = ipv;
        bool ipip = false;
        if (proto == 4 || proto == 41) {
            ipip = true;
        } else if (proto == 47) {
            if (!(cfg.select & SEL_GRE)) break;
            if (!gre_next(pkt)) break;
        } else if (proto == 17 && (cfg.select & (SEL_GRE | SEL_VXLAN | SEL_GENEVE))) {
            Cur u = pkt;
            const uint8_t *uh = cget_ptr(u, 8);
            const uint32_t dport = uh ? (ld(uh + 2) << 8) | ld(uh + 3) : 0u;
            const uint32_t sport = uh ? (ld(uh) << 8) | ld(uh + 1) : 0u;
            if ((cfg.block & BLK_UDP_PORTS) && udp_other_port(sport, dport, cfg.block)) {
                break;                                                  // a port-table protocol first
            } else if ((cfg.select & SEL_VXLAN) && dport == 4789) {     // vxlan.hpp
                pkt = u;
                const uint32_t fl = rd_u8(pkt);
                Cur t; cparse(t, pkt, 3); cparse(t, pkt, 3); cparse(t, pkt, 1);
                if (!(fl & 0x08)) break;
                if (!eth_get_ip(pkt)) break;
            } else if ((cfg.select & SEL_GENEVE) && dport == 6081) {    // geneve.hpp
                pkt = u;
                const uint32_t fb = rd_u8(pkt);
                rd_u8(pkt);
                uint64_t pt;
                rd_uint(pkt, 2, pt);
                Cur t; cparse(t, pkt, 3);
                rd_u8(pkt);
                cparse(t, pkt, 4 * (long)(fb & 0x3f));
                if (pt == 0x6558) { if (!eth_get_ip(pkt)) break; }
                else if (pt == 0x0800 || pt == 0x86dd) { }
                else if (pt == 0) {                                      // BSD loopback (loopback.hpp)
                    uint64_t lt;
                    rd_uint(pkt, 4, lt);
                    if (cnull(pkt)) break;
                    if (!(lt == 2 || lt == 0x02000000 || lt == 24 || lt == 0x18000000 || lt == 28 || lt == 0x1c000000 ||
                          lt == 30 || lt == 0x1e000000))
                        break;
                } else {
                    break;
                }
            } else if ((cfg.select & SEL_GRE) && dport == 4754) {       // GRE over UDP
                pkt = u;
                if (!gre_next(pkt)) break;
            } else {
                break;
            }
        } else {
            break;
        }
        proto = ip_parse(pkt, iph, ipv);
        o.flags |= MFP_FLAG_ENCAP;
        if (ov == 6) enc |= 8u << n;
        if (!ipip || !oh || !iph || iph - oh != (ov == 6 ? 40 : 20)) enc |= 128u;
        enc = (enc & ~7u) | (uint32_t)(n + 1);
    }
    if (iph) o.net = (uint32_t)(iph - base) | ((uint32_t)ipv << 16) | (enc << 20);
    if (proto == 6) {
        const uint8_t *tcph = cget_ptr(pkt, 20);
        if (!tcph) return;
        Cur opts; cset_null(opts);
        cparse(opts, pkt, (long)(ld(tcph + 12) >> 4) * 4 - 20);
        o.src_port = (ld(tcph) << 8) | ld(tcph + 1);
        o.dst_port = (ld(tcph + 2) << 8) | ld(tcph + 3);
        uint32_t fl = ld(tcph + 13);
        bool syn = fl & 0x02, ack = fl & 0x10;
        if (cfg.seg) {
            // every whole TCP header resets flow_state_pkts_needed on the analysis
            // path, which skips SYN, SYN/ACK and RST (pkt_proc.cc:1629-1634)
            o.seg_kind |= MFP_SEG_TCP | ((fl & 0x06) ? MFP_SEG_SYN_RST : 0u);
            if (!(syn && cfg.mode == MFP_MODE_WRITE_JSON) && clen(pkt) > 0) {   // process_tcp_data's data segments
                o.seq = (ld(tcph + 4) << 24) | (ld(tcph + 5) << 16) | (ld(tcph + 6) << 8) | ld(tcph + 7);
                o.seg_kind |= MFP_SEG_DATA;
                o.pay_off = (uint32_t)(pkt.d - base);
                o.pay_len = (uint32_t)clen(pkt);
            }
        }
        if (cfg.mode == MFP_MODE_WRITE_JSON) {
            if (syn && !ack) {
                if (cfg.select & SEL_TCP_SYN) {
                    o.msg = MFP_MSG_TCP_SYN;
                    if (cfg.classify) return;
                    o.flags |= MFP_FLAG_EMIT; o.fp_type = 7;
                    if constexpr (E::SEG || !(FAM & FAM_TCP)) { b.punt_pkt(); return; }
                    else {
                        fp_type_prefix(b, 7);
                        tcp_syn_fp(b, ipv, iph, tcph, opts);
                    }
                }
                return;
            }
            if (syn && ack) {
                if ((cfg.select & SEL_TCP_SYN) && (cfg.select & SEL_TCP_SYNACK)) {
                    o.msg = MFP_MSG_TCP_SYNACK;
                    if (cfg.classify) return;
                    o.flags |= MFP_FLAG_EMIT; o.fp_type = 13;
                    if constexpr (E::SEG || !(FAM & FAM_TCP)) { b.punt_pkt(); return; }
                    else {
                        fp_type_prefix(b, 13);
                        tcp_syn_fp(b, ipv, iph, tcph, opts);
                    }
                }
                return;
            }
            if (clen(pkt) == 0) return;
        }
        tcp_data<FAM>(b, cfg, o, pkt, tcph, base);
    } else if (proto == 17) {
        const uint8_t *udph = cget_ptr(pkt, 8);
        if (udph) {
            o.src_port = (ld(udph) << 8) | ld(udph + 1);
            o.dst_port = (ld(udph + 2) << 8) | ld(udph + 3);
        }
        udp_data<FAM>(b, cfg, o, pkt, base);
    }
}

// link layer: stateful_pkt_proc::write_json(..., linktype) pkt_proc.cc:1328
// and analyze_packet pkt_proc.cc:1814
template <uint32_t FAM = FAM_ALL, class E>
DEV void packet_walk(E &b, const Cfg &cfg, Out &o, const uint8_t *data, uint32_t len, uint32_t linktype) {
    o.fp_type = 0; o.msg = 0; o.flags = 0; o.xflags = 0;
    o.sni_off = o.ua_off = 0; o.sni_len = o.ua_len = 0xffff;
    o.src_port = o.dst_port = 0;
    o.net = 0;
    o.pay_off = o.pay_len = 0;
    o.seq = o.more = o.seg_kind = 0;
    Cur p = cmk(data, data + len);
    switch (linktype) {
    case 1:                                             // eth::get_ip eth.h:114
        if (!eth_get_ip(p)) return;
        break;
    case 9:
        if (!ppp_is_ip(p)) return;
        break;
    case 101:
        break;
    case 113: {                                         // linux_sll.hpp
        uint64_t pt, ar, al, pr; Cur lla;
        rd_uint(p, 2, pt); rd_uint(p, 2, ar); rd_uint(p, 2, al); cparse(lla, p, 8); rd_uint(p, 2, pr);
        if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return;
        break;
    }
    case 276: {                                         // linux_sll2.hpp
        uint64_t pr, t, ar; Cur lla;
        rd_uint(p, 2, pr); rd_uint(p, 2, t); rd_uint(p, 4, t); rd_uint(p, 2, ar);
        rd_uint(p, 1, t); rd_uint(p, 1, t); cparse(lla, p, 8);
        if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return;
        break;
    }
    case 0: {                                           // loopback.hpp
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
    ip_path<FAM>(b, cfg, o, p, data);
}

// parameters of the fingerprint kernels (mfp_kernels.hip, mfp_quic.hip)
struct KParams {
    Cfg cfg;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    uint8_t *fp_arena;
    uint64_t fp_cap;
    unsigned long long *fp_used;     // [0] bytes reserved, [1] overflow flag, [2] bytes written, [3] fallback count
    mfp_tcp_seg *seg;                // reassembly inputs per packet (nullptr: not requested)
    const uint32_t *idx;             // packet indices (count = *count); nullptr = all n packets
    const unsigned long long *count;
    uint32_t *quic_idx;              // QUIC packets found by the walkers, for k_quic (count *quic_count)
    unsigned long long *quic_count;
    // spread small batch written straight into page-locked host buffers
    // (mfp_process_small_pinned): the waves count themselves done in *fin;
    // the last copies fp_used to host_out[0..3], resets the counters for
    // the slot's next batch and sets host_out[4] (nullptr: not this mode)
    unsigned long long *fin;
    unsigned long long *host_out;
};
// the reassembly inputs of packet i (when the caller asked for them)
DEV void write_seg(const KParams &P, uint64_t i, const Out &o) {
    if (!P.seg) return;
    mfp_tcp_seg t;
    t.seq = o.seq; t.more = o.more; t.pay_off = o.pay_off;
    t.pay_len = (uint16_t)(o.pay_len > 0xffff ? 0xffff : o.pay_len);
    t.kind = (uint8_t)o.seg_kind; t.reserved = 0;
    P.seg[i] = t;
}


}  // namespace mfp
