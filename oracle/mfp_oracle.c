/*
 * mfp_oracle.c -- plain-C CPU restatement of cisco/mercury's fingerprint path
 * (TEST INFRASTRUCTURE ONLY: the checker for the HIP product path and the
 * "port" CPU baseline in bench.py; the product never links this file).
 *
 * Parity pinned against oracle/_ref (the reference itself, compiled from
 * /root/reference) and the reference golden file
 * test/data/top_100_fingerprints.fp; see tests/test_oracle.py.
 *
 * File:line citations are relative to /root/reference/src/libmerc/.
 */
#define _GNU_SOURCE
#include "mfp_oracle.h"

#include <stddef.h>

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------
 * cursor: restates struct datum (datum.h:220-850).  A null cursor has d==NULL.
 * ---------------------------------------------------------------------- */
typedef struct { const uint8_t *d, *e; } cur;

static inline long clen(cur c) { return c.d ? (long)(c.e - c.d) : 0; }
static inline int cnull(cur c) { return c.d == NULL; }
static inline int cnotempty(cur c) { return c.d != NULL && c.d < c.e; }   /* datum.h:283 */
static inline void cset_null(cur *c) { c->d = c->e = NULL; }

/* datum::skip datum.h:365 */
static int cskip(cur *c, long n) {
    if (!c->d) return 0;
    if (n > c->e - c->d) { c->d = c->e; return 0; }
    c->d += n;
    return 1;
}
/* datum::parse datum.h:294 */
static void cparse(cur *dst, cur *r, long n) {
    if (clen(*r) < n || n < 0) { cset_null(r); cset_null(dst); return; }
    dst->d = r->d; dst->e = r->d ? r->d + n : NULL;
    if (r->d) r->d += n;
}
/* datum::parse_soft_fail datum.h:305 */
static void cparse_soft(cur *dst, cur *r, long n) {
    if (clen(*r) < n) n = clen(*r);
    dst->d = r->d; dst->e = r->d ? r->d + n : NULL;
    if (r->d) r->d += n;
}
/* datum::read_uint8 / read_uint16 / read_uint32 / read_uint datum.h:749-812 */
static int rd_u8(cur *c, unsigned *out) {
    if (c->d && c->e > c->d) { *out = c->d[0]; c->d += 1; return 1; }
    cset_null(c); *out = 0; return 0;
}
static int rd_uint(cur *c, unsigned n, uint64_t *out) {
    if (c->d && c->d + n <= c->e) {
        uint64_t v = 0;
        for (unsigned i = 0; i < n; i++) v = (v << 8) | c->d[i];
        c->d += n; *out = v; return 1;
    }
    cset_null(c); *out = 0; return 0;
}
/* datum::lookahead_uint8 datum.h:702 */
static unsigned look_u8(cur *c) {
    if (c->d && c->e > c->d) return c->d[0];
    cset_null(c); return 0;
}
/* datum::lookahead_uint datum.h:712 (does not null on failure) */
static int look_uint(cur *c, unsigned n, uint64_t *out) {
    if (c->d && c->d + n <= c->e) {
        uint64_t v = 0;
        for (unsigned i = 0; i < n; i++) v = (v << 8) | c->d[i];
        *out = v; return 1;
    }
    return 0;
}
/* datum::init_from_outer_parser datum.h:825 */
static void cinit_outer(cur *dst, cur *outer, uint64_t len) {
    if (!cnotempty(*outer)) return;
    const uint8_t *end = (len > (uint64_t)(outer->e - outer->d)) ? outer->e : outer->d + len;
    dst->d = outer->d; dst->e = end; outer->d = end;
}
/* datum::get_pointer datum.h:737 */
static const uint8_t *cget_ptr(cur *c, long n) {
    if (c->d && c->d + n <= c->e) { const uint8_t *p = c->d; c->d += n; return p; }
    return NULL;
}
/* datum::trim_to_length datum.h:383 (ssize arithmetic restated) */
static void ctrim_to_length(cur *c, long len) {
    if (c->d && len <= (long)(c->e - c->d)) c->e = c->d + len;
}
/* datum::parse_up_to_delim datum.h:313 */
static void cparse_to_delim(cur *dst, cur *r, uint8_t delim) {
    if (!cnotempty(*r)) { cset_null(r); cset_null(dst); return; }
    dst->d = r->d;
    const uint8_t *c = memchr(r->d, delim, r->e - r->d);
    if (c) { dst->e = r->d = c; return; }
    dst->e = r->e;
}
/* datum::parse_up_to_delimiters datum.h:328 */
static uint8_t cparse_to_delims(cur *dst, cur *r, uint8_t d1, uint8_t d2) {
    dst->d = r->d;
    if (r->d) {
        while (r->d < r->e) {
            if (*r->d == d1) { dst->e = r->d; return d1; }
            if (*r->d == d2) { dst->e = r->d; return d2; }
            r->d++;
        }
    }
    dst->e = r->e;
    return 0;
}
/* datum::compare_nbytes datum.h:873 */
static int ccompare_n(cur c, const uint8_t *x, long n) {
    return c.d && clen(c) >= n && (n == 0 || memcmp(x, c.d, n) == 0);
}
/* datum::cmp datum.h:456 */
static int ccmp(cur a, cur b) {
    if (cnull(a)) return cnull(b) ? 0 : -1;
    if (cnull(b)) return 1;
    long la = clen(a), lb = clen(b);
    int r = memcmp(a.d, b.d, la < lb ? la : lb);
    if (r == 0) return (int)(la - lb);
    return r;
}
static inline int c_isupper(uint8_t c) { return c >= 'A' && c <= 'Z'; }
static inline int c_isalpha(uint8_t c) { return (c | 0x20) >= 'a' && (c | 0x20) <= 'z'; }
static inline uint8_t c_tolower(uint8_t c) { return c_isupper(c) ? (uint8_t)(c + 32) : c; }

/* ------------------------------------------------------------------------
 * string builder: restates buffer_stream's truncation rules
 * (buffer_stream.h:100-240, 990-1140); a truncated fingerprint is dropped
 * (fingerprint::final fingerprint.h:136).
 * ---------------------------------------------------------------------- */
#define DLEN MFPO_MAX_FP
typedef struct { char *buf; int off; int trunc; } sb;

static void sb_putc(sb *b, char c) {                       /* append_putc */
    if (b->trunc) return;
    if (b->off >= DLEN) { b->trunc = 1; return; }
    if (b->off < DLEN - 1) b->buf[b->off++] = c; else b->trunc = 1;
}
static void sb_mem(sb *b, const void *s, long len) {       /* append_memcpy */
    if (b->trunc) return;
    if (b->off >= DLEN) { b->trunc = 1; return; }
    if (b->off < (DLEN - 1) - len) { memcpy(b->buf + b->off, s, len); b->off += (int)len; }
    else b->trunc = 1;
}
static void sb_puts(sb *b, const char *s) {                /* append_strncpy */
    if (b->trunc) return;
    if (b->off >= DLEN) { b->trunc = 1; return; }
    int i = 0, gn = 0;
    while (b->off + i < DLEN - 1) {
        if (s[i] != '\0') { b->buf[b->off + i] = s[i]; i++; } else { gn = 1; break; }
    }
    if (!gn) b->trunc = 1;
    b->off += i;
}
static const char hexd[] = "0123456789abcdef";
static void sb_hex(sb *b, const uint8_t *data, long len) { /* raw_as_hex + append_raw_as_hex */
    if (data == NULL) return;
    if (b->trunc) return;
    char outb[256]; int oi = 0;
    for (long i = 0; i < len && !b->trunc; i++) {
        outb[oi] = hexd[data[i] >> 4]; outb[oi + 1] = hexd[data[i] & 15];
        if (oi < 253) oi += 2; else { sb_mem(b, outb, 256); oi = 0; }
    }
    if (oi > 0) sb_mem(b, outb, oi);
}
static void sb_hex16(sb *b, unsigned v) {                  /* append_uint16_hex */
    char o[4] = { hexd[(v >> 12) & 15], hexd[(v >> 8) & 15], hexd[(v >> 4) & 15], hexd[v & 15] };
    sb_mem(b, o, 4);
}
static void sb_uint8(sb *b, unsigned n) {                  /* append_uint8 */
    char o[3]; int i = 0, lead = 1;
    for (int p = 100; p >= 10; p /= 10) {
        int d = n / p; n %= p;
        if (d == 0 && lead) continue;
        lead = 0; o[i++] = '0' + d;
    }
    o[i++] = '0' + n;
    sb_mem(b, o, i);
}

/* fingerprint::get_type_name fingerprint.h:159 */
static const char *fp_name(int t) {
    static const char *name[] = { "unknown", "tls", "tls_server", "http", "http_server", "ssh", "ssh_kex",
                                  "tcp", "dhcp", "smtp_server", "dtls", "dtls_server", "quic", "tcp_server",
                                  "openvpn", "tofsee", "stun", "ssh_init", "ssh_server", "ssh_kex_server",
                                  "ssh_init_server" };
    return (t >= 0 && t <= 20) ? name[t] : name[0];
}
/* fingerprint::set_type fingerprint.h:44 (format_version argument unused by
 * the protocols on this path) */
static void fp_set_type(sb *b, int *type, int t) {
    *type = t;
    sb_puts(b, fp_name(t));
    sb_putc(b, '/');
}

/* ------------------------------------------------------------------------
 * TLS (tls.h)
 * ---------------------------------------------------------------------- */
/* degrease_uint16 tls.h:776 */
static unsigned degrease16(unsigned x) {
    if ((x & 0x0f0f) == 0x0a0a && ((x >> 12) == ((x >> 4) & 15))) return 0x0a0a;
    return x;
}
/* raw_as_hex_degrease tls.h:802 */
static void sb_hex_degrease(sb *b, const uint8_t *p, long len) {
    if (len % 2) len--;
    for (long i = 0; i < len; i += 2) {
        unsigned v = degrease16(((unsigned)p[i] << 8) | p[i + 1]);
        uint8_t t[2] = { (uint8_t)(v >> 8), (uint8_t)v };
        sb_hex(b, t, 2);
    }
}

/* static_extension_types tls.h:1000 */
static int is_static_ext(unsigned t) {
    switch (t) {
    case 1: case 5: case 7: case 8: case 9: case 10: case 11: case 13: case 15: case 16: case 17:
    case 24: case 27: case 28: case 0x39: case 43: case 45: case 50: case 21760: case 0xffa5:
        return 1;
    }
    return 0;
}

typedef struct {
    unsigned type, length, encoded_type;
    const uint8_t *type_ptr, *length_ptr;
    cur value;
    int ok;   /* value.data != NULL */
} tls_ext;

/* tls_extension ctor tls.h:1383 */
static tls_ext ext_parse(cur *p) {
    tls_ext x; memset(&x, 0, sizeof x);
    x.type_ptr = p->d;
    uint64_t v;
    if (!rd_uint(p, 2, &v)) return x;
    x.type = (unsigned)v;
    x.length_ptr = p->d;
    if (!rd_uint(p, 2, &v)) return x;
    x.length = (unsigned)v;
    if ((long)x.length <= clen(*p)) {
        x.value.d = p->d; x.value.e = p->d + x.length; p->d += x.length; x.ok = 1;
    }
    x.encoded_type = ((x.type & 0x0f0f) == 0x0a0a) ? 0x0a0a : x.type;
    return x;
}
static int ext_is_grease(const tls_ext *x) { return (x->type & 0x0f0f) == 0x0a0a; }

/* write_degreased_value tls.h:1513 */
static void ext_write_degreased_value(sb *b, const tls_ext *x, long ungreased) {
    if (!cnotempty(x->value)) return;
    long vl = clen(x->value), skip, gl;
    if (ungreased < vl) { skip = ungreased; gl = vl - ungreased; } else { skip = vl; gl = 0; }
    sb_hex(b, x->value.d, skip);
    sb_hex_degrease(b, x->value.d + skip, gl);
}

/* QUIC varint id datum (quic_vli.hpp:71) */
typedef struct { cur id; int ok; } qtp;
static uint64_t vli_value(cur c) {                      /* variable_length_integer quic_vli.hpp:38 */
    unsigned b; rd_u8(&c, &b);
    int len = (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1;
    uint64_t v = b & 0x3f;
    for (int i = 1; i < len; i++) { rd_u8(&c, &b); v = v * 256 + b; }
    return v;
}
/* quic_transport_parameter ctor tls.h:1247 */
static qtp qtp_parse(cur *d) {
    qtp q; q.ok = 0;
    unsigned b = look_u8(d);
    int len = (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1;
    cparse(&q.id, d, len);
    /* _length: variable_length_integer read from d */
    unsigned bb; rd_u8(d, &bb);
    int l2 = (bb & 0xc0) == 0xc0 ? 8 : (bb & 0xc0) == 0x80 ? 4 : (bb & 0xc0) == 0x40 ? 2 : 1;
    uint64_t v = bb & 0x3f;
    for (int i = 1; i < l2; i++) { rd_u8(d, &bb); v = v * 256 + bb; }
    cur val;
    long vlen = (v > (uint64_t)0x7fffffffffffffffULL) ? -1 : (long)v;
    cparse(&val, d, vlen);
    q.ok = !cnull(val);
    return q;
}
static int qtp_is_grease(cur id) { return vli_value(id) % 31 == 27; }
static void qtp_write_id(sb *b, cur id) {
    if (!qtp_is_grease(id)) sb_hex(b, id.d, clen(id));
    else { sb_putc(b, '1'); sb_putc(b, 'b'); }
}
/* fmt-1 QTP id comparator tls.h:1453 */
static int qtp_less(cur a, cur bb) {
    int ga = qtp_is_grease(a), gb = qtp_is_grease(bb);
    if (ga) { if (gb) return 0; return 0x1b < vli_value(bb); }
    if (gb) return vli_value(a) < 0x1b;
    return ccmp(a, bb) < 0;
}

/* libstdc++ __insertion_sort (exactly the order std::sort yields for
 * n <= 16; for consistent comparators, any n) */
#define INSERTION_SORT(T, arr, n, LESS)                                      \
    for (long _i = 1; _i < (long)(n); _i++) {                                \
        T _v = (arr)[_i];                                                    \
        if (LESS(&_v, &(arr)[0])) {                                          \
            memmove(&(arr)[1], &(arr)[0], sizeof(T) * _i); (arr)[0] = _v;    \
        } else {                                                             \
            long _j = _i;                                                    \
            while (LESS(&_v, &(arr)[_j - 1])) { (arr)[_j] = (arr)[_j - 1]; _j--; } \
            (arr)[_j] = _v;                                                  \
        }                                                                    \
    }

static int qtpid_less_p(const cur *a, const cur *b) { return qtp_less(*a, *b); }

/* tls_extension::fingerprint_format1 tls.h:1413 (role: 0 client, 1 server) */
static void ext_fp_format1(sb *b, tls_ext *x, int role) {
    if (is_static_ext(x->type)) {
        if (x->type == 0x000a) {
            sb_putc(b, '('); sb_hex16(b, x->encoded_type);
            if (x->length_ptr) sb_hex_degrease(b, x->length_ptr, 2);
            ext_write_degreased_value(b, x, 2);
            sb_putc(b, ')');
        } else if (x->type == 0x002b) {
            sb_putc(b, '('); sb_hex16(b, x->encoded_type);
            if (x->length_ptr) sb_hex_degrease(b, x->length_ptr, 2);
            ext_write_degreased_value(b, x, role == 0 ? 1 : 0);
            sb_putc(b, ')');
        } else if (x->type == 0x39 || x->type == 0xffa5) {
            sb_putc(b, '('); sb_putc(b, '('); sb_hex16(b, x->encoded_type); sb_putc(b, ')');
            cur ids[4096]; long n = 0;
            cur v = x->value;
            while (!cnull(v)) {
                cur save_id; qtp q = qtp_parse(&v); save_id = q.id;
                if (q.ok && n < 4096) ids[n++] = save_id;
            }
            INSERTION_SORT(cur, ids, n, qtpid_less_p);
            sb_putc(b, '[');
            for (long i = 0; i < n; i++) { sb_putc(b, '('); qtp_write_id(b, ids[i]); sb_putc(b, ')'); }
            sb_putc(b, ']');
            sb_putc(b, ')');
        } else {
            sb_putc(b, '('); sb_hex16(b, x->encoded_type);
            if (x->length_ptr) sb_hex_degrease(b, x->length_ptr, 2);
            if (cnotempty(x->value)) sb_hex(b, x->value.d, clen(x->value));
            sb_putc(b, ')');
        }
    } else {
        sb_putc(b, '('); sb_hex16(b, x->encoded_type); sb_putc(b, ')');
    }
}

/* tls_extensions::fingerprint (format 0) tls.h:1549 */
static void exts_fp0(sb *b, cur exts, int role) {
    cur p = exts;
    sb_putc(b, '(');
    while (clen(p) > 0) {
        tls_ext x = ext_parse(&p);
        if (!x.ok) break;
        if (is_static_ext(x.type)) {
            if (x.type == 0x000a || x.type == 0x002b) {
                sb_putc(b, '(');
                if (x.type_ptr) sb_hex_degrease(b, x.type_ptr, 2);
                if (x.length_ptr) sb_hex_degrease(b, x.length_ptr, 2);
                ext_write_degreased_value(b, &x, x.type == 0x000a ? 2 : (role == 0 ? 1 : 0));
                sb_putc(b, ')');
            } else if (x.type == 0x39 || x.type == 0xffa5) {
                sb_putc(b, '('); sb_putc(b, '(');
                if (x.type_ptr) sb_hex_degrease(b, x.type_ptr, 2);
                sb_putc(b, ')');
                sb_putc(b, '(');
                cur v = x.value;
                while (!cnull(v)) {
                    qtp q = qtp_parse(&v);
                    if (q.ok) { sb_putc(b, '('); qtp_write_id(b, q.id); sb_putc(b, ')'); }
                }
                sb_putc(b, ')'); sb_putc(b, ')');
            } else {
                sb_putc(b, '(');
                if (x.type_ptr) sb_hex_degrease(b, x.type_ptr, 2);
                if (x.length_ptr) sb_hex_degrease(b, x.length_ptr, 2);
                if (cnotempty(x.value)) sb_hex(b, x.value.d, clen(x.value));
                sb_putc(b, ')');
            }
        } else {
            sb_putc(b, '(');
            if (x.type_ptr) sb_hex_degrease(b, x.type_ptr, 2);
            sb_putc(b, ')');
        }
    }
    sb_putc(b, ')');
}

/* fmt-1 comparator tls.h:1637 */
static int ext_less1(const tls_ext *a, const tls_ext *b) {
    int ga = ext_is_grease(a), gb = ext_is_grease(b);
    if (ga) { if (gb) return 0; return 0x0a0a < b->type; }
    if (gb) return a->type < 0x0a0a;
    if (a->type != b->type) return a->type < b->type;
    if (a->length != b->length) return a->length < b->length;
    return ccmp(a->value, b->value) < 0;
}
/* fmt-2 within-bucket comparator tls.h:1709 */
static int ext_less2(const tls_ext *a, const tls_ext *b) {
    int ga = ext_is_grease(a), gb = ext_is_grease(b);
    if (ga) { if (gb) return 0; return 0x0a0a < b->type; }
    if (gb) return a->type < 0x0a0a;
    if (a->length != b->length) return a->length < b->length;
    return ccmp(a->value, b->value) < 0;
}

#define MAX_EXTS 16384
/* tls_extensions::fingerprint_quic_tls (format 1) tls.h:1618 */
static void exts_fp1(sb *b, cur exts, int role) {
    tls_ext *v = malloc(sizeof(tls_ext) * MAX_EXTS);
    long n = 0;
    cur p = exts;
    while (clen(p) > 0) {
        tls_ext x = ext_parse(&p);
        if (!x.ok) break;
        if (n < MAX_EXTS) v[n++] = x;
    }
    INSERTION_SORT(tls_ext, v, n, ext_less1);
    sb_putc(b, '[');
    for (long i = 0; i < n; i++) ext_fp_format1(b, &v[i], role);
    sb_putc(b, ']');
    free(v);
}

/* tls_extensions_assign::get_index tls_extensions.h:15-110 */
static int fmt2_index(unsigned t) {
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
/* tls_extensions::fingerprint_format2 tls.h:1664 */
static void exts_fp2(sb *b, cur exts, int role) {
    static __thread tls_ext list[71][3];
    int cnt[71]; memset(cnt, 0, sizeof cnt);
    cur p = exts;
    while (clen(p) > 0) {
        tls_ext x = ext_parse(&p);
        if (!x.ok) break;
        int idx = fmt2_index(x.type);
        if (idx == -1) {
            if (x.type == 65280 || x.type >= 65282) x.encoded_type = 65280;          /* private */
            else if (x.type >= 62 && x.type <= 65279 && !ext_is_grease(&x)) x.encoded_type = 62;  /* unassigned */
            idx = fmt2_index(x.encoded_type);
        }
        if (idx >= 0 && cnt[idx] < 3) list[idx][cnt[idx]++] = x;
    }
    sb_putc(b, '[');
    for (int k = 0; k < 71; k++) {
        if (cnt[k] > 1) { INSERTION_SORT(tls_ext, list[k], cnt[k], ext_less2); }
        for (int j = 0; j < cnt[k]; j++) ext_fp_format1(b, &list[k][j], role);
    }
    sb_putc(b, ']');
}

/* tls_record::parse tls.h:153; tls_handshake::parse tls.h:244 */
typedef struct { cur fragment; } tls_record;
static tls_record tls_record_parse(cur *d) {
    tls_record r; cset_null(&r.fragment);
    if (clen(*d) < 5) return r;
    uint64_t len, tmp;
    rd_uint(d, 1, &tmp); rd_uint(d, 2, &tmp); rd_uint(d, 2, &len);
    cinit_outer(&r.fragment, d, len);
    return r;
}
typedef struct { unsigned msg_type; uint64_t length; cur body; uint64_t more; } tls_hs;
static tls_hs tls_hs_parse(cur *d) {
    tls_hs h; h.msg_type = 0; h.length = 0; cset_null(&h.body); h.more = 0;
    if (clen(*d) < 4) return h;
    uint64_t t;
    rd_uint(d, 1, &t); h.msg_type = (unsigned)t;
    rd_uint(d, 3, &t); h.length = t;
    if (h.length > 32768) return h;
    cinit_outer(&h.body, d, h.length);
    h.more = h.length - (uint64_t)clen(h.body);
    return h;
}

typedef struct {
    cur version, random, session_id, ciphers, compression, extensions;
    int dtls;
} tls_ch;
/* tls_client_hello::parse tls.h:1811 */
static void tls_ch_parse(tls_ch *ch, cur p) {
    memset(ch, 0, sizeof *ch);
    uint64_t l;
    cparse(&ch->version, &p, 2);
    if (!cnotempty(ch->version)) return;
    if (ch->version.d[0] == 0xfe) ch->dtls = 1;
    cparse(&ch->random, &p, 32);
    if (!rd_uint(&p, 1, &l)) return;
    cparse(&ch->session_id, &p, (long)l);
    if (ch->dtls) {
        if (!look_uint(&p, 1, &l)) return;
        if (!cskip(&p, (long)l + 1)) return;
    }
    if (!rd_uint(&p, 2, &l)) return;
    if (l & 1) return;
    cparse(&ch->ciphers, &p, (long)l);
    if (!rd_uint(&p, 1, &l)) return;
    cparse(&ch->compression, &p, (long)l);
    if (!rd_uint(&p, 2, &l)) return;
    cparse_soft(&ch->extensions, &p, (long)l);
}
/* tls_client_hello::fingerprint tls.h:1928 */
static void tls_ch_fp(sb *b, const tls_ch *ch, unsigned fmt) {
    if (!cnotempty(ch->compression)) return;
    if (fmt >= 1 && fmt <= 2) { sb_uint8(b, fmt); sb_putc(b, '/'); }
    else if (fmt != 0) return;
    sb_putc(b, '('); sb_hex(b, ch->version.d, clen(ch->version)); sb_putc(b, ')');
    sb_putc(b, '('); sb_hex_degrease(b, ch->ciphers.d, clen(ch->ciphers)); sb_putc(b, ')');
    if (fmt == 0) exts_fp0(b, ch->extensions, 0);
    else if (fmt == 1) exts_fp1(b, ch->extensions, 0);
    else exts_fp2(b, ch->extensions, 0);
}
/* tls_extensions::set_meta_data tls.h:1316: server_name and the ALPN
 * protocol_name_list (tls.h:1172-1176; a short list is none) */
static void tls_sni(cur exts, int32_t *off, int32_t *len, int32_t *aoff, int32_t *alen, const uint8_t *base) {
    cur p = exts;
    while (clen(p) > 0) {
        const uint8_t *start = p.d;
        uint64_t t, l;
        if (!rd_uint(&p, 2, &t)) break;
        if (!rd_uint(&p, 2, &l)) break;
        if (!cskip(&p, (long)l)) break;
        if (t == 0) {
            cur e = { start, p.d };
            cskip(&e, 9);
            *off = (int32_t)(e.d - base); *len = (int32_t)clen(e);
        }
        if (t == 16) {
            cur e = { start, p.d };
            uint64_t al;
            cskip(&e, 4);
            if (rd_uint(&e, 2, &al) && (uint64_t)clen(e) >= al) { *aoff = (int32_t)(e.d - base); *alen = (int32_t)al; }
            else { *aoff = 0; *alen = -1; }
        }
    }
}

typedef struct { cur version, random, cipher, compression, extensions; } tls_sh;
/* tls_server_hello::parse_tls_server_hello tls.h:2097 */
static void tls_sh_parse(tls_sh *sh, cur *rec) {
    uint64_t l;
    cparse(&sh->version, rec, 2);
    cparse(&sh->random, rec, 32);
    if (!look_uint(rec, 1, &l)) return;
    if (!cskip(rec, (long)l + 1)) return;
    cparse(&sh->cipher, rec, 2);
    cparse(&sh->compression, rec, 1);
    if (!rd_uint(rec, 2, &l)) return;
    cparse(&sh->extensions, rec, (long)l);
}
/* tls_server_hello::is_not_empty tls.h:513 */
static int tls_sh_not_empty(const tls_sh *sh) {
    cur t = sh->version; uint64_t v;
    rd_uint(&t, 2, &v);
    if (!(v == 0x0303 || v == 0x0302 || v == 0x0301 || v == 0x0300 || v == 0xfeff || v == 0xfefd)) return 0;
    return cnotempty(sh->cipher);
}
/* tls_server_hello::fingerprint tls.h:2126 */
static void tls_sh_fp(sb *b, const tls_sh *sh) {
    if (!tls_sh_not_empty(sh)) return;
    sb_putc(b, '('); sb_hex(b, sh->version.d, clen(sh->version)); sb_putc(b, ')');
    sb_putc(b, '('); sb_hex(b, sh->cipher.d, clen(sh->cipher)); sb_putc(b, ')');
    exts_fp0(b, sh->extensions, 1);
}
/* tls_server_certificate::parse tls.h:281 */
typedef struct { cur list; uint64_t more; } tls_cert;
static void tls_cert_parse(tls_cert *c, cur *d) {
    uint64_t t = 0;
    if (!rd_uint(d, 3, &t)) return;
    if (t > 65536) { cset_null(d); return; }
    cinit_outer(&c->list, d, t);
    c->more = t - (uint64_t)clen(c->list);
}

/* ------------------------------------------------------------------------
 * SSH (ssh.h)
 * ---------------------------------------------------------------------- */
typedef struct { cur payload; uint64_t more; cur trailing; } ssh_bin;
/* ssh_binary_packet ssh.h:56 */
static void ssh_bin_parse(ssh_bin *b, cur *p) {
    memset(b, 0, sizeof *b);
    uint64_t plen, pad;
    rd_uint(p, 4, &plen);     /* encoded<uint32_t> */
    rd_uint(p, 1, &pad);      /* encoded<uint8_t>  */
    if (plen > 16384 || plen < 1) { if (p->d) p->d = p->e; return; }   /* set_empty */
    if (!cnotempty(*p)) return;
    long left = (long)plen - 1;
    if (left > clen(*p)) b->more = left - clen(*p);
    cparse_soft(&b->payload, p, left);
    if (cnotempty(*p)) b->trailing = *p;
}
typedef struct { cur nl[10]; } ssh_kex;
/* name_list::parse ssh.h:110 */
static void name_list_parse(cur *nl, cur *p) {
    uint64_t l;
    rd_uint(p, 4, &l);
    if (l > 2048) { if (p->d) p->d = p->e; return; }
    cparse(nl, p, (long)l);
}
/* ssh_kex_init::parse ssh.h:190 */
static void ssh_kex_parse(ssh_kex *k, cur p) {
    memset(k, 0, sizeof *k);
    cur t;
    cparse(&t, &p, 1);
    cparse(&t, &p, 16);
    for (int i = 0; i < 10; i++) name_list_parse(&k->nl[i], &p);
}
/* ssh_kex_init::fingerprint ssh.h:240 */
static void ssh_kex_fp(sb *b, const ssh_kex *k) {
    if (!cnotempty(k->nl[0])) return;
    for (int i = 0; i < 10; i++) {
        sb_putc(b, '(');
        if (cnotempty(k->nl[i])) sb_hex(b, k->nl[i].d, clen(k->nl[i]));
        sb_putc(b, ')');
    }
}
typedef struct { cur proto, comment; ssh_bin bin; ssh_kex kex; int has_kex; } ssh_init;
/* ssh_init_packet::parse ssh.h:342 */
static void ssh_init_parse(ssh_init *s, cur p) {
    memset(s, 0, sizeof *s);
    uint8_t delim = cparse_to_delims(&s->proto, &p, '\n', ' ');
    if (delim != '\n') {
        cskip(&p, 1);
        cparse_to_delim(&s->comment, &p, '\n');
    }
    cskip(&p, 1);
    if (cnotempty(p)) {
        ssh_bin_parse(&s->bin, &p);
        if (cnotempty(s->bin.payload)) {
            ssh_kex_parse(&s->kex, s->bin.payload);
            s->has_kex = 1;
        }
    }
}
/* ssh_init_packet::write_fingerprint_data ssh.h:382 / fingerprint ssh.h:411 */
static void ssh_init_fp(sb *b, const ssh_init *s) {
    if (s->has_kex && cnotempty(s->kex.nl[0])) { ssh_kex_fp(b, &s->kex); return; }
    if (!cnotempty(s->proto)) return;
    sb_putc(b, '(');
    if (cnotempty(s->comment)) {
        sb_hex(b, s->proto.d, clen(s->proto));
        sb_putc(b, '2'); sb_putc(b, '0');
        cur t = s->comment; t.e -= 1; if (t.e < t.d) t.e = t.d;
        sb_hex(b, t.d, clen(t));
    } else {
        cur t = s->proto; t.e -= 1; if (t.e < t.d) t.e = t.d;
        sb_hex(b, t.d, clen(t));
    }
    sb_putc(b, ')');
}

/* ------------------------------------------------------------------------
 * HTTP (http.h, http.cc)
 * ---------------------------------------------------------------------- */
/* http.cc:426-445 request header fingerprint table: 1 = include value */
static const char *req_fp_names[] = { "accept", "accept-encoding", "connection", "dnt", "dpr",
    "upgrade-insecure-requests", "x-requested-with", "accept-charset", "accept-language", "authorization",
    "cache-control", "host", "if-modified-since", "keep-alive", "user-agent", "x-flash-version",
    "x-p2p-peerdist", NULL };
static const int req_fp_val[] = { 1,1,1,1,1,1,1, 0,0,0,0,0,0,0,0,0,0 };
/* http.cc:487-536 response table */
static const char *resp_fp_names[] = { "access-control-allow-credentials", "access-control-allow-headers",
    "access-control-allow-methods", "access-control-expose-headers", "cache-control", "code", "connection",
    "content-language", "content-transfer-encoding", "p3p", "pragma", "reason", "server",
    "strict-transport-security", "version", "x-aspnetmvc-version", "x-aspnet-version", "x-cid",
    "x-ms-version", "x-xss-protection", "appex-activity-id", "cdnuuid", "cf-ray", "content-range",
    "content-type", "date", "etag", "expires", "flow_context", "ms-cv", "msregion", "ms-requestid",
    "request-id", "vary", "x-amz-cf-pop", "x-amz-request-id", "x-azure-ref-originshield", "x-cache",
    "x-cache-hits", "x-ccc", "x-diagnostic-s", "x-feserver", "x-hw", "x-msedge-ref",
    "x-ocsp-responder-id", "x-requestid", "x-served-by", "x-timer", "x-trace-context", NULL };
static const int resp_fp_nval = 20;   /* first 20 entries include the value */

/* perfect_hash::lookup perfect_hash.h:256 (exact ASCII case-insensitive
 * membership); returns index or -1 */
static int name_lookup(const char **names, cur n) {
    long l = clen(n);
    for (int i = 0; names[i]; i++) {
        if ((long)strlen(names[i]) != l) continue;
        int ok = 1;
        for (long j = 0; j < l; j++) if (c_tolower(n.d[j]) != c_tolower((uint8_t)names[i][j])) { ok = 0; break; }
        if (ok) return i;
    }
    return -1;
}

/* delimiter::delimiter(datum&, const datum&) http.h:113 ; returns is_valid */
static int http_delim(cur *p, cur del) {
    cur dl; cset_null(&dl);
    if (ccompare_n(*p, del.d, clen(del))) cparse(&dl, p, clen(del));
    else if (ccompare_n(*p, (const uint8_t *)"\r\n", 2)) cparse(&dl, p, 2);
    else if (ccompare_n(*p, (const uint8_t *)"\n", 1)) cparse(&dl, p, 1);
    return cnotempty(dl);
}

typedef struct { cur method, protocol, version, status, reason, body, delim; } http_msg;

/* new_http_headers::fingerprint http.h:335 + httpheader http.h:146 ;
 * also captures first host / user-agent values (request only) */
static void http_headers_fp(sb *b, const http_msg *m, const char **names, int nval_mode, int nval,
                            const int *valflags, cur *host, cur *ua) {
    cur tmp = m->body;
    while (1) {
        if (http_delim(&tmp, m->delim)) break;
        /* httpheader(tmp, delim) */
        cur hdr_body = tmp, name;
        cset_null(&name);
        if (!cnotempty(tmp)) { cset_null(&tmp); } else {
            name.d = tmp.d;
            const uint8_t *c = memchr(tmp.d, ':', tmp.e - tmp.d);
            if (c) { name.e = c; tmp.d = c; } else name.e = tmp.e;
        }
        /* literal_byte<':'> */
        if (tmp.d && tmp.e > tmp.d && tmp.d[0] == ':') tmp.d++; else cset_null(&tmp);
        /* LWS */
        while (tmp.d && tmp.d < tmp.e && (*tmp.d == '\t' || *tmp.d == ' ')) tmp.d++;
        cur value;
        cparse_to_delims(&value, &tmp, '\r', '\n');
        http_delim(&tmp, m->delim);
        hdr_body.e = value.e;
        int valid = !cnull(tmp);
        if (!valid) break;
        int idx = name_lookup(names, name);
        if (idx >= 0) {
            int incl = nval_mode ? (idx < nval) : valflags[idx];
            sb_putc(b, '(');
            if (incl) sb_hex(b, hdr_body.d, clen(hdr_body)); else sb_hex(b, name.d, clen(name));
            sb_putc(b, ')');
        }
        if (host && ua) {
            static const char *cap[] = { "host", "user-agent", NULL };
            int ci = name_lookup(cap, name);
            if (ci == 0 && cnull(*host)) *host = value;
            if (ci == 1 && cnull(*ua)) *ua = value;
        }
    }
}

/* http_request::parse http.cc:105 */
static void http_req_parse(http_msg *m, cur p) {
    memset(m, 0, sizeof *m);
    cur uri;
    cparse_to_delim(&m->method, &p, ' ');
    long ml = clen(m->method);
    if (ml < 3 || ml > 16) return;
    for (long i = 0; i < ml; i++) if (!c_isupper(m->method.d[i])) return;
    cskip(&p, 1);
    cparse_to_delim(&uri, &p, ' ');
    cskip(&p, 1);
    cparse_to_delims(&m->protocol, &p, '\r', '\n');
    if (!(m->protocol.d && clen(m->protocol) >= 5 && memcmp(m->protocol.d, "HTTP/", 5) == 0)) {
        cset_null(&m->protocol); return;
    }
    /* delimiter(p) http.h:106 */
    m->delim.d = p.d;
    while (p.d && p.d < p.e && !c_isalpha(*p.d)) p.d++;
    m->delim.e = p.d;
    m->body = p;
}
/* http_response::parse http.cc:369 */
static void http_resp_parse(http_msg *m, cur p) {
    memset(m, 0, sizeof *m);
    cparse_to_delim(&m->version, &p, ' ');
    cskip(&p, 1);
    cparse_to_delim(&m->status, &p, ' ');
    cskip(&p, 1);
    cparse_to_delims(&m->reason, &p, '\r', '\n');
    m->delim.d = p.d;
    while (p.d && p.d < p.e && !c_isalpha(*p.d)) p.d++;
    m->delim.e = p.d;
    m->body = p;
}

/* ------------------------------------------------------------------------
 * TCP SYN (tcpip.h:215-249, ip.h:141-163,478-503)
 * ---------------------------------------------------------------------- */
static void tcp_syn_fp(sb *b, int ipv, const uint8_t *iph, const uint8_t *tcph, cur opts) {
    if (ipv == 4) {
        sb_puts(b, "(40)");
        sb_putc(b, '(');
        if (iph[4] == 0 && iph[5] == 0) { sb_putc(b, '0'); sb_putc(b, '0'); }
        sb_putc(b, ')');
        sb_putc(b, '('); uint8_t t = iph[8] & 0xe0; sb_hex(b, &t, 1); sb_putc(b, ')');
    } else {
        sb_puts(b, "(60)");
        sb_putc(b, '(');
        /* ipv6_header::flow_label ip.h:393: uint20_t{bytes[1]<<16|bytes[2]<<8|bytes[3]}
         * (no masking: the traffic-class nibble in bytes[1] counts too) */
        uint32_t fl = ((uint32_t)iph[1] << 16) | ((uint32_t)iph[2] << 8) | iph[3];
        if (fl == 0) { sb_putc(b, '0'); sb_putc(b, '0'); }
        sb_putc(b, ')');
        sb_putc(b, '('); uint8_t t = iph[7] & 0xe0; sb_hex(b, &t, 1); sb_putc(b, ')');
    }
    sb_putc(b, '('); sb_hex(b, tcph + 14, 2); sb_putc(b, ')');
    sb_putc(b, '(');
    cur tmp = opts;
    while (clen(tmp) > 0) {
        unsigned kind = 0, len = 0; cur od; cset_null(&od);
        rd_u8(&tmp, &kind);
        if (!(kind == 0 || kind == 1)) {
            rd_u8(&tmp, &len);
            if (len >= 2) cparse(&od, &tmp, (long)len - 2);
        }
        sb_putc(b, '(');
        uint8_t k = (uint8_t)kind; sb_hex(b, &k, 1);
        if (kind == 2 || kind == 3) {
            uint8_t l8 = (uint8_t)len; sb_hex(b, &l8, 1);
            sb_hex(b, od.d, clen(od));
        }
        sb_putc(b, ')');
    }
    sb_putc(b, ')');
}

/* ------------------------------------------------------------------------
 * packet walk (pkt_proc.cc, eth.h, ip.h, tcpip.h, udp.h)
 * ---------------------------------------------------------------------- */
static int matches(cur p, const uint8_t *mask, const uint8_t *val, int n) {   /* match.h:64 */
    if (!p.d || clen(p) < n) return 0;
    for (int i = 0; i < n; i++) if ((p.d[i] & mask[i]) != val[i]) return 0;
    return 1;
}
static const uint8_t M_TLS[8]  = { 0xff, 0xff, 0xfc, 0, 0, 0xff, 0, 0 };
static const uint8_t V_CH[8]   = { 0x16, 0x03, 0, 0, 0, 0x01, 0, 0 };
static const uint8_t V_SH[8]   = { 0x16, 0x03, 0, 0, 0, 0x02, 0, 0 };
static const uint8_t V_CERT[8] = { 0x16, 0x03, 0, 0, 0, 0x0b, 0, 0 };
static const uint8_t M_SSH[8]  = { 0xff, 0xff, 0xff, 0xff, 0, 0, 0, 0 };
static const uint8_t V_SSH[8]  = { 'S', 'S', 'H', '-', 0, 0, 0, 0 };
static const uint8_t M_KEX[8]  = { 0xff, 0xff, 0xf0, 0, 0, 0xff, 0, 0 };
static const uint8_t V_KEX[8]  = { 0, 0, 0, 0, 0, 0x14, 0, 0 };
static const uint8_t M_DTLS[16] = { 0xff, 0xff, 0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0, 0 };
static const uint8_t V_DCH[16]  = { 0x16, 0xfe, 0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01, 0, 0 };
static const uint8_t V_DSH[16]  = { 0x16, 0xfe, 0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0 };
static const uint8_t V_DHV[16]  = { 0x16, 0xfe, 0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x03, 0, 0 };

/* HTTP request keywords of tcp_keyword_matcher proto_identify.h:200-236
 * that map to http_request (incl. "DELE", which also maps to ftp) */
static int is_http_req_keyword(uint32_t k) {
    static const char *kw[] = { "ACL ", "BASE", "BIND", "CHEC", "CONN", "COPY", "DELE", "GET ", "HEAD",
        "LABE", "LINK", "LOCK", "MERG", "MKAC", "MKCA", "MKCO", "MKRE", "MKWO", "MOVE", "OPTI", "ORDE",
        "PATC", "POST", "PRI ", "PROP", "PUT ", "REBI", "REPO", "SEAR", "TRAC", "UNBI", "UNCH", "UNLI",
        "UNLO", "UPDA", "VERS", NULL };
    for (int i = 0; kw[i]; i++) {
        uint32_t v = ((uint32_t)(uint8_t)kw[i][0] << 24) | ((uint32_t)(uint8_t)kw[i][1] << 16) |
                     ((uint32_t)(uint8_t)kw[i][2] << 8) | (uint8_t)kw[i][3];
        if (v == k) return 1;
    }
    return 0;
}

typedef struct {
    const mfpo_config *cfg;
    mfpo_result *res;
    sb b;
    int type;
    const uint8_t *base;
} ctx;

static void finish_fp(ctx *c) {
    /* fingerprint::final fingerprint.h:136 */
    if (c->b.trunc || c->type == 0) {
        /* the 8191-char corner: putc may reach doff 8191 without truncation */
        c->res->fp_type = 0; c->res->fp_len = 0; c->res->fp[0] = 0;
        return;
    }
    c->res->fp_type = (uint32_t)c->type;
    c->res->fp_len = (uint32_t)c->b.off;
    c->res->fp[c->b.off] = 0;
}

/* set_tcp_protocol pkt_proc.cc:488 (selection subset) */
static void tcp_data(ctx *c, cur pkt, const uint8_t *tcph) {
    const mfpo_config *cfg = c->cfg;
    mfpo_result *r = c->res;
    unsigned sel = cfg->select;
    unsigned sport = ((unsigned)tcph[0] << 8) | tcph[1], dport = ((unsigned)tcph[2] << 8) | tcph[3];
    int msg = 0;
    if (clen(pkt) >= 4) {
        if ((sel & MFPO_SEL_TLS_CH) && matches(pkt, M_TLS, V_CH, 8)) msg = MFPO_MSG_TLS_CH;
        else if ((sel & MFPO_SEL_TLS_SH) && matches(pkt, M_TLS, V_SH, 8)) msg = MFPO_MSG_TLS_SH;
        else if ((sel & MFPO_SEL_TLS_CERT) && matches(pkt, M_TLS, V_CERT, 8)) msg = MFPO_MSG_TLS_CERT;
        else if ((sel & (MFPO_SEL_SSH_CLIENT | MFPO_SEL_SSH_SERVER)) && matches(pkt, M_SSH, V_SSH, 8)) msg = MFPO_MSG_SSH_INIT;
        else if ((sel & (MFPO_SEL_SSH_CLIENT | MFPO_SEL_SSH_SERVER)) && matches(pkt, M_KEX, V_KEX, 8)) msg = MFPO_MSG_SSH_KEX;
    }
    if (msg == 0 && clen(pkt) >= 4) {
        uint32_t kw = ((uint32_t)pkt.d[0] << 24) | ((uint32_t)pkt.d[1] << 16) | ((uint32_t)pkt.d[2] << 8) | pkt.d[3];
        if ((sel & MFPO_SEL_HTTP_REQ) && is_http_req_keyword(kw)) {
            http_msg m; http_req_parse(&m, pkt);
            if (cnotempty(m.protocol)) {
                r->msg = MFPO_MSG_HTTP_REQ; r->emit = 1;
                fp_set_type(&c->b, &c->type, MFPO_FP_HTTP);
                sb_putc(&c->b, '('); sb_hex(&c->b, m.method.d, clen(m.method)); sb_putc(&c->b, ')');
                sb_putc(&c->b, '('); sb_hex(&c->b, m.protocol.d, clen(m.protocol)); sb_putc(&c->b, ')');
                sb_putc(&c->b, '(');
                cur host = { NULL, NULL }, ua = { NULL, NULL };
                http_headers_fp(&c->b, &m, req_fp_names, 0, 0, req_fp_val, &host, &ua);
                sb_putc(&c->b, ')');
                if (!cnull(host)) { r->sni_off = (int32_t)(host.d - c->base); r->sni_len = (int32_t)clen(host); }
                if (!cnull(ua)) { r->ua_off = (int32_t)(ua.d - c->base); r->ua_len = (int32_t)clen(ua); }
                finish_fp(c);
            }
            return;
        }
        if ((sel & MFPO_SEL_HTTP_RESP) && kw == 0x48545450u /* "HTTP" */) {
            http_msg m; http_resp_parse(&m, pkt);
            if (cnotempty(m.status)) {
                r->msg = MFPO_MSG_HTTP_RESP; r->emit = 1;
                fp_set_type(&c->b, &c->type, MFPO_FP_HTTP_SERVER);
                sb_putc(&c->b, '('); sb_hex(&c->b, m.version.d, clen(m.version)); sb_putc(&c->b, ')');
                sb_putc(&c->b, '('); sb_hex(&c->b, m.status.d, clen(m.status)); sb_putc(&c->b, ')');
                sb_putc(&c->b, '('); sb_hex(&c->b, m.reason.d, clen(m.reason)); sb_putc(&c->b, ')');
                sb_putc(&c->b, '(');
                http_headers_fp(&c->b, &m, resp_fp_names, 1, resp_fp_nval, NULL, NULL, NULL);
                sb_putc(&c->b, ')');
                finish_fp(c);
            }
            return;
        }
        return;
    }
    switch (msg) {
    case MFPO_MSG_TLS_CH: {
        cur p = pkt;
        tls_record rec = tls_record_parse(&p);
        tls_hs hs = tls_hs_parse(&rec.fragment);
        if (hs.more) r->truncated = 1;
        tls_ch ch; tls_ch_parse(&ch, hs.body);
        r->msg = MFPO_MSG_TLS_CH;
        if (!cnotempty(ch.compression)) return;
        r->emit = 1;
        fp_set_type(&c->b, &c->type, MFPO_FP_TLS);
        tls_ch_fp(&c->b, &ch, cfg->tls_format);
        tls_sni(ch.extensions, &r->sni_off, &r->sni_len, &r->ua_off, &r->ua_len, c->base);
        finish_fp(c);
        return;
    }
    case MFPO_MSG_TLS_SH: {
        /* tls_server_hello_and_certificate::parse tls.h:573 */
        cur p = pkt;
        tls_sh sh; memset(&sh, 0, sizeof sh);
        tls_cert cert; memset(&cert, 0, sizeof cert);
        tls_record rec = tls_record_parse(&p);
        tls_hs hs = tls_hs_parse(&rec.fragment);
        if (hs.msg_type == 2) {
            tls_sh_parse(&sh, &hs.body);
            if (cnotempty(rec.fragment)) {
                tls_hs h2 = tls_hs_parse(&rec.fragment);
                tls_cert_parse(&cert, &h2.body);
            }
        } else if (hs.msg_type == 11) {
            tls_cert_parse(&cert, &hs.body);
        }
        tls_record rec2 = tls_record_parse(&p);
        tls_hs hs2 = tls_hs_parse(&rec2.fragment);
        if (hs2.msg_type == 11) tls_cert_parse(&cert, &hs2.body);
        if (cert.more) r->truncated = 1;
        r->msg = MFPO_MSG_TLS_SH;
        int hello = tls_sh_not_empty(&sh);
        r->emit = hello || cnotempty(cert.list);
        if (hello) {
            fp_set_type(&c->b, &c->type, MFPO_FP_TLS_SERVER);
            tls_sh_fp(&c->b, &sh);
            finish_fp(c);
        }
        return;
    }
    case MFPO_MSG_TLS_CERT: {
        /* tls_certificate::parse tls.h:720 (no fingerprint) */
        cur p = pkt;
        tls_cert cert; memset(&cert, 0, sizeof cert);
        tls_record rec = tls_record_parse(&p);
        tls_hs hs = tls_hs_parse(&rec.fragment);
        if (hs.msg_type == 11) tls_cert_parse(&cert, &hs.body);
        if (cert.more) r->truncated = 1;
        r->msg = MFPO_MSG_TLS_CERT;
        r->emit = cnotempty(cert.list);
        return;
    }
    case MFPO_MSG_SSH_INIT: {
        /* direction tcpip.h:196; selector ssh_direction proto_identify.h:645 */
        int server = !(dport <= sport);
        unsigned need = server ? MFPO_SEL_SSH_SERVER : MFPO_SEL_SSH_CLIENT;
        if (!(sel & need)) return;
        ssh_init s; ssh_init_parse(&s, pkt);
        int kex = s.has_kex && cnotempty(s.kex.nl[0]);
        /* more_bytes_needed ssh.h:464 */
        uint64_t more = kex ? s.bin.more : 8192;
        if (more) r->truncated = 1;
        r->msg = MFPO_MSG_SSH_INIT;
        if (!cnotempty(s.proto)) return;
        r->emit = 1;
        if (kex) fp_set_type(&c->b, &c->type, server ? MFPO_FP_SSH_SERVER : MFPO_FP_SSH);
        else fp_set_type(&c->b, &c->type, server ? MFPO_FP_SSH_INIT_SERVER : MFPO_FP_SSH_INIT);
        ssh_init_fp(&c->b, &s);
        finish_fp(c);
        return;
    }
    case MFPO_MSG_SSH_KEX: {
        int server = !(dport <= sport);
        unsigned need = server ? MFPO_SEL_SSH_SERVER : MFPO_SEL_SSH_CLIENT;
        if (!(sel & need)) return;
        cur p = pkt;
        ssh_bin bin; ssh_bin_parse(&bin, &p);
        if (bin.more) r->truncated = 1;
        ssh_kex k; ssh_kex_parse(&k, bin.payload);
        r->msg = MFPO_MSG_SSH_KEX;
        if (!cnotempty(k.nl[0])) return;
        r->emit = 1;
        fp_set_type(&c->b, &c->type, server ? MFPO_FP_SSH_KEX_SERVER : MFPO_FP_SSH_KEX);
        ssh_kex_fp(&c->b, &k);
        finish_fp(c);
        return;
    }
    }
}

/* set_udp_protocol pkt_proc.cc:677 (selection subset: DTLS) */
static void udp_data(ctx *c, cur pkt) {
    mfpo_result *r = c->res;
    if (!(c->cfg->select & MFPO_SEL_DTLS) || clen(pkt) < 4) return;
    int msg = 0;
    if (matches(pkt, M_DTLS, V_DCH, 16)) msg = MFPO_MSG_DTLS_CH;
    else if (matches(pkt, M_DTLS, V_DSH, 16)) msg = MFPO_MSG_DTLS_SH;
    else if (matches(pkt, M_DTLS, V_DHV, 16)) msg = MFPO_MSG_DTLS_HVR;
    if (!msg) return;
    r->msg = msg;
    /* dtls_record dtls.h:19 + dtls_handshake dtls.h:49 */
    cur d = pkt, frag, body; cset_null(&frag); cset_null(&body);
    uint64_t t, len = 0, foff = 0, flen = 0;
    if (clen(d) < 13) cset_null(&d);
    else { rd_uint(&d, 1, &t); rd_uint(&d, 2, &t); rd_uint(&d, 2, &t); rd_uint(&d, 6, &t); rd_uint(&d, 2, &t); cparse(&frag, &d, (long)t); }
    uint64_t more = 0;
    if (clen(frag) < 12) cset_null(&frag);
    else {
        rd_uint(&frag, 1, &t); rd_uint(&frag, 3, &len); rd_uint(&frag, 2, &t);
        rd_uint(&frag, 3, &foff); rd_uint(&frag, 3, &flen);
        cparse(&body, &frag, (long)flen);
        if (foff == 0) {
            long bl = clen(body);
            if (flen <= len && bl >= 0 && (uint64_t)bl <= len) more = len - (uint64_t)bl;
        }
    }
    if (msg == MFPO_MSG_DTLS_CH) {
        if ((uint32_t)more) r->truncated = 1;
        tls_ch ch; tls_ch_parse(&ch, body);
        if (!cnotempty(ch.compression)) return;
        r->emit = 1;
        fp_set_type(&c->b, &c->type, MFPO_FP_DTLS);
        tls_ch_fp(&c->b, &ch, c->cfg->tls_format);
        tls_sni(ch.extensions, &r->sni_off, &r->sni_len, &r->ua_off, &r->ua_len, c->base);
        finish_fp(c);
    } else if (msg == MFPO_MSG_DTLS_SH) {
        tls_sh sh; memset(&sh, 0, sizeof sh);
        cur b2 = body;
        tls_sh_parse(&sh, &b2);
        if (!tls_sh_not_empty(&sh)) return;
        r->emit = 1;
        fp_set_type(&c->b, &c->type, MFPO_FP_DTLS_SERVER);
        tls_sh_fp(&c->b, &sh);
        finish_fp(c);
    } else {
        /* dtls_hello_verify_request dtls.h:160: valid = body not null after
         * reading version(2), cookie_len(1), cookie */
        cur b2 = body; uint64_t cl;
        rd_uint(&b2, 2, &t); rd_uint(&b2, 1, &cl);
        cur ck; cparse(&ck, &b2, (long)cl);
        r->emit = !cnull(b2);
    }
}

/* ipv4_packet::parse ip.h:124 / ipv6_packet::parse ip.h:448 ; returns
 * transport protocol (255 = none) and sets *iph */
static unsigned ip_parse(cur *p, mfpo_result *r, const uint8_t **iph, int *ipv) {
    unsigned v = look_u8(p);
    *iph = NULL; *ipv = 0;
    if ((v & 0xf0) == 0x40) {
        const uint8_t *h = cget_ptr(p, 20);
        *ipv = 4;
        if (!h) return 255;
        *iph = h;
        long tl = ((long)h[2] << 8) | h[3];
        ctrim_to_length(p, tl - 20);
        if (tl - 20 < 0 && p->d) p->e = p->d + (tl - 20);   /* size_t wrap: negative length */
        r->ip_vers = 4; r->ip_proto = h[9];
        memcpy(r->src_addr, h + 12, 4); memcpy(r->dst_addr, h + 16, 4);
        return h[9];
    }
    if ((v & 0xf0) == 0x60) {
        const uint8_t *h = cget_ptr(p, 40);
        *ipv = 6;
        if (!h) return 255;
        *iph = h;
        ctrim_to_length(p, ((long)h[4] << 8) | h[5]);
        r->ip_vers = 6;
        memcpy(r->src_addr, h + 8, 16); memcpy(r->dst_addr, h + 24, 16);
        unsigned nh = h[6];
        while (clen(*p) > 0) {
            int ext = (nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135 || nh == 139 || nh == 140);
            if (!ext) break;
            unsigned hdr = nh, nnh, hl; cur dd;
            rd_u8(p, &nnh);
            switch (hdr) {
            case 44: cparse(&dd, p, 7); break;
            case 51: rd_u8(p, &hl); cparse(&dd, p, (long)hl * 4 + 6); break;
            default: rd_u8(p, &hl); cparse(&dd, p, (long)hl * 8 + 6); break;
            }
            nh = nnh;
        }
        r->ip_proto = (uint8_t)nh;
        return nh;
    }
    return 255;
}

/* ip_write_json pkt_proc.cc:1063 / analyze_ip_packet pkt_proc.cc:1597 */
static void ip_path(ctx *c, cur pkt) {
    mfpo_result *r = c->res;
    const uint8_t *iph; int ipv;
    unsigned proto = ip_parse(&pkt, r, &iph, &ipv);
    /* encapsulations pkt_proc.cc:959: IP-in-IP (GRE/VXLAN/Geneve need their
     * selectors, which are outside this path's selection set) */
    for (int n = 0; n < 4 && (proto == 4 || proto == 41); n++) {
        proto = ip_parse(&pkt, r, &iph, &ipv);
    }
    if (proto == 6) {
        const uint8_t *tcph = cget_ptr(&pkt, 20);
        if (!tcph) return;                                  /* !is_valid() */
        cur opts; cset_null(&opts);
        cparse(&opts, &pkt, (long)(tcph[12] >> 4) * 4 - 20);
        r->src_port = ((unsigned)tcph[0] << 8) | tcph[1];
        r->dst_port = ((unsigned)tcph[2] << 8) | tcph[3];
        uint8_t fl = tcph[13];
        int syn = (fl & 0x02) != 0, ack = (fl & 0x10) != 0;
        if (c->cfg->mode == MFPO_MODE_WRITE_JSON) {
            if (syn && !ack) {
                if (c->cfg->select & MFPO_SEL_TCP_SYN) {
                    r->msg = MFPO_MSG_TCP_SYN; r->emit = 1;
                    fp_set_type(&c->b, &c->type, MFPO_FP_TCP);
                    tcp_syn_fp(&c->b, ipv, iph, tcph, opts);
                    finish_fp(c);
                }
                return;
            }
            if (syn && ack) {
                if ((c->cfg->select & MFPO_SEL_TCP_SYN) && (c->cfg->select & MFPO_SEL_TCP_SYNACK)) {
                    r->msg = MFPO_MSG_TCP_SYNACK; r->emit = 1;
                    fp_set_type(&c->b, &c->type, MFPO_FP_TCP_SERVER);
                    tcp_syn_fp(&c->b, ipv, iph, tcph, opts);
                    finish_fp(c);
                }
                return;
            }
            if (clen(pkt) == 0) return;                     /* process_tcp_data: !data_length */
        }
        tcp_data(c, pkt, tcph);
    } else if (proto == 17) {
        const uint8_t *udph = cget_ptr(&pkt, 8);
        if (udph) {
            r->src_port = ((unsigned)udph[0] << 8) | udph[1];
            r->dst_port = ((unsigned)udph[2] << 8) | udph[3];
        }
        udp_data(c, pkt);
    }
}

/* eth::eth eth.h:137 ; returns ethertype */
static unsigned eth_parse(cur *p) {
    uint64_t et;
    cskip(p, 12);
    if (!rd_uint(p, 2, &et)) return 0;
    if (et < 0x600) {
        static const uint8_t cdp[] = { 0xaa, 0xaa, 0x03, 0x00, 0x00, 0x0c, 0x20, 0x00 };
        (void)cdp;  /* CDP: not IP, irrelevant to this path */
    }
    if (et == 0x88a8) { cskip(p, 2); if (!rd_uint(p, 2, &et)) return 0; }
    while (et == 0x8100) { cskip(p, 2); if (!rd_uint(p, 2, &et)) return 0; }
    if (et == 0x8847) {
        uint64_t lbl = 0;
        while (!(lbl & 0x100)) { if (!rd_uint(p, 4, &lbl)) return 0; }
        et = 0x0800;
    }
    if (et == 0x8909) { cskip(p, 6); if (!rd_uint(p, 2, &et)) return 0; }
    return (unsigned)et;
}
/* ppp::is_ip ppp.h:76 */
static int ppp_is_ip(cur *p) {
    unsigned b = look_u8(p);
    if (b == 0x7e) {
        unsigned t; rd_u8(p, &t);
        b = look_u8(p);
        if (b == 0xff) { rd_u8(p, &t); rd_u8(p, &t); }
    } else if (b == 0xff) {
        unsigned t; rd_u8(p, &t); rd_u8(p, &t);
    }
    unsigned proto;
    b = look_u8(p);
    if (b & 1) { if (!rd_u8(p, &b)) proto = 0; else proto = b; }
    else { unsigned x, v = 0; for (int i = 0; i < 2; i++) { v *= 256; rd_u8(p, &x); v += x; } proto = v; }
    return proto == 0x21 || proto == 0x57;
}

int mfpo_process(const uint8_t *data, size_t len, uint16_t linktype, const mfpo_config *cfg, mfpo_result *res) {
    memset(res, 0, offsetof(mfpo_result, fp));
    res->fp[0] = 0;
    res->sni_off = res->ua_off = -1;
    ctx c; c.cfg = cfg; c.res = res; c.b.buf = res->fp; c.b.off = 0; c.b.trunc = 0; c.type = 0; c.base = data;
    cur p = { data, data + len };
    switch (linktype) {
    case 1: {                                             /* write_json pkt_proc.cc:1258 */
        unsigned et = eth_parse(&p);
        if (et == 0x0800 || et == 0x86dd) break;
        if (et == 0x8864) {
            cur t; cparse(&t, &p, 1); cparse(&t, &p, 1); cparse(&t, &p, 2); cparse(&t, &p, 2);
            if (!ppp_is_ip(&p)) return 0;
            break;
        }
        return 0;
    }
    case 9:                                               /* LINKTYPE_PPP */
        if (!ppp_is_ip(&p)) return 0;
        break;
    case 101:                                             /* LINKTYPE_RAW */
        break;
    case 113: {                                           /* linux_sll linux_sll.hpp */
        uint64_t pt, ar, al, pr; cur lla;
        rd_uint(&p, 2, &pt); rd_uint(&p, 2, &ar); rd_uint(&p, 2, &al); cparse(&lla, &p, 8); rd_uint(&p, 2, &pr);
        if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return 0;
        break;
    }
    case 276: {                                           /* linux_sll2 linux_sll2.hpp */
        uint64_t pr, t, ar; cur lla;
        rd_uint(&p, 2, &pr); rd_uint(&p, 2, &t); rd_uint(&p, 4, &t); rd_uint(&p, 2, &ar);
        rd_uint(&p, 1, &t); rd_uint(&p, 1, &t); cparse(&lla, &p, 8);
        if (cnull(p) || !((ar == 1 || ar == 772) && (pr == 0x0800 || pr == 0x86dd))) return 0;
        break;
    }
    case 0: {                                             /* LINKTYPE_NULL loopback.hpp */
        if (cfg->mode != MFPO_MODE_WRITE_JSON) return 0;  /* analyze_packet has no NULL case */
        uint64_t v; rd_uint(&p, 4, &v);
        if (!cnull(p)) {
            if (!(v == 2 || v == 0x02000000 || v == 24 || v == 0x18000000 || v == 28 || v == 0x1c000000 ||
                  v == 30 || v == 0x1e000000)) return 0;
        }
        break;
    }
    default:
        return 0;
    }
    if (cnull(p)) return 0;
    ip_path(&c, p);
    return (int)res->fp_type;
}

long long mfpo_process_batch(const uint8_t *arena, const mfpo_desc *desc, size_t n, const mfpo_config *cfg,
                             uint8_t *fp_type, uint32_t *fp_len, uint8_t *flags, uint64_t *fp_off,
                             char *fp_arena, size_t fp_cap) {
    mfpo_result *r = malloc(sizeof *r);
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        mfpo_process(arena + desc[i].offset, desc[i].caplen, desc[i].linktype, cfg, r);
        fp_type[i] = (uint8_t)r->fp_type;
        fp_len[i] = r->fp_len;
        flags[i] = (uint8_t)((r->emit ? 1 : 0) | (r->truncated ? 2 : 0));
        fp_off[i] = off;
        if (off + r->fp_len > fp_cap) { free(r); return -1; }
        memcpy(fp_arena + off, r->fp, r->fp_len);
        off += r->fp_len;
    }
    free(r);
    return (long long)off;
}

typedef struct {
    const uint8_t *arena; const mfpo_desc *desc; size_t lo, hi; const mfpo_config *cfg; int reps;
    unsigned long long bytes;
} worker_arg;

static void *worker(void *a_) {
    worker_arg *a = a_;
    mfpo_result *r = malloc(sizeof *r);
    unsigned long long bytes = 0;
    for (int k = 0; k < a->reps; k++)
        for (size_t i = a->lo; i < a->hi; i++) {
            mfpo_process(a->arena + a->desc[i].offset, a->desc[i].caplen, a->desc[i].linktype, a->cfg, r);
            bytes += r->fp_len;
        }
    a->bytes = bytes;
    free(r);
    return NULL;
}

double mfpo_time_batch(const uint8_t *arena, const mfpo_desc *desc, size_t n, const mfpo_config *cfg,
                       int threads, int reps, unsigned long long *fp_bytes_out) {
    if (threads < 1) threads = 1;
    pthread_t *th = malloc(sizeof(pthread_t) * threads);
    worker_arg *args = malloc(sizeof(worker_arg) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        args[t].arena = arena; args[t].desc = desc; args[t].cfg = cfg; args[t].reps = reps;
        args[t].lo = n * t / threads; args[t].hi = n * (t + 1) / threads; args[t].bytes = 0;
        pthread_create(&th[t], NULL, worker, &args[t]);
    }
    unsigned long long tot = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); tot += args[t].bytes; }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (fp_bytes_out) *fp_bytes_out = tot;
    free(th); free(args);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
