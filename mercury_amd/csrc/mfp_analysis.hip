// mfp_analysis.hip -- the --analysis process classifier on gfx950.
//
// k_analyze: one wavefront per classified packet (grid-stride over groups of
// 64 fingerprint records; a ballot picks the records whose fingerprint type
// the resource archive covers, classifier::analyze_fingerprint_and_
// destination_context analysis.h:1141-1172):
//   1. the fingerprint string is hashed lane-parallel (one 8-byte word per
//      lane, XOR of position-salted mixes, mfp_common.hpp) and looked up in
//      the open-addressing fingerprint table; the match is verified byte for
//      byte (fpdb.find, analysis.h:1043-1083);
//   2. destination context (destination_context::init result.h:346): server
//      name (TLS SNI / HTTP Host) normalised exactly as server_identifier
//      (watchlist.hpp:242-390), its top-two-label domain, user agent, dst
//      port and address from the flow key; ASN by LPM over disjoint address
//      intervals (subnet_data::get_asn_info addr.cc:172-208);
//   3. lane i holds process i's score: prior + the six feature updates in
//      the reference's order (naive_bayes_tls_quic_http::classify
//      naive_bayes.hpp:752-772) -- fp64, same addition order per process;
//   4. max / second max with the reference's first-index tie rule, softmax
//      with expf in fp32 (softmax.hpp:227-264), malware probability, the
//      "generic dmz process" swap and normalisation
//      (compute_score_and_probability / get_analysis_result analysis.h:222-358),
//      encrypted_channel attribute (analysis.h:1161-1163).
// Unknown TLS fingerprints follow fingerprint_prevalence (analysis.h:362-421):
// the known set is a device table; the adaptive set, an LRU of 100000
// fingerprints, is decided on the host in stream order (mfp_prevalence.cpp)
// from this batch's sightings per distinct fingerprint (a batch-local device
// table), and k_analyze_resolve applies the decisions.
#include <hip/hip_runtime.h>

#include "mfp_analysis.h"
#include "mfp_common.hpp"
#include "mfp_internal.h"

namespace mfpa {

#define ADEV __device__ __forceinline__
using namespace mfpc;

constexpr int MAXP_CHUNKS = 8;     // up to 512 processes per fingerprint in k_analyze_wave
constexpr int MAXP_CHUNKS_BIG = 64; // up to 4096 in k_analyze_big

ADEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
ADEV uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
ADEV uint64_t rfl64(uint64_t v) { return (uint64_t)rfl((uint32_t)v) | ((uint64_t)rfl((uint32_t)(v >> 32)) << 32); }
ADEV uint64_t xor_all(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { lo ^= __shfl_xor(lo, d, 64); hi ^= __shfl_xor(hi, d, 64); }
    return rfl64((uint64_t)hi << 32 | lo);
}
ADEV double sum_all(double v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// lane-parallel hash / compare of byte strings (global or LDS)
ADEV uint64_t wave_hash(const uint8_t *s, uint32_t len, uint32_t lane) {
    uint64_t acc = 0;
    for (uint32_t j = lane; 8 * j < len; j += 64) acc ^= word_term(load_word(s, len, j), j);
    return hash_final(xor_all(acc), len);
}
ADEV bool wave_eq(const uint8_t *a, const uint8_t *b, uint32_t len, uint32_t lane) {
    bool bad = false;
    for (uint32_t j = lane; j < len; j += 64) bad |= a[j] != b[j];
    return __ballot(bad) == 0;
}

ADEV uint32_t probe_string(const mfp_fp_slot *slots, uint64_t mask, const char *pool, const uint8_t *s, uint32_t len,
                           uint64_t h, uint32_t lane) {
    for (uint64_t k = h & mask;; k = (k + 1) & mask) {
        const mfp_fp_slot sl = slots[k];
        const uint32_t id = rfl(sl.id);
        if (id == 0xffffffffu) return 0xffffffffu;
        if (rfl64(sl.hash) == h && rfl(sl.str_len) == len && wave_eq(s, (const uint8_t *)pool + rfl(sl.str_off), len, lane))
            return id;
    }
}

struct Hit { uint32_t off, cnt; };
// an entry's region of the feature table (mfp_entry::feat_base / feat_mask)
struct FeatRegion { uint32_t base, mask; };
ADEV FeatRegion feat_region(const mfp_entry &E) { return FeatRegion{E.feat_base, E.feat_mask}; }
ADEV Hit probe_feature(const mfp_classifier_dev &D, FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key,
                       const uint8_t *s, uint32_t len, bool verify, uint32_t lane) {
    for (uint32_t k = (uint32_t)feat_slot_hash(entry, kind, key) & R.mask;; k = (k + 1) & R.mask) {
        const mfp_feat_slot sl = D.feat_slots[R.base + k];
        const uint32_t e = rfl(sl.entry);
        if (e == 0xffffffffu) return Hit{0, 0};
        if (e == entry && rfl(sl.kind) == kind && rfl64(sl.key) == key) {
            if (!verify || (rfl(sl.str_len) == len && wave_eq(s, (const uint8_t *)D.pool + rfl(sl.str_off), len, lane)))
                return Hit{rfl(sl.upd_off), rfl(sl.upd_cnt)};
        }
    }
}

// apply one feature's update list to the per-lane scores
ADEV void apply(const mfp_classifier_dev &D, Hit h, double (&sc)[MAXP_CHUNKS], uint32_t lane) {
    const uint32_t cnt = h.cnt & ~MFP_UPD_SERIAL;   // applied in list order either way
    for (uint32_t u = 0; u < cnt; u++) {
        const mfp_update up = D.upd[h.off + u];
        const uint32_t idx = rfl(up.idx);
        const double v = __hiloint2double((int)rfl((uint32_t)(__double_as_longlong(up.value) >> 32)),
                                          (int)rfl((uint32_t)__double_as_longlong(up.value)));
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++)
            if ((idx >> 6) == (uint32_t)c && (idx & 63) == lane) sc[c] += v;
    }
}

// ---------------------------------------------------------------------------
// lane-serial helpers: one packet per lane (phase A of k_analyze)
// ---------------------------------------------------------------------------
// little-endian 8-byte word j of s[0, len) (bytes past len read as 0) from
// aligned 8-byte loads; never reads the aligned word after the last byte
ADEV uint64_t word_at(const uint8_t *s, uint32_t len, uint32_t j) {
    const uintptr_t p = (uintptr_t)s + 8u * j;
    const uint32_t rem = len - 8u * j;                 // >= 1
    const uintptr_t a = p & ~(uintptr_t)7;
    const uint32_t sh = (uint32_t)(p & 7) * 8u;
    uint64_t w = *(const uint64_t *)a;
    if (sh) {
        w >>= sh;
        if (p + (rem < 8 ? rem : 8) > a + 8) w |= *(const uint64_t *)(a + 8) << (64 - sh);
    }
    if (rem < 8) w &= (1ull << (8 * rem)) - 1;
    return w;
}

// string-relative 8-byte words j0 .. j0+B-1 of s[0, len) (bytes past len read
// as 0), from B+1 aligned 8-byte loads issued together: one memory round
// trip per 8*B bytes; never reads an aligned word past the last byte
template <int B>
ADEV void load_words(const uint8_t *s, uint32_t len, uint32_t j0, uint64_t (&w)[B]) {
    const uintptr_t base = (uintptr_t)s & ~(uintptr_t)7;
    const uint32_t sh = (uint32_t)((uintptr_t)s & 7) * 8;
    const uintptr_t end = (uintptr_t)s + len;
    uint64_t a[B + 1];
#pragma unroll
    for (int k = 0; k <= B; k++) {
        const uintptr_t p = base + 8 * (uintptr_t)(j0 + k);
        a[k] = p < end ? *(const uint64_t *)p : 0;
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
        uint64_t x = sh ? (a[k] >> sh) | (a[k + 1] << (64 - sh)) : a[k];
        const uint32_t pos = 8 * (j0 + k);
        if (pos >= len) x = 0;
        else if (len - pos < 8) x &= (1ull << (8 * (len - pos))) - 1;
        w[k] = x;
    }
}
constexpr int LB = 4;   // words per batch (8: more registers than the classifier kernels can spare)

// mfpc::str_hash, one lane
ADEV uint64_t lane_hash(const uint8_t *s, uint32_t len) {
    uint64_t acc = 0;
    for (uint32_t j0 = 0; 8 * j0 < len; j0 += LB) {
        uint64_t w[LB];
        load_words<LB>(s, len, j0, w);
#pragma unroll
        for (int k = 0; k < LB; k++)
            if (8 * (j0 + k) < len) acc ^= word_term(w[k], j0 + k);
    }
    return hash_final(acc, len);
}

// the fingerprint's str_hash: stored after the string by the fingerprint
// kernels (MFP_FLAG_HASHED, one 8-byte load) or computed here
ADEV uint64_t fp_key(const mfp_record &r, const uint8_t *fp, uint32_t len) {
    if (r.flags & MFP_FLAG_HASHED) return *(const uint64_t *)(fp + ((len + 7) & ~7u));
    return lane_hash(fp, len);
}

// B words of each string per round trip (B = 4 where registers are short)
template <int B = LB>
ADEV bool lane_eq(const uint8_t *a, const uint8_t *b, uint32_t len) {
    for (uint32_t j0 = 0; 8 * j0 < len; j0 += B) {
        uint64_t x[B], y[B];
        load_words<B>(a, len, j0, x);
        load_words<B>(b, len, j0, y);
        bool same = true;
#pragma unroll
        for (int k = 0; k < B; k++) same &= x[k] == y[k];
        if (!same) return false;
    }
    return true;
}

// C-string view of s[0, n) (strncpy into the destination context stops at a
// NUL): its length, and its str_hash
ADEV uint32_t cstr_hash(const uint8_t *s, uint32_t n, uint64_t &h) {
    uint64_t acc = 0;
    for (uint32_t j0 = 0; 8 * j0 < n; j0 += LB) {
        uint64_t w[LB];
        load_words<LB>(s, n, j0, w);
#pragma unroll
        for (int k = 0; k < LB; k++) {
            const uint32_t pos = 8 * (j0 + k);
            if (pos < n) {
                uint64_t v = w[k];
                if (n - pos < 8) v |= ~0ull << (8 * (n - pos));   // bytes past n are not NUL
                const uint64_t z = (v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull;
                if (z) {   // a NUL inside: the C string is shorter (rare)
                    const uint32_t m = pos + (uint32_t)(__builtin_ctzll(z) >> 3);
                    h = lane_hash(s, m);
                    return m;
                }
                acc ^= word_term(w[k], j0 + k);
            }
        }
    }
    h = hash_final(acc, n);
    return n;
}

ADEV uint32_t probe_string_lane(const mfp_fp_slot *slots, uint64_t mask, const char *pool, const uint8_t *s,
                                uint32_t len, uint64_t h) {
    for (uint64_t k = h & mask;; k = (k + 1) & mask) {
        const mfp_fp_slot sl = slots[k];
        if (sl.id == 0xffffffffu) return 0xffffffffu;
#ifdef MFP_PROBE_AN_NOVERIFY
        if (sl.hash == h && sl.str_len == len) return sl.id;
#else
        if (sl.hash == h && sl.str_len == len && lane_eq(s, (const uint8_t *)pool + sl.str_off, len)) return sl.id;
#endif
    }
}

// first slot whose hash and length match (no byte comparison): the
// candidate that wave_verify then checks; ~0u when the probe hits an empty slot
ADEV uint32_t cand_string_lane(const mfp_fp_slot *slots, uint64_t mask, uint64_t h, uint32_t len, uint32_t &str_off) {
    for (uint64_t k = h & mask;; k = (k + 1) & mask) {
        const mfp_fp_slot sl = slots[k];
        if (sl.id == 0xffffffffu) return 0xffffffffu;
        if (sl.hash == h && sl.str_len == len) { str_off = sl.str_off; return sl.id; }
    }
}
ADEV bool cand_feature_lane(const mfp_classifier_dev &D, FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key,
                            uint32_t len, Hit &hit, uint32_t &str_off) {
    for (uint32_t k = (uint32_t)feat_slot_hash(entry, kind, key) & R.mask;; k = (k + 1) & R.mask) {
        const mfp_feat_slot sl = D.feat_slots[R.base + k];
        if (sl.entry == 0xffffffffu) return false;
        if (sl.entry == entry && sl.kind == kind && sl.key == key && sl.str_len == len) {
            hit = Hit{sl.upd_off, sl.upd_cnt};
            str_off = sl.str_off;
            return true;
        }
    }
}

ADEV uint64_t rl64(uint64_t v, int j) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j) << 32);
}

// Byte-exact comparison of a[0, len) with b[0, len) for every lane with
// `has`, done by the whole wave one string (up to four at a time) after the
// other: lane k compares word k, so each string is read with coalesced loads
// instead of a lane walking its own string.  Returns false on lanes whose
// strings differ (true on lanes without `has`).
ADEV bool wave_verify(bool has, const uint8_t *a, const uint8_t *b, uint32_t len, uint32_t lane) {
#ifdef MFP_PROBE_AN_NOVERIFY
    return true;
#endif
    bool ok = true;
    uint64_t m = __ballot(has);
    while (m) {
        int js[4];
        int nj = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            js[t] = 0;
            if (m) { js[t] = (int)__builtin_ctzll(m); m &= m - 1; nj = t + 1; }
        }
        bool bad[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            bad[t] = false;
            if (t < nj) {
                const uint8_t *aj = (const uint8_t *)rl64((uint64_t)a, js[t]);
                const uint8_t *bj = (const uint8_t *)rl64((uint64_t)b, js[t]);
                const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)len, js[t]);
                for (uint32_t k = lane; 8 * k < lj; k += 64) bad[t] |= word_at(aj, lj, k) != word_at(bj, lj, k);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (t < nj && __ballot(bad[t]) && (int)lane == js[t]) ok = false;
    }
    return ok;
}

// feature slot of (entry, kind, key); s/len: the string to verify (len ==
// ~0u: integer key, nothing to verify)
ADEV Hit probe_feature_lane(const mfp_classifier_dev &D, FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key,
                            const uint8_t *s, uint32_t len) {
    for (uint32_t k = (uint32_t)feat_slot_hash(entry, kind, key) & R.mask;; k = (k + 1) & R.mask) {
        const mfp_feat_slot sl = D.feat_slots[R.base + k];
        if (sl.entry == 0xffffffffu) return Hit{0, 0};
        if (sl.entry == entry && sl.kind == kind && sl.key == key &&
#ifdef MFP_PROBE_AN_NOVERIFY
            (len == 0xffffffffu || sl.str_len == len))
#else
            (len == 0xffffffffu || (sl.str_len == len && lane_eq(s, (const uint8_t *)D.pool + sl.str_off, len))))
#endif
            return Hit{sl.upd_off, sl.upd_cnt};
    }
}

// The same probes started from their home slot, loaded beforehand: the
// kernel issues the home-slot loads of all its lookups together (one memory
// round trip instead of one per lookup); a probe that does not end at its
// home slot walks on from there
ADEV uint32_t home_slot(FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key) {
    return (uint32_t)feat_slot_hash(entry, kind, key) & R.mask;
}
ADEV mfp_feat_slot empty_slot() {
    mfp_feat_slot s;
    s.key = 0; s.entry = 0xffffffffu; s.kind = 0; s.upd_off = 0; s.upd_cnt = 0; s.str_off = 0; s.str_len = 0;
    return s;
}
ADEV Hit probe_int_from(const mfp_classifier_dev &D, FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key,
                        uint32_t k, mfp_feat_slot sl) {
    for (;;) {
        if (sl.entry == 0xffffffffu) return Hit{0, 0};
        if (sl.entry == entry && sl.kind == kind && sl.key == key) return Hit{sl.upd_off, sl.upd_cnt};
        k = (k + 1) & R.mask;
        sl = D.feat_slots[R.base + k];
    }
}
ADEV bool cand_from(const mfp_classifier_dev &D, FeatRegion R, uint32_t entry, uint32_t kind, uint64_t key,
                    uint32_t len, uint32_t k, mfp_feat_slot sl, Hit &hit, uint32_t &str_off) {
    for (;;) {
        if (sl.entry == 0xffffffffu) return false;
        if (sl.entry == entry && sl.kind == kind && sl.key == key && sl.str_len == len) {
            hit = Hit{sl.upd_off, sl.upd_cnt};
            str_off = sl.str_off;
            return true;
        }
        k = (k + 1) & R.mask;
        sl = D.feat_slots[R.base + k];
    }
}

// subnet_data::get_asn_info (addr.cc:172-208): lct_find on the reference's
// tries (mfp_lctrie.hpp), the subnet's ASN or 0
ADEV uint32_t asn_v4_lane(const mfp_classifier_dev &D, uint32_t addr_host) {
    if (!D.n_asn4) return 0;
    const uint32_t s = lct_find4(D.asn4_node, D.asn4_net, addr_host);
    return s == MFP_LCT_NIL ? 0 : D.asn4_net[s].val;
}
ADEV uint32_t asn_v6_lane(const mfp_classifier_dev &D, uint64_t xh, uint64_t xl) {
    if (!D.n_asn6) return 0;
    const uint32_t s = lct_find6(D.asn6_node, D.asn6_net, xh, xl);
    return s == MFP_LCT_NIL ? 0 : D.asn6_net[s].val;
}

// ---------------------------------------------------------------------------
// classifier-agnostic attributes (check_additional_attributes_util
// analysis.h:555-570, tls_client_hello::do_analysis tls.h:1977-1996)
// ---------------------------------------------------------------------------
// the destination as the reference reads it back from dst_ip_str
struct Dst {
    uint32_t ipv;        // 4, 6, or 0
    uint32_t v4;         // address bytes in packet order (ipv4_address_string value)
    uint64_t hi, lo;     // IPv6 as big-endian halves, after the text round trip
};

ADEV Dst dst_of(const uint8_t *pkt, uint32_t net) {
    Dst d;
    d.ipv = (net >> 16) & 15;
    d.v4 = 0; d.hi = 0; d.lo = 0;
    const uint32_t ipo = net & 0xffff;
    if (d.ipv == 4) {
        d.v4 = (uint32_t)word_at(pkt + ipo + 16, 4, 0);
    } else if (d.ipv == 6) {
        d.hi = __builtin_bswap64(word_at(pkt + ipo + 24, 16, 0));
        d.lo = __builtin_bswap64(word_at(pkt + ipo + 24, 16, 1));
        v6_text_roundtrip(d.hi, d.lo);
    }
    return d;
}

// watchlist::contains (dns name) || watchlist::contains_addr (watchlist.hpp:574-599)
ADEV bool doh_hit(const mfp_classifier_dev &D, const uint8_t *sn, uint32_t cl, uint64_t ch, const Dst &d) {
    if (probe_string_lane(D.doh_names, D.doh_names_mask, D.pool, sn, cl, ch) != 0xffffffffu) return true;
    if (d.ipv == 4) {
        int lo = 0, hi = (int)D.n_doh_v4 - 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            const uint32_t v = D.doh_v4[mid];
            if (v == d.v4) return true;
            if (v < d.v4) lo = mid + 1; else hi = mid - 1;
        }
    } else if (d.ipv == 6) {
        int lo = 0, hi = (int)D.n_doh_v6 - 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            const uint64_t a = D.doh_v6[2 * mid], b = D.doh_v6[2 * mid + 1];
            if (a == d.hi && b == d.lo) return true;
            if (a < d.hi || (a == d.hi && b < d.lo)) lo = mid + 1; else hi = mid - 1;
        }
    }
    return false;
}

// subnet_data::is_domain_faking (addr.cc:707-792): a mapped domain (a leading
// "www." dropped) whose public destination is not in one of its prefixes nor
// in an exception prefix
ADEV bool domain_faking(const mfp_classifier_dev &D, const uint8_t *sn, uint32_t cl, const Dst &d) {
    const bool www = cl >= 4 && sn[0] == 'w' && sn[1] == 'w' && sn[2] == 'w' && sn[3] == '.';
    const uint8_t *nm = www ? sn + 4 : sn;
    const uint32_t nl = www ? cl - 4 : cl;
    const uint32_t didx = probe_string_lane(D.dom_slots, D.dom_mask, D.pool, nm, nl, lane_hash(nm, nl));
    if (didx == 0xffffffffu) return false;
    uint32_t info = 0;
    if (d.ipv == 4) {
        const uint32_t v = d.v4;   // ipv4_address::get_addr_type private_use (ip_address.hpp:119-123)
        if ((v & 0xff) == 0x0a || (v & 0xf0ff) == 0x10ac || (v & 0xffff) == 0xa8c0) return false;
        if (!D.n_dom4) return true;    // no IPv4 mappings: nothing holds it
        const uint32_t sub = lct_find4(D.dom4_node, D.dom4_net, __builtin_bswap32(v));
        if (sub != MFP_LCT_NIL) info = D.dom4_net[sub].val;
    } else if (d.ipv == 6 && D.n_dom6) {
        // is_private_address (ipv6_lctrie.h:255): the first byte in memory of
        // the host-order high half, i.e. address byte 7
        if ((d.hi & 0xff) == 0xfc || (d.hi & 0xff) == 0xfd) return false;
        const uint32_t sub = lct_find6(D.dom6_node, D.dom6_net, d.hi, d.lo);
        if (sub != MFP_LCT_NIL) info = D.dom6_net[sub].val;
    } else {
        return false;
    }
    if (info == 0) return true;                    // no prefix holds the destination
    const uint32_t ty = D.dom_info[2 * (info - 1)], off = D.dom_info[2 * (info - 1) + 1];
    if ((ty & 0xff) == MFP_DOM_EXCEPTION) return false;
    for (uint32_t k = 0; k < (ty >> 8); k++)
        if ((uint32_t)D.dom_bytes[off + k] == didx) return false;   // uint8_t entry vs uint32_t index
    return true;
}

// is_faketls_util (tls.h:923-949) on the fingerprint string: its second
// parenthesised group is the ClientHello's cipher suites, degreased, as hex
// (raw_as_hex_degrease tls.h:802-813); faketls when none is in the IANA list
// or the exception list (no suites at all included)
__constant__ uint16_t kCipherRanges[][2] = {
#include "mfp_cipher_ranges.inc"
};
ADEV bool faketls_fp(const uint8_t *fp, uint32_t len) {
    uint32_t p = 0;
    while (p < len && fp[p] != ')') p++;
    p += 2;                                        // ")("
    for (; p + 4 <= len && fp[p] != ')'; p += 4) {
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            const uint32_t c = fp[p + k];
            v = v << 4 | (c <= '9' ? c - '0' : c - 'a' + 10);
        }
        for (uint32_t r = 0; r < sizeof(kCipherRanges) / sizeof(kCipherRanges[0]); r++)
            if (v >= kCipherRanges[r][0] && v <= kCipherRanges[r][1]) return false;
    }
    return true;
}

// A server name that server_identifier::get_normalized_domain_name leaves
// unchanged (watchlist.hpp:326-390): 1..256 bytes of label characters and
// dots, no empty label, at least two labels, the last one with a letter.
// Such a name is no IPv6 literal (a dot ends the hex run), a dns_string
// consuming every byte, neither "None" nor "localhost" and not unqualified,
// so the normalized name is the input itself.  *tld: offset of the top two
// labels (get_tld_domain_name, naive_bayes.hpp:557).  Anything else takes the
// wave path (normalize_server_name, mfp_common.hpp).
ADEV uint64_t swar_eq8(uint64_t w, uint32_t c) {
    const uint64_t x = w ^ (0x0101010101010101ull * (c & 0xff));
    return ~(((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x) & 0x8080808080808080ull;
}
ADEV uint64_t swar_range8(uint64_t w, uint32_t lo, uint32_t hi) {   // lo <= byte <= hi (ASCII, hi < 0x80)
    const uint64_t x = w & 0x7f7f7f7f7f7f7f7full;
    const uint64_t ge = x + 0x0101010101010101ull * (0x80 - lo);
    const uint64_t gt = x + 0x0101010101010101ull * (0x7f - hi);
    return ge & ~gt & ~w & 0x8080808080808080ull;
}
ADEV bool plain_server_name(const uint8_t *s, uint32_t n, uint32_t &tld, uint64_t &h) {
    // word at a time (SWAR byte classes, bit 7 of each byte flags it)
    if (n == 0 || n > 256) return false;
    int last_dot = -1, prev_dot = -1;
    bool ok = true, alpha_last = false, prev_is_dot = true;   // a leading dot is an empty label
    uint64_t acc = 0;
    for (uint32_t j0 = 0; 8 * j0 < n; j0 += LB) {
        uint64_t w[LB];
        load_words<LB>(s, n, j0, w);
#pragma unroll
        for (int q = 0; q < LB; q++) {
            const uint32_t pos = 8 * (j0 + q);
            if (pos < n) {
                acc ^= word_term(w[q], j0 + q);
                const uint64_t valid = n - pos >= 8 ? 0x8080808080808080ull : (0x8080808080808080ull >> (8 * (8 - (n - pos))));
                const uint64_t x = w[q];
                const uint64_t dot = swar_eq8(x, '.') & valid;
                const uint64_t alpha = (swar_range8(x, 'a', 'z') | swar_range8(x, 'A', 'Z')) & valid;
                const uint64_t label = alpha | swar_range8(x, '0', '9') | swar_eq8(x, '-') | swar_eq8(x, '_');
                ok &= ((label & valid) | dot) == valid;
                // empty label: a dot right after a dot (or at the start)
                ok &= (dot & ((dot << 8) | (prev_is_dot ? 0x80ull : 0ull))) == 0;
                if (dot) {
                    const int hi = 63 - __builtin_clzll(dot);
                    const uint64_t rest = dot & ~(1ull << hi);
                    prev_dot = rest ? (int)pos + ((63 - __builtin_clzll(rest)) >> 3) : last_dot;
                    last_dot = (int)pos + (hi >> 3);
                    alpha_last = (alpha >> hi) != 0;       // letters after this word's last dot
                } else {
                    alpha_last |= alpha != 0;
                }
                const uint32_t top = (n - pos >= 8 ? 8 : n - pos) * 8 - 1;   // bit 7 of the word's last byte
                prev_is_dot = (dot >> top) & 1;
            }
        }
    }
    ok &= !prev_is_dot && last_dot >= 0 && alpha_last;
    tld = (uint32_t)(prev_dot + 1);
    h = hash_final(acc, n);
    return ok;
}

// ---------------------------------------------------------------------------
// expf as the reference computes it: the softmax calls the C library's expf
// (softmax.hpp:252); on x86-64 glibc resolves it to its FMA build of the
// table method -- x*32/ln2 = k + r, 2^(k/32) from a 32-entry table of
// 2^(i/32), a cubic in r, all in double, one rounding to float at the end.
// Restated here with the same operations and the same fused multiply-adds
// (the table holds round-to-nearest 2^(i/32), minus i << 47), so the
// probabilities are bit-identical to the reference's; checked against the
// host's expf on every float in [-110, 0] (the softmax only takes x <= 0).
// ---------------------------------------------------------------------------
__constant__ uint64_t kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
ADEV float expf_ref(float x) {
#pragma clang fp contract(off)
    const uint32_t ux = __float_as_uint(x);
    const uint32_t abstop = (ux >> 20) & 0x7ff;
    if (abstop >= 0x42b) {                              // |x| >= 88 or NaN
        if (ux == 0xff800000u) return 0.0f;             // -inf
        if (abstop >= 0x7f8) return x + x;              // +inf, NaN
        if (x > 0x1.62e42ep6f) return __uint_as_float(0x7f800000u);   // overflow
        if (x < -0x1.9fe368p6f) return 0.0f;            // underflow
    }
    const double inv_ln2_n = 0x1.71547652b82fep+0 * 32, shift = 0x1.8p+52;
    const double c0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, c1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                 c2 = 0x1.62e42ff0c52d6p-1 / 32;
    const double xd = (double)x;
    const double z = inv_ln2_n * xd;
    double kd = z + shift;
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= shift;
    const double r = __builtin_fma(inv_ln2_n, xd, -kd);
    const uint64_t t = kExp2Tab[ki & 31] + (ki << 47);
    const double s = __longlong_as_double((long long)t);
    const double zz = __builtin_fma(c0, r, c1);
    const double r2 = r * r;
    double y = __builtin_fma(c2, r, 1.0);
    y = __builtin_fma(zz, r2, y);
    y = y * s;
    return (float)y;
}

// a packet k_analyze hands to k_analyze_wave, with its feature lookups done
// a packet to score, with its feature lookups done (k_an_features -> k_an_score /
// k_analyze_wave): slow_sni: domain / SNI lookups still to do (the wave path
// normalises the name); slow_ua: the SSH user agent; xattr: encrypted_dns,
// domain_faking, faketls bits found by k_an_features
struct Deferred {
    uint32_t i, entry, slow_sni, slow_ua;
    uint32_t off[6], cnt[6];
};
// a packet k_an_features hands to the wave scorers (k_analyze_wave /
// k_analyze_big): the Deferred fields plus what the scorer would otherwise
// fetch first (its fingerprint entry, the fingerprint type), so one load of
// these 20 words -- lane k holds word k -- starts a packet
struct WItem {
    uint32_t i, entry, flags, ft;   // flags: bit 0 slow server name, bit 1 SSH user agent, xattr << 16
    uint32_t po, np, mdb, dmz;      // mfp_entry: proc_off, nproc, malware_db, generic_dmz
    uint32_t off[6], cnt[6];
};
constexpr uint32_t WITEM_WORDS = sizeof(WItem) / 4;
static_assert(WITEM_WORDS == 20, "WItem layout");
enum : uint32_t { WI_I = 0, WI_ENTRY = 1, WI_FLAGS = 2, WI_FT = 3, WI_PO = 4, WI_NP = 5, WI_MDB = 6, WI_DMZ = 7,
                  WI_OFF = 8, WI_CNT = 14 };
// a packet k_analyze hands to k_an_features: its fingerprint entry (~0u: none)
// and what to do (WK_SCORE, WK_XCHECK, WK_PENDING)
struct WorkItem { uint32_t i, entry, flags, pad; };
enum { WK_SCORE = 1, WK_XCHECK = 2, WK_PENDING = 4 };

struct AParams {
    mfp_classifier_dev D;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    const uint8_t *fp_arena;
    mfp_analysis *out;
    double *attr_prob;           // optional: archive-tag probabilities, MFP_ATTR_DB_TAGS per packet
    uint64_t *pend_bits;         // per group of 64 packets: unknown-TLS sightings (k_analyze_resolve)
    mfp_seen_tab seen;           // this batch's sightings per distinct fingerprint
    struct WItem *deferred;      // packets scored by k_analyze_wave / k_analyze_big (per-segment lists)
    uint32_t mode;
    uint32_t lane_max_p;         // k_an_score takes fingerprints with P <= min(lane_max_p, PL)
    unsigned long long *stats;   // MFP_AN_STATS_WORDS: the counters of mfp_analysis_counters, then the wave scorer's segment queue
    // the packets to score travel in per-wave segments (k_analyze wave s
    // writes segment s; the later kernels' wave s reads it): no global
    // counter, no atomics, dense lanes
    struct WorkItem *work;       // k_analyze -> k_an_features
    struct Deferred *lanel;      // k_an_features -> k_an_score
    uint32_t *seg_n;             // per segment: [0] work items, [1] lane-scored, [2] wave-scored (3 words each)
    uint32_t nseg, seg_cap;      // segments (k_analyze waves), items per segment
    double *hrow;                // k_analyze_huge's per-wave score rows (HUGE_WAVES * hstride doubles + as many flag bytes)
    uint32_t hstride;            // >= the archive's largest P
};

constexpr uint32_t NFEAT = 6;    // ASN, port, IP, UA, domain, SNI: naive_bayes.hpp:752-772 order

// The classifier's front end, three kernels per batch:
//  k_analyze      lane per packet, groups of 64 records: verified fingerprint-
//                 table lookup and status (perform_analysis_common
//                 analysis.h:1043-1083), the known prevalence set, the
//                 unknown-TLS bitmap; the analysis record of every packet;
//                 the packets that need more (scoring, the classifier-agnostic
//                 attributes, faketls) go to the wave's work segment;
//  k_an_features  lane per work item, dense: destination context
//                 (destination_context::init result.h:346), ASN, server-name
//                 normalisation (plain names), user agent, the six feature-
//                 table lookups with their byte-exact verification, the
//                 classifier-agnostic attributes -> lane-scored or wave-scored
//                 lists;
//  k_an_score     lane per packet with P <= PL: prior + update lists in lane-
//                 private LDS rows, max / second max, fp32 softmax, result --
//                 the reference's own sequential loops (naive_bayes.hpp:752-772,
//                 compute_score_and_probability analysis.h:222-277, softmax
//                 softmax.hpp:227-264).
// Each kernel carries only its stage's state, so none spills, and the later
// two run on dense lists (no idle lanes for packets without work).
#ifndef MFP_AN_PL
#define MFP_AN_PL 16
#endif
constexpr uint32_t PL = MFP_AN_PL;   // k_an_score: fingerprints with at most PL processes, scored lane per packet
constexpr int AW = 4;                // waves per k_analyze / k_an_features block
constexpr int SW = 2;                // waves per k_an_score block (LDS: PL * 512 bytes of score rows per wave)

ADEV mfp_analysis no_info() {        // analysis_result() (result.h:174-210)
    mfp_analysis a;
    a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0; a.status = 0; a.flags = 0;
    a.proc_slot = MFP_NO_PROCESS; a.reserved = 0;
    return a;
}

__global__ __launch_bounds__(64 * AW) void k_analyze(AParams P) {
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    const mfp_classifier_dev &D = P.D;
    const uint64_t ngroups = (P.n + 63) / 64;
    const uint64_t nw = (uint64_t)gridDim.x * AW;
    const uint32_t seg = (uint32_t)(blockIdx.x * AW + wid);
    WorkItem *wk = P.work + (uint64_t)seg * P.seg_cap;
    uint32_t n_wk = 0;               // this wave's work items (wave-uniform)
    uint32_t n_an = 0, n_pend = 0;   // per-wave counts, one atomic each at the end
    for (uint64_t g = seg; g < ngroups; g += nw) {
        const uint64_t i = g * 64 + lane;
        const bool live = i < P.n;
        mfp_record r;
        if (live) r = P.rec[i];
        else { r.fp_len = 0; r.fp_type = 0; r.flags = 0; }
        mfp_analysis a = no_info();
        // messages whose do_analysis calls the classifier: TLS ClientHello
        // (tls.h:1977), HTTP request (http.cc:571), SSH client KEXINIT
        // (ssh.h:480), QUIC Initial (quic.h:1722), STUN request (stun.h:1021);
        // their type must also be in the archive (fp_types)
        const bool typed = live && r.fp_len != 0 &&
                           (r.fp_type == 1 || r.fp_type == 3 || r.fp_type == 5 || r.fp_type == 12 || r.fp_type == 16);
        const bool analyzable = typed && ((D.types_mask >> r.fp_type) & 1u);
        if (typed && !analyzable) { a.status = 4; a.flags = MFP_AN_VALID; }   // fingerprint_status_unanalyzed
        // the classifier-agnostic attributes of TLS and QUIC ClientHellos, analysed
        // or not (check_additional_attributes analysis.h:544-549, pkt_proc.cc:1686)
        const bool xcheck = typed && (r.fp_type == 1 || r.fp_type == 12) && (D.doh_enabled | D.faking_enabled);
        const uint64_t am = __ballot(analyzable || xcheck);
        if (!am) {
            if (live) P.out[i] = a;
            if (lane == 0) P.pend_bits[g] = 0;
            continue;
        }
        n_an += (uint32_t)__builtin_popcountll(am);

        // ---- fingerprint lookup / status (perform_analysis_common, analysis.h:1043-1083):
        // hash and candidate slot per lane, byte-exact check by the wave
        const uint8_t *fp = P.fp_arena + r.fp_offset;
        const uint32_t fl = analyzable ? r.fp_len : 0u;
        uint64_t fh = 0, w0 = 0;
        uint32_t cid = 0xffffffffu, coff = 0;
        if (analyzable) {
            fh = fp_key(r, fp, fl);
            w0 = word_at(fp, fl, 0);
            cid = cand_string_lane(D.fp_slots, D.fp_mask, fh, fl, coff);
        }
        {
            const bool ok = wave_verify(cid != 0xffffffffu, fp, (const uint8_t *)D.pool + coff, fl, lane);
            if (cid != 0xffffffffu && !ok) cid = probe_string_lane(D.fp_slots, D.fp_mask, D.pool, fp, fl, fh);
        }
        uint32_t entry = cid, status = 0;
        bool pending = false;
        const bool tls_unknown = analyzable && entry == 0xffffffffu && fl >= 4 && (uint32_t)w0 == 0x2f736c74u;  // "tls/"
        uint32_t pid = 0xffffffffu, poff = 0;
        if (tls_unknown) pid = cand_string_lane(D.prev_slots, D.prev_mask, fh, fl, poff);
        {
            const bool ok = wave_verify(pid != 0xffffffffu, fp, (const uint8_t *)D.pool + poff, fl, lane);
            if (pid != 0xffffffffu && !ok) pid = probe_string_lane(D.prev_slots, D.prev_mask, D.pool, fp, fl, fh);
        }
        if (analyzable) {
            if (entry != 0xffffffffu) {
                status = 1;                                                   // labeled
            } else if (tls_unknown) {
                if (pid != 0xffffffffu) {
                    status = 3;                    // unlabeled (known set; no LRU update)
                } else {
                    // adaptive set (fingerprint_prevalence LRU): the host
                    // decides the sighting in stream order (mfp_prevalence.cpp);
                    // meanwhile it is classified as a first sighting would be
                    pending = true;
                    status = 2;
                    // classify with "<prefix>randomized" when the DB has it
                    const uint32_t c4 = (uint32_t)(w0 >> 32) & 0xff, c5 = (uint32_t)(w0 >> 40) & 0xff;
                    const uint32_t pre = fl > 5 && c5 == '/' ? (c4 == '1' ? 1u : c4 == '2' ? 2u : 0u) : 0u;
                    entry = D.randomized_entry[pre];
                }
            } else {
                status = 3;                                                   // unlabeled
            }
        }
        {   // unknown-TLS sightings of this group: the per-group bitmap (their
            // first / last / count per distinct fingerprint: k_seen_scan)
            const uint64_t pm = __ballot(pending);
            if (lane == 0) P.pend_bits[g] = pm;
            n_pend += (uint32_t)__builtin_popcountll(pm);
        }
        const bool scored = analyzable && entry != 0xffffffffu;
        if (analyzable) {
            // no process distribution yet: the scorers fill it in
            a.flags = MFP_AN_VALID;
            a.status = (uint8_t)status;
            if (pending) a.flags |= MFP_AN_PENDING;
            // analyze_ip_packet: a truncated message reports "unlabeled" and
            // keeps its classification (pkt_proc.cc:1716-1719)
            if (P.mode == MFP_MODE_ANALYSIS && (r.flags & MFP_FLAG_TRUNCATED) && !pending) a.status = 3;
        }
        if (live) P.out[i] = a;   // the status lives in the analysis record only (no 1-byte record rewrite)
        // the work segment: packets to score, to check for the classifier-
        // agnostic attributes, or (pending) for faketls
        const bool work = scored || xcheck || pending;
        const uint64_t wm = __ballot(work);
        if (work) {
            WorkItem w;
            w.i = (uint32_t)i; w.entry = scored ? entry : 0xffffffffu;
            w.flags = (scored ? WK_SCORE : 0u) | (xcheck ? WK_XCHECK : 0u) | (pending ? WK_PENDING : 0u);
            w.pad = 0;
            wk[n_wk + __builtin_popcountll(wm & ((1ull << lane) - 1))] = w;
        }
        n_wk += (uint32_t)__builtin_popcountll(wm);
    }
    if (lane == 0) P.seg_n[3 * seg] = n_wk;
    if (lane == 0 && n_an) atomicAdd(&P.stats[0], (unsigned long long)n_an);
    if (lane == 0 && n_pend) atomicAdd(&P.stats[1], (unsigned long long)n_pend);
    if (lane == 0 && n_wk) atomicAdd(&P.stats[8], (unsigned long long)n_wk);
}

#ifndef MFP_AN_FEAT_MINW
#define MFP_AN_FEAT_MINW 4   // 4 waves/SIMD: 10.4 -> 9.0 ms (r03l A/B), no spill
#endif
// MFP_AN_FEAT_PREF: a batch's work items, records and descriptors arrive in
// LDS by direct-to-LDS 16-byte loads (global_load_lds_dwordx4: no VGPRs) one
// batch ahead -- the work items two batches ahead, since the records' addresses
// come from them -- so a batch starts from its packet bytes and entry, two
// dependent memory round trips fewer per batch
#ifndef MFP_AN_FEAT_PREF
#define MFP_AN_FEAT_PREF 1
#endif
ADEV void lds_load16(const void *src, void *lds_base) {   // lane l's 16 bytes at lds_base + 16 l
    __builtin_amdgcn_global_load_lds(src, (void __attribute__((address_space(3))) *)lds_base, 16, 0, 0);
}
__global__ __launch_bounds__(64 * AW, MFP_AN_FEAT_MINW) void k_an_features(AParams P) {
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    const mfp_classifier_dev &D = P.D;
    const uint32_t seg = (uint32_t)(blockIdx.x * AW + wid);
#if MFP_AN_FEAT_PREF
    static_assert(sizeof(WorkItem) == 16 && sizeof(mfp_record) == 32 && sizeof(mfp_pkt_desc) == 16, "16-byte rows");
    __shared__ __attribute__((aligned(16))) uint4 pf_w[AW][2][64];   // work items, by batch parity
    __shared__ __attribute__((aligned(16))) uint4 pf_r[AW][2][64];   // the batch's records, two halves
    __shared__ __attribute__((aligned(16))) uint4 pf_d[AW][64];      // the batch's descriptors
#endif
    if (seg >= P.nseg) return;
    const WorkItem *wk = P.work + (uint64_t)seg * P.seg_cap;
    Deferred *ll = P.lanel + (uint64_t)seg * P.seg_cap;
    WItem *dl = P.deferred + (uint64_t)seg * P.seg_cap;
    const uint32_t total = rfl(P.seg_n[3 * seg]);
    uint32_t n_l = 0, n_d = 0;       // wave-uniform list counts
    uint32_t n_look = 0;             // feature-table lookups issued by this lane (mfp_analysis_counters [10])
#if MFP_AN_FEAT_PREF
    // the records and descriptors of the work item at pf_w[wid][par][lane]
    auto pref_rows = [&](uint32_t par) {
        const WorkItem x = *(const WorkItem *)&pf_w[wid][par][lane];
        const uint8_t *rp = (const uint8_t *)(P.rec + x.i);
        lds_load16(rp, &pf_r[wid][0][0]);
        lds_load16(rp + 16, &pf_r[wid][1][0]);
        lds_load16(P.desc + x.i, &pf_d[wid][0]);
    };
    if (lane < total) lds_load16(wk + lane, &pf_w[wid][0][0]);
    if (64 + lane < total) lds_load16(wk + 64 + lane, &pf_w[wid][1][0]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < total) pref_rows(0);
#endif
    for (uint32_t b0 = 0; b0 < total; b0 += 64) {
        const bool live = b0 + lane < total;
        WorkItem w;
        mfp_record r;
#if MFP_AN_FEAT_PREF
        const uint32_t par = (b0 >> 6) & 1u;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this batch's rows, the next batch's items
        uint64_t doff = 0;
        if (live) {
            w = *(const WorkItem *)&pf_w[wid][par][lane];
            const uint4 r0 = pf_r[wid][0][lane], r1 = pf_r[wid][1][lane];
            uint4 rr[2] = {r0, r1};
            __builtin_memcpy(&r, rr, 32);
            doff = ((const mfp_pkt_desc *)&pf_d[wid][lane])->offset;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read before the next batch's rows land
        if (b0 + 64 + lane < total) pref_rows(par ^ 1u);
        if (b0 + 128 + lane < total) lds_load16(wk + b0 + 128 + lane, &pf_w[wid][par][0]);
#else
        if (live) w = wk[b0 + lane];
#endif
        if (!live) { w.i = 0; w.entry = 0xffffffffu; w.flags = 0; w.pad = 0; }
        const uint64_t i = w.i;
        const bool xcheck = w.flags & WK_XCHECK, pending = w.flags & WK_PENDING;
        bool scored = w.flags & WK_SCORE;
        const uint32_t entry = w.entry;
#if !MFP_AN_FEAT_PREF
        if (live) r = P.rec[i];
#endif
        if (!live) { r.fp_len = 0; r.fp_type = 0; r.flags = 0; r.fp_offset = 0; r.net = 0; r.msg = 0;
                     r.sni_off = 0; r.sni_len = 0xffff; r.ua_off = 0; r.ua_len = 0xffff; r.dst_port = 0; r.xflags = 0; }
        const uint8_t *fp = P.fp_arena + r.fp_offset;
        mfp_entry E;
        E.proc_off = 0; E.nproc = 0; E.malware_db = 0; E.generic_dmz = 0;
        if (scored) E = D.entry[entry];
        const FeatRegion FR = scored ? feat_region(E) : FeatRegion{0, 0};
        uint32_t np = E.nproc;
        if (scored && np > 64 * MAXP_CHUNKS_BIG) atomicAdd(&P.stats[2], 1ull);   // scored by k_analyze_huge
        uint32_t hoff[NFEAT], hcnt[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) { hoff[f] = 0; hcnt[f] = 0; }
        bool plain = false, ssh_ua = false, stun_ua = false;
        // string features UA, domain, SNI (hoff/hcnt slots 3..5)
        const uint8_t *vs[3] = {nullptr, nullptr, nullptr};
        uint32_t vl[3] = {0, 0, 0}, voff[3] = {0, 0, 0};
        uint64_t vk[3] = {0, 0, 0};
        Hit vh[3] = {Hit{0, 0}, Hit{0, 0}, Hit{0, 0}};
        bool has[3] = {false, false, false};
        // ---- destination context (destination_context::init, result.h:346)
        // and the classifier-agnostic attributes of a ClientHello
#if MFP_AN_FEAT_PREF
        const uint8_t *pkt = P.arena + (scored || xcheck ? doff : 0);
#else
        const uint8_t *pkt = P.arena + (scored || xcheck ? P.desc[i].offset : 0);
#endif
        // server name / user agent: packet bytes, or the QUIC sidecar behind the string's hash
        const uint8_t *sbase = (r.flags & MFP_FLAG_SIDECAR) ? fp + ((r.fp_len + 7) & ~7u) + 8 : pkt;
        Dst dd;
        dd.ipv = 0; dd.v4 = 0; dd.hi = 0; dd.lo = 0;
        if (scored || xcheck) dd = dst_of(pkt, r.net);
        uint32_t xattr = 0;   // encrypted_dns, domain_faking, faketls
        if (xcheck) {
            // sn_str: the server name as a C string (strncpy MAX_SNI_LEN, result.h:348)
            const uint32_t sl0 = r.sni_len == 0xffff ? 0u : r.sni_len;
            uint64_t ch = 0;
            const uint32_t cl = cstr_hash(sbase + r.sni_off, sl0 < 256 ? sl0 : 256u, ch);
            if (D.doh_enabled && doh_hit(D, sbase + r.sni_off, cl, ch, dd)) xattr |= 1u << D.doh_idx;
            if (D.faking_enabled && domain_faking(D, sbase + r.sni_off, cl, dd)) xattr |= 1u << D.domain_faking_idx;
        }
        if (pending && faketls_fp(fp, r.fp_len)) xattr |= 1u << D.faketls_idx;   // randomized ClientHellos only
        if (scored) {
            const uint32_t ipv = dd.ipv;
            uint32_t asn = 0;
            uint64_t ipkey = 0, v6w0 = 0, v6w1 = 0;
            if (ipv == 4) {
#ifndef MFP_PROBE_AN_NOASN
                asn = asn_v4_lane(D, __builtin_bswap32(dd.v4));
#endif
                ipkey = normalize_ipv4(dd.v4);
            } else if (ipv == 6) {
                v6w0 = __builtin_bswap64(dd.hi);
                v6w1 = __builtin_bswap64(dd.lo);
                if (D.n_asn6) asn = asn_v6_lane(D, dd.hi, dd.lo);
                // normalize_ipv6 (mfp_common.hpp) on the two words
                const bool gu = (v6w0 & 0xe0) == 0x20;
                const bool mapped = v6w0 == 0 && (v6w1 & 0xffffffffull) == 0xffff0000ull;
                if (!(gu || mapped)) { v6w0 = 0xfd; v6w1 = 1ull << 56; }
                ipkey = hash_final(word_term(v6w0, 0) ^ word_term(v6w1, 1), 16);
            }
            // server name: TLS SNI / HTTP Host (strncpy 256, NUL stops); STUN has
            // none (its span holds the message, for the JSON writer)
            const uint32_t sl = r.sni_len == 0xffff || r.msg == MFP_MSG_STUN ? 0u : r.sni_len;
            const uint8_t *sp = sbase + r.sni_off;
            uint32_t tld = 0;
            uint64_t nh = 0;
#ifdef MFP_PROBE_AN_NOSTR
            plain = sl != 0; nh = sl; tld = 0;
#else
            plain = plain_server_name(sp, sl, tld, nh);   // no NUL in a plain name
#endif
            // user agent (strncpy 511, NUL stops); TLS has none (its slot holds
            // the ALPN list); QUIC's is transport parameter 0x3129 (tls.h:1346-1355)
            // SSH (protocol + comment, the delimiting space dropped) is built and
            // probed by k_analyze_wave
            // STUN's SOFTWARE goes through utf8_safe_string (stun.h:1024): the
            // wave scorer escapes it into LDS (slow_lookups)
            ssh_ua = r.msg == MFP_MSG_SSH_INIT && r.ua_len != 0xffff;
            stun_ua = r.msg == MFP_MSG_STUN;
            // (a TLS ClientHello's ua span is its ALPN list unless MFP_XF_TLS_UA: the
            // user agent of a draft transport-parameter extension, tls.h:1346-1355)
            const bool tls_alpn_span = r.msg == MFP_MSG_TLS_CH && !(r.xflags & MFP_XF_TLS_UA);
            uint32_t ul = r.ua_len == 0xffff || tls_alpn_span || ssh_ua || stun_ua ? 0u : r.ua_len;
            if (ul > 511) ul = 511;
            const uint8_t *up = sbase + r.ua_off;
            uint64_t uh = 0;
#ifdef MFP_PROBE_AN_NOSTR
            uh = ul;
#else
            ul = cstr_hash(up, ul, uh);
#endif
            const uint32_t dport = r.dst_port;

            // ---- the six feature lookups: every home slot loaded at once
            n_look += 2u + (ipv != 0) + (!ssh_ua && !stun_ua) + (plain ? 2u : 0u);
            const bool has_ua = !ssh_ua && !stun_ua;
            uint64_t dk = 0;
            if (plain) dk = lane_hash(sp + tld, sl - tld);
            const uint32_t kA = home_slot(FR, entry, F_ASN, asn), kP = home_slot(FR, entry, F_PORT, dport);
            const uint32_t kI = home_slot(FR, entry, ipv == 6 ? F_IPV6 : F_IPV4, ipkey);
            const uint32_t kU = home_slot(FR, entry, F_UA, uh), kD = home_slot(FR, entry, F_DOMAIN, dk);
            const uint32_t kS = home_slot(FR, entry, F_SNI, nh);
            const mfp_feat_slot sA = D.feat_slots[FR.base + kA], sP = D.feat_slots[FR.base + kP];
            const mfp_feat_slot sI = ipv ? D.feat_slots[FR.base + kI] : empty_slot();
            const mfp_feat_slot sU = has_ua ? D.feat_slots[FR.base + kU] : empty_slot();
            const mfp_feat_slot sD = plain ? D.feat_slots[FR.base + kD] : empty_slot();
            const mfp_feat_slot sS = plain ? D.feat_slots[FR.base + kS] : empty_slot();
            Hit h;
            h = probe_int_from(D, FR, entry, F_ASN, asn, kA, sA);
            hoff[0] = h.off; hcnt[0] = h.cnt;
            h = probe_int_from(D, FR, entry, F_PORT, dport, kP, sP);
            hoff[1] = h.off; hcnt[1] = h.cnt;
            if (ipv == 4) {
                h = probe_int_from(D, FR, entry, F_IPV4, ipkey, kI, sI);
                hoff[2] = h.off; hcnt[2] = h.cnt;
            } else if (ipv == 6) {
                // the 16 normalized bytes, verified against the pool
                mfp_feat_slot s6 = sI;
                for (uint32_t k = kI;; k = (k + 1) & FR.mask, s6 = D.feat_slots[FR.base + k]) {
                    if (s6.entry == 0xffffffffu) break;
                    if (s6.entry == entry && s6.kind == F_IPV6 && s6.key == ipkey && s6.str_len == 16) {
                        const uint8_t *ps = (const uint8_t *)D.pool + s6.str_off;
                        if (word_at(ps, 16, 0) == v6w0 && word_at(ps, 16, 1) == v6w1) {
                            hoff[2] = s6.upd_off; hcnt[2] = s6.upd_cnt;
                            break;
                        }
                    }
                }
            }
            // string features: candidate slots here, byte-exact check by the wave below
            vs[0] = up; vl[0] = ul; vk[0] = uh;
            has[0] = has_ua && cand_from(D, FR, entry, F_UA, uh, ul, kU, sU, vh[0], voff[0]);
            if (plain) {   // else k_analyze_wave normalises the name (wave, LDS)
                vs[1] = sp + tld; vl[1] = sl - tld; vk[1] = dk;
                has[1] = cand_from(D, FR, entry, F_DOMAIN, dk, vl[1], kD, sD, vh[1], voff[1]);
                vs[2] = sp; vl[2] = sl; vk[2] = nh;
                has[2] = cand_from(D, FR, entry, F_SNI, nh, sl, kS, sS, vh[2], voff[2]);
            }
        }
        // byte-exact check of the candidates.  Lane by lane: each lane compares
        // its own (short: server names, user agents) strings with a few wide
        // loads, all lanes at once; the wave-cooperative check would take one
        // memory round trip per string of the wave, one after another
#pragma unroll
        for (int v = 0; v < 3; v++) {
#ifdef MFP_AN_FEAT_WAVE_VERIFY
            const bool ok = wave_verify(has[v], vs[v], (const uint8_t *)D.pool + voff[v], vl[v], lane);
#else
            const bool ok = !has[v] || lane_eq<4>(vs[v], (const uint8_t *)D.pool + voff[v], vl[v]);
#endif
            if (has[v]) {
                // a hash collision (ok == false) takes the full probe, which keeps looking
                const Hit h = ok ? vh[v] : probe_feature_lane(D, FR, entry, v == 0 ? F_UA : v == 1 ? F_DOMAIN : F_SNI, vk[v],
                                                              vs[v], vl[v]);
                hoff[3 + v] = h.off; hcnt[3 + v] = h.cnt;
            }
        }
        // scored: to the lane scorer (small P, plain name) or the wave scorer;
        // not scored: the attributes go into the record now
        const bool lanep = scored && np <= PL && np <= P.lane_max_p && plain && !ssh_ua && !stun_ua;
        const bool defer = scored && !lanep;
        if (live && !scored && xattr) P.out[i].attr = (uint16_t)(P.out[i].attr | xattr);
        const uint64_t lm = __ballot(lanep), dm = __ballot(defer);
        if (lanep) {
            Deferred d;
            d.i = (uint32_t)i; d.entry = entry; d.slow_sni = 0u; d.slow_ua = xattr << 16;
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) { d.off[f] = hoff[f]; d.cnt[f] = hcnt[f]; }
            ll[n_l + __builtin_popcountll(lm & ((1ull << lane) - 1))] = d;
        }
        if (defer) {
            WItem w;
            w.i = (uint32_t)i; w.entry = entry; w.flags = (plain ? 0u : 1u) | (ssh_ua ? 2u : 0u) | (stun_ua ? 4u : 0u) | (xattr << 16);
            w.ft = r.fp_type;
            w.po = E.proc_off; w.np = np; w.mdb = E.malware_db; w.dmz = E.generic_dmz;
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) { w.off[f] = hoff[f]; w.cnt[f] = hcnt[f]; }
            dl[n_d + __builtin_popcountll(dm & ((1ull << lane) - 1))] = w;
        }
        n_l += (uint32_t)__builtin_popcountll(lm);
        n_d += (uint32_t)__builtin_popcountll(dm);
    }
    if (lane == 0) { P.seg_n[3 * seg + 1] = n_l; P.seg_n[3 * seg + 2] = n_d; }
    if (lane == 0 && n_d) atomicAdd(&P.stats[3], (unsigned long long)n_d);
    if (lane == 0 && n_l) atomicAdd(&P.stats[9], (unsigned long long)n_l);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) n_look += __shfl_xor(n_look, d, 64);
    if (lane == 0 && n_look) atomicAdd(&P.stats[10], (unsigned long long)n_look);
}

__global__ __launch_bounds__(64 * SW) void k_an_score(AParams P) {
    __shared__ double sc_lds[SW][64 * PL];   // per wave: lane-private score rows S[p][lane]
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    double *scl = sc_lds[wid];
    const mfp_classifier_dev &D = P.D;
    uint32_t c_prior = 0, c_upd = 0; // per-lane table entries read (mfp_analysis_counters)
    for (uint32_t seg = blockIdx.x * SW + wid; seg < P.nseg; seg += gridDim.x * SW) {
        const Deferred *ll = P.lanel + (uint64_t)seg * P.seg_cap;
        const uint32_t total = rfl(P.seg_n[3 * seg + 1]);
        for (uint32_t b0 = 0; b0 < total; b0 += 64) {
            if (b0 + lane >= total) continue;
            const Deferred d = ll[b0 + lane];
            const uint64_t i = d.i;
            const mfp_entry E = D.entry[d.entry];
            const uint32_t np = E.nproc, po = E.proc_off, mdb = E.malware_db, dmz = E.generic_dmz, mbits = E.mal_bits;
            c_prior += np;
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) c_upd += d.cnt[f] & ~MFP_UPD_SERIAL;
            double *S = scl + lane;                    // S[p * 64]
            for (uint32_t p = 0; p < np; p++) S[p * 64] = D.prior[po + p];
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) {
                const uint32_t c = d.cnt[f] & ~MFP_UPD_SERIAL;
                const mfp_update *ul = D.upd + d.off[f];
                uint32_t k = 0;
                for (; k + 4 <= c; k += 4) {
                    const mfp_update x0 = ul[k], x1 = ul[k + 1], x2 = ul[k + 2], x3 = ul[k + 3];
                    S[x0.idx * 64] += x0.value;
                    S[x1.idx * 64] += x1.value;
                    S[x2.idx * 64] += x2.value;
                    S[x3.idx * 64] += x3.value;
                }
                for (; k < c; k++) { const mfp_update x = ul[k]; S[x.idx * 64] += x.value; }
            }
            double mx = -1.7976931348623157e308, sx = -1.7976931348623157e308;
            uint32_t imx = 0, isx = 0;
            for (uint32_t p = 0; p < np; p++) {
                const double v = S[p * 64];
                if (v > mx) { sx = mx; isx = imx; mx = v; imx = p; }
                else if (v > sx) { sx = v; isx = p; }
            }
            // the "generic dmz process" swap is decided by the ranks alone
            const bool swap = mdb && dmz == imx && !((mbits >> isx) & 1u);
            const uint32_t ibest = swap ? isx : imx;
            // archive tags of the selected process: their probability is the
            // softmax mass of the processes carrying them (analysis.h:268-277;
            // the swapped-out maximum counts 0)
            const uint32_t tags = D.proc_attr[po + ibest] & D.db_tags;
            double ap[MFP_ATTR_DB_TAGS];
#pragma unroll
            for (int k = 0; k < MFP_ATTR_DB_TAGS; k++) ap[k] = 0.0;
            double ssum = 0.0, swo = 0.0, mal = 0.0, p_imx = 0.0, p_isx = 0.0;
            for (uint32_t p = 0; p < np; p++) {
                const double e = (double)expf_ref((float)(S[p * 64] - mx));
                ssum += e;
                if (p != imx) swo += e;
                if ((mbits >> p) & 1u) mal += e;
                if (p == imx) p_imx = e;
                if (p == isx) p_isx = e;
                if (tags && !(swap && p == imx)) {
                    const uint32_t pa = D.proc_attr[po + p] & tags;
#pragma unroll
                    for (int k = 0; k < MFP_ATTR_DB_TAGS; k++)
                        if ((pa >> (MFP_ATTR_DB_FIRST + k)) & 1u) ap[k] += e;
                }
            }
            double max_score = p_imx;
            if (ssum > 0.0 && mdb) mal /= ssum;
            if (swap) {
                ssum = swo;
                max_score = p_isx;
            }
            if (ssum > 0.0) max_score /= ssum;
            if (tags && P.attr_prob) {
                double *o = P.attr_prob + i * MFP_ATTR_DB_TAGS;
#pragma unroll
                for (int k = 0; k < MFP_ATTR_DB_TAGS; k++)
                    if ((tags >> (MFP_ATTR_DB_FIRST + k)) & 1u) o[k] = ssum > 0.0 ? ap[k] / ssum : ap[k];
            }
            mfp_analysis a = P.out[i];   // status and pending flag from k_analyze
            a.score = max_score;
            a.process = D.proc_id[po + ibest];
            a.proc_slot = po + ibest;
            a.attr = (uint16_t)(D.proc_attr[po + ibest] | (d.slow_ua >> 16));
            a.malware_prob = -1.0;
            a.flags = (uint8_t)(MFP_AN_VALID | (a.flags & MFP_AN_PENDING));
            if (mdb) {
                a.malware_prob = mal;
                a.flags |= MFP_AN_CLASSIFY_MALWARE;
                if ((mbits >> ibest) & 1u) a.flags |= MFP_AN_MALWARE;
            }
            if ((a.flags & MFP_AN_MALWARE) && P.rec[i].fp_type == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
            P.out[i] = a;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { c_prior += __shfl_xor(c_prior, d, 64); c_upd += __shfl_xor(c_upd, d, 64); }
    if (lane == 0 && c_prior) atomicAdd(&P.stats[4], (unsigned long long)c_prior);
    if (lane == 0 && c_upd) atomicAdd(&P.stats[5], (unsigned long long)c_upd);
}

// The wave scorers: the packets k_an_features deferred (more than PL
// processes, a server name that needs the full normalisation, an SSH user
// agent) -- one wavefront per packet, lane i holds process i.  Scores live in
// the wave's LDS row: the prior and the first 64 entries of every update list
// arrive in one round trip, then the lists are applied feature by feature as
// lane-parallel scatters (a list names each process at most once, so every
// process sees the reference's addition order; lists flagged MFP_UPD_SERIAL
// go one by one); max / second max, the dmz swap, softmax and the sums in the
// reference's order (naive_bayes.hpp:752-772, analysis.h:222-358,
// softmax.hpp:227-264).

// the slow feature lookups of a wave-scored packet (WItem flags): the server
// name normalised on lane 0 into LDS, hashed and verified lane-parallel
// (strncpy 256, NUL stops); the SSH user agent (ssh_init_packet::do_analysis
// ssh.h:480-487): protocol then comment into a data_buffer<512> (nulled --
// empty -- when they do not fit), strncpy 511, NUL stops.  The record's span
// is "protocol SP comment"; its first space is the delimiter.  The STUN
// SOFTWARE value (flag 4) as utf8_safe_string<512> makes it (stun.h:1024,
// mfpc::utf8_safe_512).  Updates off/cnt of features 3 (UA), 4 (domain), 5
// (SNI); returns the features changed.
ADEV uint32_t slow_lookups(const AParams &P, uint32_t i, uint32_t entry, uint32_t flags, char *nbuf, char *ub,
                           uint32_t (&off)[NFEAT], uint32_t (&cnt)[NFEAT], uint32_t lane) {
    const mfp_classifier_dev &D = P.D;
    uint32_t changed = 0;
    const FeatRegion FR{rfl(D.entry[entry].feat_base), rfl(D.entry[entry].feat_mask)};
    if (flags & 1u) {
        const mfp_record r = P.rec[i];
        const uint32_t sni = rfl((uint32_t)r.sni_off | ((uint32_t)r.sni_len << 16));
        const uint32_t sl = (sni >> 16) == 0xffff ? 0 : (sni >> 16);
        const uint8_t *sp = ((r.flags & MFP_FLAG_SIDECAR) ? P.fp_arena + r.fp_offset + ((r.fp_len + 7) & ~7u) + 8
                                                         : P.arena + P.desc[i].offset) + (sni & 0xffff);
        int nlen = 0;
        if (lane == 0) nlen = normalize_server_name(sp, (int)sl, nbuf);
        nlen = (int)rfl((uint32_t)nlen);
        __builtin_amdgcn_wave_barrier();
        const int tld = (int)rfl((uint32_t)(lane == 0 ? tld_domain_offset(nbuf, nlen) : 0));
        const uint8_t *dom = (const uint8_t *)nbuf + tld;
        Hit h = probe_feature(D, FR, entry, F_DOMAIN, wave_hash(dom, (uint32_t)(nlen - tld), lane), dom,
                              (uint32_t)(nlen - tld), true, lane);
        off[4] = h.off; cnt[4] = h.cnt;
        h = probe_feature(D, FR, entry, F_SNI, wave_hash((const uint8_t *)nbuf, (uint32_t)nlen, lane),
                          (const uint8_t *)nbuf, (uint32_t)nlen, true, lane);
        off[5] = h.off; cnt[5] = h.cnt;
        __builtin_amdgcn_wave_barrier();
        changed |= 3u << 4;
    }
    if (flags & 6u) {
        const mfp_record r = P.rec[i];
        const uint8_t *sp = P.arena + P.desc[i].offset + r.ua_off;
        const uint32_t L = r.ua_len;
        int ulen = 0;
        if (lane == 0 && (flags & 4u)) {
            ulen = L == 0xffff ? 0 : (int)mfpc::utf8_safe_512(sp, L, ub);
        } else if (lane == 0) {
            uint32_t pl = 0;
            while (pl < L && sp[pl] != ' ') pl++;
            const uint32_t total = pl < L ? L - 1 : L;
            uint32_t n = total > 512 ? 0u : (total > 511 ? 511u : total);
            uint32_t k = 0;
            for (uint32_t j = 0; k < n && j < L; j++) {
                if (j == pl) continue;
                const char c = (char)sp[j];
                if (c == 0) break;
                ub[k++] = c;
            }
            ulen = (int)k;
        }
        ulen = (int)rfl((uint32_t)ulen);
        __builtin_amdgcn_wave_barrier();
        const Hit h = probe_feature(D, FR, entry, F_UA, wave_hash((const uint8_t *)ub, (uint32_t)ulen, lane),
                                    (const uint8_t *)ub, (uint32_t)ulen, true, lane);
        off[3] = h.off; cnt[3] = h.cnt;
        __builtin_amdgcn_wave_barrier();
        changed |= 1u << 3;
    }
    return changed;
}

// one feature's update list applied to the wave's score row; u_idx/u_val:
// entries 0..63 (lane k: entry k), the rest loaded here
ADEV void scatter_list(const mfp_classifier_dev &D, double *scl, uint32_t off, uint32_t cntf, uint32_t u_idx,
                       double u_val, bool anylong, uint32_t lane) {
    const uint32_t c = cntf & ~MFP_UPD_SERIAL;
    if (cntf & MFP_UPD_SERIAL) {
        for (uint32_t k = 0; k < c; k++) {
            const mfp_update x = k < 64 && !anylong ? mfp_update{(uint32_t)__shfl((int)u_idx, (int)k, 64), 0,
                                                                __shfl(u_val, (int)k, 64)}
                                                    : D.upd[off + k];
            if (lane == 0) scl[x.idx] += x.value;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        if (lane < c) scl[u_idx] += u_val;
        for (uint32_t b = 64; b < c; b += 64) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (b + lane < c) { const mfp_update x = D.upd[off + b + lane]; scl[x.idx] += x.value; }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// max, then second max, over the wave's CH chunks (sequential first-index rule)
template <int CH>
ADEV void max_two(const double (&sc)[CH], uint32_t np, uint32_t lane, double &mx, uint32_t &imx, uint32_t &isx) {
    mx = -1.7976931348623157e308;
    imx = 0xffffffffu;
#pragma unroll
    for (int c = 0; c < CH; c++) {
        const uint32_t pi = (uint32_t)c * 64 + lane;
        if (pi < np && (imx == 0xffffffffu || sc[c] > mx)) { mx = sc[c]; imx = pi; }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const double om = __shfl_xor(mx, d, 64);
        const uint32_t oi = (uint32_t)__shfl_xor((int)imx, d, 64);
        if (oi != 0xffffffffu && (imx == 0xffffffffu || om > mx || (om == mx && oi < imx))) { mx = om; imx = oi; }
    }
    imx = rfl(imx);
    mx = __hiloint2double((int)rfl((uint32_t)(__double_as_longlong(mx) >> 32)), (int)rfl((uint32_t)__double_as_longlong(mx)));
    double sx = -1.7976931348623157e308;
    isx = 0xffffffffu;
#pragma unroll
    for (int c = 0; c < CH; c++) {
        const uint32_t pi = (uint32_t)c * 64 + lane;
        if (pi < np && pi != imx && (isx == 0xffffffffu || sc[c] > sx)) { sx = sc[c]; isx = pi; }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const double om = __shfl_xor(sx, d, 64);
        const uint32_t oi = (uint32_t)__shfl_xor((int)isx, d, 64);
        if (oi != 0xffffffffu && (isx == 0xffffffffu || om > sx || (om == sx && oi < isx))) { sx = om; isx = oi; }
    }
    isx = rfl(isx);
    if (isx == 0xffffffffu) isx = 0;   // P == 1: index_sec stays 0
}

// the softmax sums in process order, as the reference adds them
// (softmax.hpp:250-263, analysis.h:268-277), one sum per lane: 0 score_sum,
// 1 score_sum_without_max, 2 malware_prob, 3.. the archive tags.  Each lane
// adds e or +0.0 (e >= 0: the same sums), eight row entries per LDS batch.
ADEV double row_sums(const double *scl, const uint8_t *fl, uint32_t np, uint32_t imx, uint32_t nsum, uint32_t lane) {
    double acc = 0.0;
    if (lane < nsum) {
        // which entries this lane adds, as masks (no branches per entry)
        const bool l_all = lane == 0, l_wo = lane == 1;
        const uint32_t m = lane == 2 ? 1u : lane >= 3 ? 1u << (lane - 2) : 0u;
        const uint32_t x80 = lane >= 3 ? 0x80u : 0u;   // the swapped-out maximum counts 0 for the tags
        auto take = [&](uint32_t p, uint32_t f) {
            return l_all | (l_wo & (p != imx)) | (((f & m) != 0u) & ((f & x80) == 0u));
        };
        uint32_t p = 0;
        for (; p + 8 <= np; p += 8) {
            double e[8];
            uint32_t f[8];
#pragma unroll
            for (int k = 0; k < 8; k++) { e[k] = scl[p + k]; f[k] = fl[p + k]; }
#pragma unroll
            for (int k = 0; k < 8; k++) acc += take(p + k, f[k]) ? e[k] : 0.0;
        }
        for (; p < np; p++) acc += take(p, fl[p]) ? scl[p] : 0.0;
    }
    return acc;
}
ADEV double lane_d(double v, uint32_t l) {
    return __hiloint2double(__builtin_amdgcn_readlane((int)(__double_as_longlong(v) >> 32), (int)l),
                            __builtin_amdgcn_readlane((int)__double_as_longlong(v), (int)l));
}

// ---- k_analyze_wave (P <= 64 * MAXP_CHUNKS): software-pipelined over each
// segment's packets.  Packet q + 1's table rows (update-list heads, the first
// SCH chunks of priors, process attributes and ids, malware bytes, its
// analysis-record word) are loaded while packet q is scored, and packet q + 2's
// WItem one step earlier, so the scoring tail of q runs on LDS and registers
// only and a packet costs about one memory round trip instead of a chain of
// them.  Chunks SCH.. (P > 64 * SCH, rare) are loaded when the packet starts.
constexpr int SCH = 4;
struct WStage {
    uint32_t uidx[NFEAT];
    double uval[NFEAT];
    double pr[SCH];
    uint32_t attr[SCH], pid[SCH];
    uint32_t malb[SCH];
    uint32_t outw;               // the analysis record's attr / status / flags word (k_analyze's)
};
ADEV uint32_t wf(uint32_t w, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)w, k); }
ADEV uint32_t wi_load(const WItem *seg, uint32_t q, uint32_t total, uint32_t lane) {
    return q < total && lane < WITEM_WORDS ? ((const uint32_t *)(seg + q))[lane] : 0u;
}
// issue (no use of the results: the loads stay in flight)
ADEV void stage_issue(const AParams &P, uint32_t w, WStage &st, uint32_t lane) {
    const mfp_classifier_dev &D = P.D;
    const uint32_t np = wf(w, WI_NP), po = wf(w, WI_PO), i = wf(w, WI_I);
    const bool take = np != 0 && np <= 64u * MAXP_CHUNKS;      // a word of zeros past the segment's end
#pragma unroll
    for (uint32_t f = 0; f < NFEAT; f++) {
        const uint32_t c = wf(w, WI_CNT + f) & ~MFP_UPD_SERIAL, o = wf(w, WI_OFF + f);
        st.uidx[f] = 0; st.uval[f] = 0.0;
        if (take && lane < c) { st.uidx[f] = D.upd[o + lane].idx; st.uval[f] = D.upd[o + lane].value; }
    }
#pragma unroll
    for (int c = 0; c < SCH; c++) {
        const uint32_t pi = (uint32_t)c * 64 + lane;
        st.pr[c] = 0.0; st.attr[c] = 0; st.pid[c] = 0; st.malb[c] = 0;
        if (take && pi < np) {
            st.pr[c] = D.prior[po + pi];
            st.attr[c] = D.proc_attr[po + pi];
            st.pid[c] = D.proc_id[po + pi];
            st.malb[c] = D.proc_mal[po + pi];
        }
    }
    st.outw = take ? ((const uint32_t *)(P.out + i))[5] : 0u;
}

// MFP_AN_PHASES (probe builds): clock sums per phase of the pipelined scorer
// into stats[MFP_AN_NCOUNTERS + 1 + k]
#ifdef MFP_AN_PHASES
#define PH_MARK(k) do { const uint64_t t_ = clock64(); ph[k] += t_ - ph_t; ph_t = t_; } while (0)
#else
#define PH_MARK(k) do { } while (0)
#endif
__device__ __forceinline__ void wave_scorer_pipe(const AParams &P, char (*sni_buf)[336], char (*ua_buf)[520],
                                                 double (*sc_lds)[64 * MAXP_CHUNKS], uint32_t (*at_lds)[64 * MAXP_CHUNKS],
                                                 uint32_t (*id_lds)[64 * MAXP_CHUNKS], uint8_t (*fl_lds)[64 * MAXP_CHUNKS]) {
    constexpr int CH = MAXP_CHUNKS;
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    double *scl = sc_lds[wid];
    uint32_t *arow = at_lds[wid], *idrow = id_lds[wid];
    uint8_t *fl = fl_lds[wid];
    const mfp_classifier_dev &D = P.D;
    uint64_t w_prior = 0, w_upd = 0;   // table entries read (mfp_analysis_counters [6], [7])
#ifdef MFP_AN_PHASES
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t ph_t = clock64();
#endif
    for (;;) {
        // segments from a queue: the waves that draw short lists take more of them
        unsigned long long sgl = 0;
        if (lane == 0) sgl = atomicAdd(&P.stats[MFP_AN_NCOUNTERS], 1ull);
        const uint64_t sg = rfl((uint32_t)sgl);
        if (sg >= P.nseg) break;
        const WItem *seg = P.deferred + sg * P.seg_cap;
        const uint32_t total = rfl(P.seg_n[3 * sg + 2]);
        if (total == 0) continue;
        uint32_t wc = wi_load(seg, 0, total, lane), wn = wi_load(seg, 1, total, lane);
        WStage st;
        stage_issue(P, wc, st, lane);
        for (uint32_t q = 0; q < total; q++) {
            const uint32_t i = wf(wc, WI_I), np = wf(wc, WI_NP), po = wf(wc, WI_PO);
            const uint32_t flags = wf(wc, WI_FLAGS), mdb = wf(wc, WI_MDB), dmz = wf(wc, WI_DMZ), ft = wf(wc, WI_FT);
            const bool mine = np <= 64u * CH;   // larger: k_analyze_big's
            uint32_t off[NFEAT], cnt[NFEAT];
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) { off[f] = wf(wc, WI_OFF + f); cnt[f] = wf(wc, WI_CNT + f); }
            uint32_t malbits = 0, outw = 0;
            PH_MARK(0);
            if (mine) {
                // ---- [A] this packet's rows into LDS, the update lists applied
                if (flags & 7u) {
                    const uint32_t ch = slow_lookups(P, i, wf(wc, WI_ENTRY), flags, sni_buf[wid], ua_buf[wid], off, cnt, lane);
#pragma unroll
                    for (uint32_t f = 3; f < NFEAT; f++)
                        if ((ch >> f) & 1u) {
                            st.uidx[f] = 0; st.uval[f] = 0.0;
                            if (lane < (cnt[f] & ~MFP_UPD_SERIAL)) { st.uidx[f] = D.upd[off[f] + lane].idx; st.uval[f] = D.upd[off[f] + lane].value; }
                        }
                }
                w_prior += np;
                uint32_t anylong = 0;
#pragma unroll
                for (uint32_t f = 0; f < NFEAT; f++) {
                    w_upd += cnt[f] & ~MFP_UPD_SERIAL;
                    anylong |= (cnt[f] & ~MFP_UPD_SERIAL) > 64 ? 1u : 0u;
                }
#pragma unroll
                for (int c = 0; c < SCH; c++) {
                    const uint32_t pi = (uint32_t)c * 64 + lane;
                    if ((uint32_t)c * 64 < np) {
                        scl[pi] = st.pr[c];
                        arow[pi] = st.attr[c];
                        idrow[pi] = st.pid[c];
                        if (st.malb[c]) malbits |= 1u << c;
                    }
                }
                if (np > 64u * SCH) {
#pragma unroll
                    for (int c = SCH; c < CH; c++) {
                        const uint32_t pi = (uint32_t)c * 64 + lane;
                        if ((uint32_t)c * 64 < np) {
                            scl[pi] = pi < np ? D.prior[po + pi] : 0.0;
                            arow[pi] = pi < np ? D.proc_attr[po + pi] : 0u;
                            idrow[pi] = pi < np ? D.proc_id[po + pi] : 0u;
                            if (pi < np && D.proc_mal[po + pi]) malbits |= 1u << c;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                PH_MARK(1);
#pragma unroll
                for (uint32_t f = 0; f < NFEAT; f++) scatter_list(D, scl, off[f], cnt[f], st.uidx[f], st.uval[f], anylong, lane);
                outw = st.outw;
                PH_MARK(2);
            }
            // ---- [B] the next packet's rows and the WItem after it: in flight
            // while this packet's scoring tail runs
            const uint32_t w2 = wi_load(seg, q + 2, total, lane);
            stage_issue(P, wn, st, lane);
            PH_MARK(3);
            if (mine) {
                // ---- [C] scoring tail: LDS and registers only
                double sc[CH];
#pragma unroll
                for (int c = 0; c < CH; c++) sc[c] = (uint32_t)c * 64 < np ? scl[c * 64 + lane] : 0.0;
                __builtin_amdgcn_wave_barrier();
                double mx;
                uint32_t imx, isx;
                max_two<CH>(sc, np, lane, mx, imx, isx);
                PH_MARK(4);
                const uint32_t mal_isx = (wf(malbits, isx & 63) >> (isx >> 6)) & 1u;
                const uint32_t mal_imx = (wf(malbits, imx & 63) >> (imx >> 6)) & 1u;
                // the dmz swap (decided by the ranks alone) and the selected
                // process's archive tags (analysis.h:258-277)
                const bool swap = mdb && dmz == imx && !mal_isx;
                const uint32_t ibest = swap ? isx : imx;
                const uint32_t abest = rfl(arow[ibest]), pbest = rfl(idrow[ibest]);
                const uint32_t mal_best = swap ? mal_isx : mal_imx;
                const uint32_t tags = abest & D.db_tags;
                // softmax (expf in fp32, stored as double) into LDS, per-process flags
#pragma unroll
                for (int c = 0; c < CH; c++) {
                    const uint32_t pi = (uint32_t)c * 64 + lane;
                    if (pi < np) {
                        scl[pi] = (double)expf_ref((float)(sc[c] - mx));
                        uint32_t f = (malbits >> c) & 1u;
                        if (tags) f |= ((arow[pi] & tags) >> MFP_ATTR_DB_FIRST) << 1;
                        if (swap && pi == imx) f |= 0x80u;   // process_score[index_max] = 0 (analysis.h:264)
                        fl[pi] = (uint8_t)f;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                PH_MARK(5);
                const double acc = row_sums(scl, fl, np, imx, tags ? 3u + MFP_ATTR_DB_TAGS : 3u, lane);
                double ssum = lane_d(acc, 0), swo = lane_d(acc, 1), mal = lane_d(acc, 2);
                const double p_imx = scl[imx], p_isx = scl[isx];
                PH_MARK(6);
                double ap = 0.0;   // lane k < MFP_ATTR_DB_TAGS: tag k's sum
                if (tags) {
#pragma unroll
                    for (int k = 0; k < MFP_ATTR_DB_TAGS; k++) {
                        const double v = lane_d(acc, 3 + k);
                        if ((int)lane == k) ap = v;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                double max_score = p_imx;
                if (ssum > 0.0 && mdb) mal /= ssum;
                if (swap) {
                    ssum = swo;
                    max_score = p_isx;
                }
                if (ssum > 0.0) max_score /= ssum;
                if (tags && P.attr_prob && lane < MFP_ATTR_DB_TAGS && ((tags >> (MFP_ATTR_DB_FIRST + lane)) & 1u))
                    P.attr_prob[(uint64_t)i * MFP_ATTR_DB_TAGS + lane] = ssum > 0.0 ? ap / ssum : ap;
                if (lane == 0) {
                    // status, pending flag and the additional attributes from k_analyze
                    mfp_analysis a;
                    a.score = max_score;
                    a.process = pbest;
                    a.proc_slot = po + ibest;
                    a.attr = (uint16_t)(abest | (outw & 0xffffu) | (flags >> 16));
                    a.status = (uint8_t)(outw >> 16);
                    a.malware_prob = -1.0;
                    a.flags = (uint8_t)(MFP_AN_VALID | ((outw >> 24) & MFP_AN_PENDING));
                    a.reserved = 0;
                    if (mdb) {
                        a.malware_prob = mal;
                        a.flags |= MFP_AN_CLASSIFY_MALWARE;
                        if (mal_best) a.flags |= MFP_AN_MALWARE;
                    }
                    // encrypted_channel (analysis.h:1161-1163)
                    if ((a.flags & MFP_AN_MALWARE) && ft == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
                    P.out[i] = a;
                }
                __builtin_amdgcn_wave_barrier();
                PH_MARK(7);
            }
            wc = wn;
            wn = w2;
        }
    }
    if (lane == 0 && w_prior) atomicAdd(&P.stats[6], (unsigned long long)w_prior);
    if (lane == 0 && w_upd) atomicAdd(&P.stats[7], (unsigned long long)w_upd);
#ifdef MFP_AN_PHASES
    if (lane == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&P.stats[MFP_AN_NCOUNTERS + 1 + k], (unsigned long long)ph[k]);
#endif
}

// ---- k_analyze_big (64 * MAXP_CHUNKS < P <= 64 * MAXP_CHUNKS_BIG, production
// archives have a few): one wave per block, the CH chunks in registers and in
// the wave's LDS rows, one packet after another
template <int CH>
__device__ __forceinline__ void wave_scorer_big(const AParams &P, char *nbuf, char *ub, double *scl, uint8_t *fl) {
    const uint32_t lane = lane_id();
    const mfp_classifier_dev &D = P.D;
    uint64_t w_prior = 0, w_upd = 0;   // table entries read (mfp_analysis_counters [6], [7])
    for (uint64_t sg = blockIdx.x; sg < P.nseg; sg += gridDim.x) {
    const WItem *dseg = P.deferred + sg * P.seg_cap;
    const uint32_t total = rfl(P.seg_n[3 * sg + 2]);
    for (uint32_t q = 0; q < total; q++) {
        const uint32_t wc = wi_load(dseg, q, total, lane);
        const uint32_t np = wf(wc, WI_NP);
        if (np <= 64u * MAXP_CHUNKS || np > 64u * CH) continue;   // k_analyze_wave's / k_analyze_huge's
        const uint32_t i = wf(wc, WI_I), po = wf(wc, WI_PO), mdb = wf(wc, WI_MDB), dmz = wf(wc, WI_DMZ);
        const uint32_t flags = wf(wc, WI_FLAGS), ft = wf(wc, WI_FT);
        uint32_t off[NFEAT], cnt[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) { off[f] = wf(wc, WI_OFF + f); cnt[f] = wf(wc, WI_CNT + f); }
        if (flags & 7u) slow_lookups(P, i, wf(wc, WI_ENTRY), flags, nbuf, ub, off, cnt, lane);
        w_prior += np;
        uint32_t anylong = 0;
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) {
            w_upd += cnt[f] & ~MFP_UPD_SERIAL;
            anylong |= (cnt[f] & ~MFP_UPD_SERIAL) > 64 ? 1u : 0u;
        }
        mfp_update u[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) {
            u[f].idx = 0; u[f].value = 0.0;
            if (lane < (cnt[f] & ~MFP_UPD_SERIAL)) u[f] = D.upd[off[f] + lane];
        }
        uint64_t malbits = 0;   // one bit per chunk (CH <= 64)
#pragma unroll
        for (int c = 0; c < CH; c++) {
            const uint32_t pi = (uint32_t)c * 64 + lane;
            if ((uint32_t)c * 64 < np) {
                scl[pi] = pi < np ? D.prior[po + pi] : 0.0;
                if (pi < np && D.proc_mal[po + pi]) malbits |= 1ull << c;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) scatter_list(D, scl, off[f], cnt[f], u[f].idx, u[f].value, anylong, lane);
        double sc[CH];
#pragma unroll
        for (int c = 0; c < CH; c++) sc[c] = (uint32_t)c * 64 < np ? scl[c * 64 + lane] : 0.0;
        __builtin_amdgcn_wave_barrier();
        double mx;
        uint32_t imx, isx;
        max_two<CH>(sc, np, lane, mx, imx, isx);
        const bool swap = mdb && dmz == imx && !D.proc_mal[po + isx];
        const uint32_t ibest = swap ? isx : imx;
        const uint32_t tags = rfl(D.proc_attr[po + ibest] & D.db_tags);
#pragma unroll
        for (int c = 0; c < CH; c++) {
            const uint32_t pi = (uint32_t)c * 64 + lane;
            if (pi < np) {
                scl[pi] = (double)expf_ref((float)(sc[c] - mx));
                uint32_t f = (uint32_t)((malbits >> c) & 1u);
                if (tags) f |= ((D.proc_attr[po + pi] & tags) >> MFP_ATTR_DB_FIRST) << 1;
                if (swap && pi == imx) f |= 0x80u;
                fl[pi] = (uint8_t)f;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const double acc = row_sums(scl, fl, np, imx, tags ? 3u + MFP_ATTR_DB_TAGS : 3u, lane);
        double ssum = lane_d(acc, 0), swo = lane_d(acc, 1), mal = lane_d(acc, 2);
        const double p_imx = scl[imx], p_isx = scl[isx];
        double ap = 0.0;
        if (tags) {
#pragma unroll
            for (int k = 0; k < MFP_ATTR_DB_TAGS; k++) {
                const double v = lane_d(acc, 3 + k);
                if ((int)lane == k) ap = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
        double max_score = p_imx;
        if (ssum > 0.0 && mdb) mal /= ssum;
        if (swap) {
            ssum = swo;
            max_score = p_isx;
        }
        if (ssum > 0.0) max_score /= ssum;
        if (tags && P.attr_prob && lane < MFP_ATTR_DB_TAGS && ((tags >> (MFP_ATTR_DB_FIRST + lane)) & 1u))
            P.attr_prob[(uint64_t)i * MFP_ATTR_DB_TAGS + lane] = ssum > 0.0 ? ap / ssum : ap;
        if (lane == 0) {
            mfp_analysis a = P.out[i];   // status, pending flag and the additional attributes from k_analyze
            a.score = max_score;
            a.process = D.proc_id[po + ibest];
            a.proc_slot = po + ibest;
            a.attr = (uint16_t)(D.proc_attr[po + ibest] | a.attr | (flags >> 16));
            a.malware_prob = -1.0;
            a.flags = (uint8_t)(MFP_AN_VALID | (a.flags & MFP_AN_PENDING));
            if (mdb) {
                a.malware_prob = mal;
                a.flags |= MFP_AN_CLASSIFY_MALWARE;
                if (D.proc_mal[po + ibest]) a.flags |= MFP_AN_MALWARE;
            }
            if ((a.flags & MFP_AN_MALWARE) && ft == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
            P.out[i] = a;
        }
        __builtin_amdgcn_wave_barrier();
    }
    }
    if (lane == 0 && w_prior) atomicAdd(&P.stats[6], (unsigned long long)w_prior);
    if (lane == 0 && w_upd) atomicAdd(&P.stats[7], (unsigned long long)w_upd);
}

constexpr int WW = 4;   // waves per k_analyze_wave block
#ifndef MFP_AN_WAVE_MINW
#define MFP_AN_WAVE_MINW 4
#endif
__global__ __launch_bounds__(64 * WW, MFP_AN_WAVE_MINW) void k_analyze_wave(AParams P) {
    __shared__ char sni_buf[WW][336];
    __shared__ char ua_buf[WW][520];
    __shared__ double sc_lds[WW][64 * MAXP_CHUNKS];
    __shared__ uint32_t at_lds[WW][64 * MAXP_CHUNKS];   // per process: attribute bits
    __shared__ uint32_t id_lds[WW][64 * MAXP_CHUNKS];   // per process: process id
    __shared__ uint8_t fl_lds[WW][64 * MAXP_CHUNKS];    // per process: malware (bit 0), archive tags (1-6), swapped out (7)
    wave_scorer_pipe(P, sni_buf, ua_buf, sc_lds, at_lds, id_lds, fl_lds);
}

__global__ __launch_bounds__(64) void k_analyze_big(AParams P) {
    __shared__ char sni_buf[336];
    __shared__ char ua_buf[520];
    __shared__ double sc_lds[64 * MAXP_CHUNKS_BIG];
    __shared__ uint8_t fl_lds[64 * MAXP_CHUNKS_BIG];
    wave_scorer_big<MAXP_CHUNKS_BIG>(P, sni_buf, ua_buf, sc_lds, fl_lds);
}

// ---- k_analyze_huge (P > 64 * MAXP_CHUNKS_BIG, any size): one wave per
// block, the packet's score row and its per-process flags in a per-wave HBM
// scratch row (P.hrow: HUGE_WAVES rows of P.hstride doubles, then as many
// rows of P.hstride flag bytes), the same operations in the same order as the
// other scorers
constexpr uint32_t HUGE_WAVES = 128;
ADEV void row_sync() {   // the wave's global row writes visible to its other lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// max (first index of the largest) over row[0, np) without index `skip`
ADEV void row_max(const double *row, uint32_t np, uint32_t skip, uint32_t lane, double &mx, uint32_t &im) {
    mx = -1.7976931348623157e308;
    im = 0xffffffffu;
    for (uint32_t p = lane; p < np; p += 64) {
        const double v = row[p];
        if (p != skip && (im == 0xffffffffu || v > mx)) { mx = v; im = p; }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const double om = __shfl_xor(mx, d, 64);
        const uint32_t oi = (uint32_t)__shfl_xor((int)im, d, 64);
        if (oi != 0xffffffffu && (im == 0xffffffffu || om > mx || (om == mx && oi < im))) { mx = om; im = oi; }
    }
    im = rfl(im);
    mx = __hiloint2double((int)rfl((uint32_t)(__double_as_longlong(mx) >> 32)), (int)rfl((uint32_t)__double_as_longlong(mx)));
}
__global__ __launch_bounds__(64) void k_analyze_huge(AParams P) {
    __shared__ char nbuf[336];
    __shared__ char ub[520];
    const uint32_t lane = lane_id();
    const mfp_classifier_dev &D = P.D;
    double *row = P.hrow + (uint64_t)blockIdx.x * P.hstride;
    uint8_t *fl = (uint8_t *)(P.hrow + (uint64_t)HUGE_WAVES * P.hstride) + (uint64_t)blockIdx.x * P.hstride;
    uint64_t w_prior = 0, w_upd = 0;
    for (uint64_t sg = blockIdx.x; sg < P.nseg; sg += gridDim.x) {
    const WItem *dseg = P.deferred + sg * P.seg_cap;
    const uint32_t total = rfl(P.seg_n[3 * sg + 2]);
    for (uint32_t q = 0; q < total; q++) {
        const uint32_t wc = wi_load(dseg, q, total, lane);
        const uint32_t np = wf(wc, WI_NP);
        if (np <= 64u * MAXP_CHUNKS_BIG || np > P.hstride) continue;   // the other scorers'
        const uint32_t i = wf(wc, WI_I), po = wf(wc, WI_PO), mdb = wf(wc, WI_MDB), dmz = wf(wc, WI_DMZ);
        const uint32_t flags = wf(wc, WI_FLAGS), ft = wf(wc, WI_FT);
        uint32_t off[NFEAT], cnt[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) { off[f] = wf(wc, WI_OFF + f); cnt[f] = wf(wc, WI_CNT + f); }
        if (flags & 7u) slow_lookups(P, i, wf(wc, WI_ENTRY), flags, nbuf, ub, off, cnt, lane);
        w_prior += np;
        for (uint32_t p = lane; p < np; p += 64) row[p] = D.prior[po + p];
        row_sync();
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) {
            const uint32_t c = cnt[f] & ~MFP_UPD_SERIAL;
            w_upd += c;
            if (cnt[f] & MFP_UPD_SERIAL) {          // repeated processes: one entry after the other
                for (uint32_t k = 0; k < c; k++) {
                    if (lane == 0) { const mfp_update x = D.upd[off[f] + k]; row[x.idx] += x.value; }
                    row_sync();
                }
            } else {                                // a list names each process at most once
                for (uint32_t b = 0; b < c; b += 64) {
                    if (b + lane < c) { const mfp_update x = D.upd[off[f] + b + lane]; row[x.idx] += x.value; }
                    row_sync();
                }
            }
        }
        double mx, sx;
        uint32_t imx, isx;
        row_max(row, np, 0xffffffffu, lane, mx, imx);
        row_max(row, np, imx, lane, sx, isx);
        if (isx == 0xffffffffu) isx = 0;
        const bool swap = mdb && dmz == imx && !D.proc_mal[po + isx];
        const uint32_t ibest = swap ? isx : imx;
        const uint32_t tags = rfl(D.proc_attr[po + ibest] & D.db_tags);
        for (uint32_t p = lane; p < np; p += 64) {
            const double e = (double)expf_ref((float)(row[p] - mx));
            uint32_t f = D.proc_mal[po + p] ? 1u : 0u;
            if (tags) f |= ((D.proc_attr[po + p] & tags) >> MFP_ATTR_DB_FIRST) << 1;
            if (swap && p == imx) f |= 0x80u;
            row[p] = e;
            fl[p] = (uint8_t)f;
        }
        row_sync();
        const double acc = row_sums(row, fl, np, imx, tags ? 3u + MFP_ATTR_DB_TAGS : 3u, lane);
        double ssum = lane_d(acc, 0), swo = lane_d(acc, 1), mal = lane_d(acc, 2);
        const double p_imx = row[imx], p_isx = row[isx];
        double ap = 0.0;
        if (tags) {
#pragma unroll
            for (int k = 0; k < MFP_ATTR_DB_TAGS; k++) {
                const double v = lane_d(acc, 3 + k);
                if ((int)lane == k) ap = v;
            }
        }
        double max_score = p_imx;
        if (ssum > 0.0 && mdb) mal /= ssum;
        if (swap) {
            ssum = swo;
            max_score = p_isx;
        }
        if (ssum > 0.0) max_score /= ssum;
        if (tags && P.attr_prob && lane < MFP_ATTR_DB_TAGS && ((tags >> (MFP_ATTR_DB_FIRST + lane)) & 1u))
            P.attr_prob[(uint64_t)i * MFP_ATTR_DB_TAGS + lane] = ssum > 0.0 ? ap / ssum : ap;
        if (lane == 0) {
            mfp_analysis a = P.out[i];
            a.score = max_score;
            a.process = D.proc_id[po + ibest];
            a.proc_slot = po + ibest;
            a.attr = (uint16_t)(D.proc_attr[po + ibest] | a.attr | (flags >> 16));
            a.malware_prob = -1.0;
            a.flags = (uint8_t)(MFP_AN_VALID | (a.flags & MFP_AN_PENDING));
            if (mdb) {
                a.malware_prob = mal;
                a.flags |= MFP_AN_CLASSIFY_MALWARE;
                if (D.proc_mal[po + ibest]) a.flags |= MFP_AN_MALWARE;
            }
            if ((a.flags & MFP_AN_MALWARE) && ft == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
            P.out[i] = a;
        }
        row_sync();   // the row is rewritten by the next packet
    }
    }
    if (lane == 0 && w_prior) atomicAdd(&P.stats[6], (unsigned long long)w_prior);
    if (lane == 0 && w_upd) atomicAdd(&P.stats[7], (unsigned long long)w_upd);
}

// k_seen_scan: the batch's unknown-TLS sightings per distinct fingerprint
// (first and last stream position, count) in the sighting table the host
// decides from (mfp_prevalence.cpp).  Each block takes a contiguous range of
// 64-packet groups and aggregates its sightings in an LDS table (one LDS
// update per distinct fingerprint per group); the block then merges its
// entries into the global table: one insertion per new fingerprint, a
// min / max only when it improves the stored one, one count addition.  The
// distinct fingerprints of a group are found with ballots first, then their
// leader lanes update the table together.  A few
// hundred hot fingerprints thus see one global update per block, not one per
// group (global atomics on a handful of lines serialise at the memory side).
constexpr int SEEN_LDS = 2048;     // LDS table entries per block (power of two)
constexpr int SEEN_WPB = 4;        // waves per block

// merge one aggregated entry into the global table (insertion keeps its
// position in the distinct list for k_seen_export)
ADEV void seen_merge(const mfp_seen_tab &T, uint64_t h, uint32_t first, uint32_t last, uint32_t cnt) {
    uint64_t k = h & T.mask;
    for (uint32_t t = 0; t <= T.mask; t++, k = (k + 1) & T.mask) {
        mfp_seen_slot &sl = T.slots[k];
        unsigned long long cur = __hip_atomic_load(&sl.hash, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == ~0ull) {
            cur = atomicCAS(&sl.hash, ~0ull, (unsigned long long)h);
            if (cur == ~0ull) {                      // new in this batch: a position in the distinct list
                const unsigned int pos = atomicAdd(&T.counters[0], 1u);
                if (pos < T.list_cap) T.list[pos] = (uint32_t)k;
                else atomicExch(&T.counters[1], 1u);
                cur = h;
            }
        }
        if (cur == h) {                              // (slots start all-ones: min, min of ~last, count - 1)
            if (__hip_atomic_load(&sl.first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > first)
                atomicMin(&sl.first, first);
            if (__hip_atomic_load(&sl.nlast, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > ~last)
                atomicMin(&sl.nlast, ~last);
            atomicAdd(&sl.count_m1, cnt);
            return;
        }
    }
    atomicExch(&T.counters[1], 1u);                  // table full
}

__global__ __launch_bounds__(64 * SEEN_WPB) void k_seen_scan(AParams P) {
    __shared__ unsigned long long lh[SEEN_LDS];
    __shared__ unsigned int lfirst[SEEN_LDS], lnlast[SEEN_LDS], lcnt[SEEN_LDS];
    const uint32_t lane = lane_id();
    const uint32_t wid = threadIdx.x >> 6;
    uint32_t merges = 0;   // HBM sighting-slot updates (mfp_analysis_counters [11])
    for (int k = threadIdx.x; k < SEEN_LDS; k += 64 * SEEN_WPB) {
        lh[k] = ~0ull; lfirst[k] = ~0u; lnlast[k] = ~0u; lcnt[k] = 0;
    }
    __syncthreads();
    const uint64_t ngroups = (P.n + 63) / 64;
    const uint64_t per = (ngroups + gridDim.x - 1) / gridDim.x;
    const uint64_t g0 = (uint64_t)blockIdx.x * per, g1 = g0 + per < ngroups ? g0 + per : ngroups;
    // 64 groups per wave round: lane l reads group g + l's bitmap word
    for (uint64_t gb = g0 + 64 * wid; gb < g1; gb += 64 * SEEN_WPB) {
        const uint64_t gl = gb + lane;
        const uint64_t pw = gl < g1 ? P.pend_bits[gl] : 0ull;
        uint64_t todo = __ballot(pw != 0);
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint64_t g = gb + (uint64_t)j;
            const uint64_t pm = rl64(pw, j);
            const bool pending = (pm >> lane) & 1;
            const uint64_t i = g * 64 + lane;
            uint64_t fh = 0;
            if (pending) { const mfp_record r = P.rec[i]; fh = fp_key(r, P.fp_arena + r.fp_offset, r.fp_len); }
            // the group's distinct fingerprints: the lowest lane of each is its
            // leader and carries first / last / count (ballots only) ...
            uint64_t left = pm;
            bool lead = false;
            uint32_t fi = 0, la = 0, c = 0;
            while (left) {
                const int l0 = __builtin_ctzll(left);
                const uint64_t h0 = rl64(fh, l0);
                const uint64_t same = __ballot(pending && fh == h0) & left;
                left &= ~same;
                if ((int)lane == l0) {
                    lead = true;
                    fi = (uint32_t)(g * 64 + (uint64_t)__builtin_ctzll(same));
                    la = (uint32_t)(g * 64 + 63 - (uint64_t)__builtin_clzll(same));
                    c = (uint32_t)__builtin_popcountll(same);
                }
            }
            // ... then the leaders update the LDS table side by side (one update
            // per distinct fingerprint of the group, their latencies overlapped)
            if (lead) {
                uint32_t k = (uint32_t)fh & (SEEN_LDS - 1);
                bool done = false;
                for (int t = 0; t < 32; t++, k = (k + 1) & (SEEN_LDS - 1)) {
                    const unsigned long long prev = atomicCAS(&lh[k], ~0ull, (unsigned long long)fh);
                    if (prev == ~0ull || prev == fh) {
                        atomicMin(&lfirst[k], fi);
                        atomicMin(&lnlast[k], ~la);
                        atomicAdd(&lcnt[k], c);
                        done = true;
                        break;
                    }
                }
                if (!done) { seen_merge(P.seen, fh, fi, la, c); merges++; }   // the block's table is crowded: straight to HBM
            }
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < SEEN_LDS; k += 64 * SEEN_WPB)
        if (lh[k] != ~0ull) { seen_merge(P.seen, lh[k], lfirst[k], ~lnlast[k], lcnt[k]); merges++; }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) merges += __shfl_xor(merges, d, 64);
    if (lane == 0 && merges) atomicAdd(&P.stats[11], (unsigned long long)merges);
}

// k_seen_export: the batch's distinct unknown-TLS fingerprints, in the order
// they were first inserted (the host sorts them by first sighting)
__global__ __launch_bounds__(256) void k_seen_export(mfp_seen_tab T, mfp_sighting *out) {
    const uint32_t u = T.counters[0] < T.list_cap ? T.counters[0] : T.list_cap;
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < u; p += gridDim.x * 256) {
        mfp_seen_slot &sl = T.slots[T.list[p]];
        sl.pos = p;
        mfp_sighting o;
        o.hash = sl.hash; o.first = sl.first; o.last = ~sl.nlast; o.count = sl.count_m1 + 1u; o.first_seen = 0;
        out[p] = o;
    }
}

// k_seen_sequence: every sighting's fingerprint hash in stream order (the
// host's exact LRU simulation when the distinct form cannot be exact);
// group_off[g] = sightings before group g
__global__ __launch_bounds__(256) void k_seen_sequence(AParams P, const uint32_t *group_off, uint64_t *seq) {
    const uint64_t ngroups = (P.n + 63) / 64;
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups; g += (uint64_t)gridDim.x * 256) {
        uint32_t r = group_off[g];
        for (uint64_t w = P.pend_bits[g]; w; w &= w - 1) {
            const uint32_t i = (uint32_t)(g * 64 + (uint64_t)__builtin_ctzll(w));
            const mfp_record rc = P.rec[i];
            seq[r++] = fp_key(rc, P.fp_arena + rc.fp_offset, rc.fp_len);
        }
    }
}

// k_analyze_resolve: the unknown-TLS statuses the host decided.  A sighting
// stays "randomized" (classified with the randomized entry, if any) when it
// was not in the LRU; every other one becomes "unlabeled" (no process).
//   seen_pos != nullptr: per distinct fingerprint (distinct form): randomized
//     iff it is the fingerprint's first sighting and seen_pos[pos] == 0;
//   else per sighting in stream order: seen_seq[group_off[g] + rank] == 0.
__global__ __launch_bounds__(256) void k_analyze_resolve(AParams P, const uint8_t *seen_pos, const uint32_t *group_off,
                                                         const uint8_t *seen_seq) {
    // lane per packet: a wave takes one group of 64, its sightings side by
    // side (the sequence path's position = the group's offset + the
    // sighting's rank in the group)
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t ngroups = (P.n + 63) / 64;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < ngroups; g += (uint64_t)gridDim.x * 4) {
        const uint64_t w = P.pend_bits[g];
        if (!((w >> lane) & 1)) continue;
        const uint32_t i = (uint32_t)(g * 64 + lane);
        mfp_analysis a = P.out[i];
        const mfp_record rc = P.rec[i];
        bool seen;
        if (seen_pos) {
            const uint64_t h = fp_key(rc, P.fp_arena + rc.fp_offset, rc.fp_len);
            uint64_t k = h & P.seen.mask;
            seen = true;
            for (uint32_t t = 0; t <= P.seen.mask; t++, k = (k + 1) & P.seen.mask) {
                const mfp_seen_slot &sl = P.seen.slots[k];
                if (sl.hash == h) { seen = !(sl.first == i && seen_pos[sl.pos] == 0); break; }
                if (sl.hash == ~0ull) break;
            }
        } else {
            seen = seen_seq[group_off[g] + (uint32_t)__builtin_popcountll(w & ((1ull << lane) - 1))] != 0;
        }
        a.flags &= (uint8_t)~MFP_AN_PENDING;
        if (seen) {   // unlabeled: no process, no faketls; encrypted_dns / domain_faking stay
            a.status = 3;
            a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.proc_slot = MFP_NO_PROCESS;
            a.attr &= (uint16_t)((1u << P.D.doh_idx) | (1u << P.D.domain_faking_idx));
            a.flags = MFP_AN_VALID;
        }
        if (P.mode == MFP_MODE_ANALYSIS && (rc.flags & MFP_FLAG_TRUNCATED)) a.status = 3;   // pkt_proc.cc:1716-1719
        P.out[i] = a;
    }
}

}  // namespace mfpa

static mfpa::AParams make_params(const mfp_classifier_dev *D, const mfp_seen_tab &T, const uint8_t *arena,
                                 const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, const uint8_t *fp_arena,
                                 mfp_analysis *out, uint32_t *pending, void *deferred, unsigned long long *stats,
                                 uint32_t mode, uint32_t lane_max_p) {
    mfpa::AParams P;
    P.D = *D;
    P.seen = T;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.out = out; P.mode = mode;
    P.attr_prob = nullptr;
    P.pend_bits = (uint64_t *)pending;
    P.deferred = (mfpa::WItem *)deferred;
    P.lane_max_p = lane_max_p;
    P.stats = stats;
    P.hrow = nullptr;
    P.hstride = 0;
    return P;
}

// bytes of k_analyze_huge's scratch rows for an archive whose largest
// fingerprint has max_nproc processes (0: the kernel is not needed)
extern "C" size_t mfp_analysis_huge_bytes(uint32_t max_nproc) {
    if (max_nproc <= 64u * mfpa::MAXP_CHUNKS_BIG) return 0;
    const size_t stride = (max_nproc + 63u) & ~63u;
    return (size_t)mfpa::HUGE_WAVES * stride * 9;
}

// blocks of the per-segment kernels (k_analyze, k_an_features: AW segments per
// block, equal work each) at most: a whole number of resident rounds of both, so
// neither's last round leaves CUs idle (5 and 4 blocks per CU on 256 CUs: 5120;
// the flat 2048 was 1.6 rounds of k_analyze).  MFP_GRID_ROUND=0: 2048.
static uint64_t seg_block_cap() {
    static std::atomic<uint64_t> cap_cache[64];
    const uint64_t cap = (uint64_t)mfp_per_device(cap_cache, [] {
        const char *e = getenv("MFP_GRID_ROUND");
        if (e && e[0] == '0') return (uint64_t)2048;
        int dev = 0, cus = 0, a = 0, f = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, mfpa::k_analyze, 64 * mfpa::AW, 0) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&f, mfpa::k_an_features, 64 * mfpa::AW, 0) != hipSuccess ||
            cus <= 0 || a <= 0 || f <= 0) {
            (void)hipGetLastError();
            return (uint64_t)2048;
        }
        const uint64_t ra = (uint64_t)cus * (uint64_t)a, rf = (uint64_t)cus * (uint64_t)f;
        uint64_t x = ra, y = rf;
        while (y) { const uint64_t t = x % y; x = y; y = t; }
        uint64_t l = ra / x * rf;
        if (const char *r = getenv("MFP_SEG_ROUNDS")) l *= strtoul(r, nullptr, 10) ? strtoul(r, nullptr, 10) : 1;
        return l <= 32768 ? l : (uint64_t)2048;
    });
    return cap;
}

// k_an_score's grid: every block it can hold resident (10 per CU, LDS-bound:
// 5 waves per SIMD), over the segments with a stride; the flat 1024 ran it at 2
// waves per SIMD.  MFP_GRID_ROUND=0: 1024.
static uint32_t score_grid(uint32_t blocks) {
    static std::atomic<uint64_t> res_cache[64];
    const uint32_t res = (uint32_t)mfp_per_device(res_cache, [] {
        const char *e = getenv("MFP_GRID_ROUND");
        if (e && e[0] == '0') return 1024u;
        int dev = 0, cus = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, mfpa::k_an_score, 64 * mfpa::SW, 0) != hipSuccess ||
            cus <= 0 || nb <= 0) {
            (void)hipGetLastError();
            return 1024u;
        }
        return (uint32_t)(cus * nb);
    });
    return blocks < res ? blocks : res;
}

// k_seen_scan's grid: contiguous group ranges, one per block; every block the
// CUs hold (4 per CU, LDS-bound) once there are 256 groups per block, instead of
// one block per 1024 groups (763 blocks at 50 M packets: three quarters of the
// CUs).  MFP_GRID_ROUND=0: one block per 1024 groups, at most 1024.
static uint64_t seen_grid(uint64_t groups) {
    static std::atomic<uint64_t> res_cache[64];
    const uint64_t res = (uint64_t)mfp_per_device(res_cache, [] {
        const char *e = getenv("MFP_GRID_ROUND");
        if (e && e[0] == '0') return (uint64_t)0;
        int dev = 0, cus = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, mfpa::k_seen_scan, 64 * mfpa::SEEN_WPB, 0) != hipSuccess ||
            cus <= 0 || nb <= 0) {
            (void)hipGetLastError();
            return (uint64_t)0;
        }
        return (uint64_t)cus * (uint64_t)nb;
    });
    uint64_t sb = (groups + 1023) / 1024;
    if (sb > 1024) sb = 1024;
    if (res) {
        const uint64_t b = (groups + 255) / 256;
        sb = b < res ? b : res;
    }
    return sb ? sb : 1;
}

// the per-wave segments of one batch: k_analyze's waves (segments) and the
// items a segment holds at most (64 per group a wave can take)
extern "C" void mfp_analysis_segments(uint64_t n, uint32_t *nseg, uint32_t *seg_cap) {
    const uint64_t groups = (n + 63) / 64;
    uint64_t blocks = (groups + mfpa::AW - 1) / mfpa::AW;
    const uint64_t cap = seg_block_cap();
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    const uint64_t ns = blocks * mfpa::AW;
    *nseg = (uint32_t)ns;
    *seg_cap = (uint32_t)(64 * ((groups + ns - 1) / ns));
}

// scratch: work = nseg * seg_cap WorkItems (16 B), lanel = nseg * seg_cap
// Deferred (64 B), deferred = nseg * seg_cap WItems (80 B), seg_n = 3 * nseg words
extern "C" int mfp_launch_analysis(const mfp_classifier_dev *D, const mfp_seen_tab *T, const uint8_t *arena,
                                   const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, const uint8_t *fp_arena,
                                   mfp_analysis *out, double *attr_prob, uint32_t *pending, void *work, void *lanel,
                                   void *deferred, uint32_t *seg_n, unsigned long long *stats, uint32_t mode,
                                   uint32_t lane_max_p, void *huge_rows, hipStream_t stream, mfp_prof *prof) {
    if (n == 0) return 0;
    // T == nullptr: no sighting table (a small batch decided on the host from
    // its records, mfp_process_small_pinned): k_seen_scan is not launched
    const mfp_seen_tab none{};
    mfpa::AParams P = make_params(D, T ? *T : none, arena, desc, n, rec, fp_arena, out, pending, deferred, stats, mode,
                                  lane_max_p);
    P.attr_prob = attr_prob;
    P.work = (mfpa::WorkItem *)work;
    P.lanel = (mfpa::Deferred *)lanel;
    P.seg_n = seg_n;
    mfp_analysis_segments(n, &P.nseg, &P.seg_cap);
    const uint32_t blocks = P.nseg / mfpa::AW;
    const uint64_t groups = (n + 63) / 64;
    if (prof) mfp_prof_begin(prof, "k_analyze", stream);
    hipLaunchKernelGGL(mfpa::k_analyze, dim3(blocks), dim3(64 * mfpa::AW), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    if (hipGetLastError() != hipSuccess) return -1;
    if (T) {
        const uint64_t sb = seen_grid(groups);
        if (prof) mfp_prof_begin(prof, "k_seen_scan", stream);
        hipLaunchKernelGGL(mfpa::k_seen_scan, dim3((uint32_t)sb), dim3(64 * mfpa::SEEN_WPB), 0, stream, P);
        if (prof) mfp_prof_end(prof, stream);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (prof) mfp_prof_begin(prof, "k_an_features", stream);
    hipLaunchKernelGGL(mfpa::k_an_features, dim3(blocks), dim3(64 * mfpa::AW), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    if (hipGetLastError() != hipSuccess) return -1;
    if (prof) mfp_prof_begin(prof, "k_an_score", stream);
    hipLaunchKernelGGL(mfpa::k_an_score, dim3(score_grid(blocks)), dim3(64 * mfpa::SW), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    if (hipGetLastError() != hipSuccess) return -1;
    if (prof) mfp_prof_begin(prof, "k_analyze_wave", stream);
    hipLaunchKernelGGL(mfpa::k_analyze_wave, dim3(blocks < 1024 ? blocks : 1024), dim3(256), 0, stream, P);
    if (D->max_nproc > 64u * mfpa::MAXP_CHUNKS)
        hipLaunchKernelGGL(mfpa::k_analyze_big, dim3(256), dim3(64), 0, stream, P);
    if (D->max_nproc > 64u * mfpa::MAXP_CHUNKS_BIG) {
        if (!huge_rows) return -1;
        P.hrow = (double *)huge_rows;
        P.hstride = (D->max_nproc + 63u) & ~63u;
        hipLaunchKernelGGL(mfpa::k_analyze_huge, dim3(mfpa::HUGE_WAVES), dim3(64), 0, stream, P);
    }
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfp_launch_seen_export(const mfp_seen_tab *T, uint32_t u, mfp_sighting *out, hipStream_t stream) {
    if (u == 0) return 0;
    const uint32_t blocks = (u + 255) / 256 < 1024 ? (u + 255) / 256 : 1024;
    hipLaunchKernelGGL(mfpa::k_seen_export, dim3(blocks), dim3(256), 0, stream, *T, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfp_launch_seen_sequence(const mfp_classifier_dev *D, const mfp_seen_tab *T, uint64_t n,
                                        const mfp_record *rec, const uint8_t *fp_arena, uint32_t *pending,
                                        const uint32_t *group_off, uint64_t *seq, hipStream_t stream) {
    if (n == 0) return 0;
    mfpa::AParams P = make_params(D, *T, nullptr, nullptr, n, (mfp_record *)rec, fp_arena, nullptr, pending, nullptr,
                                  nullptr, 0, 0);
    uint64_t groups = (n + 63) / 64, blocks = (groups + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(mfpa::k_seen_sequence, dim3((uint32_t)blocks), dim3(256), 0, stream, P, group_off, seq);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfp_launch_analysis_resolve(const mfp_classifier_dev *D, const mfp_seen_tab *T, uint64_t n,
                                           const mfp_record *rec, const uint8_t *fp_arena, mfp_analysis *out,
                                           uint32_t *pending, uint32_t mode, const uint8_t *seen_pos,
                                           const uint32_t *group_off, const uint8_t *seen_seq, hipStream_t stream,
                                           mfp_prof *prof) {
    if (n == 0) return 0;
    mfpa::AParams P = make_params(D, *T, nullptr, nullptr, n, (mfp_record *)rec, fp_arena, out, pending, nullptr,
                                  nullptr, mode, 0);
    uint64_t groups = (n + 63) / 64, blocks = (groups + 3) / 4;   // a wave per group of 64 packets
    if (blocks > 8192) blocks = 8192;
    if (prof) mfp_prof_begin(prof, "k_analyze_resolve", stream);
    hipLaunchKernelGGL(mfpa::k_analyze_resolve, dim3((uint32_t)blocks), dim3(256), 0, stream, P, seen_pos, group_off,
                       seen_seq);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
