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

constexpr int MAXP_CHUNKS = 8;     // up to 512 processes per fingerprint

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
ADEV Hit probe_feature(const mfp_classifier_dev &D, uint32_t entry, uint32_t kind, uint64_t key, const uint8_t *s,
                       uint32_t len, bool verify, uint32_t lane) {
    for (uint64_t k = feat_slot_hash(entry, kind, key) & D.feat_mask;; k = (k + 1) & D.feat_mask) {
        const mfp_feat_slot sl = D.feat_slots[k];
        const uint32_t e = rfl(sl.entry);
        if (e == 0xffffffffu) return Hit{0, 0};
        if (e == entry && rfl(sl.kind) == kind && rfl64(sl.key) == key) {
            if (!verify || (rfl(sl.str_len) == len && wave_eq(s, (const uint8_t *)D.pool + rfl(sl.str_off), len, lane)))
                return Hit{rfl(sl.upd_off), rfl(sl.upd_cnt)};
        }
    }
}

ADEV uint32_t asn_v4(const mfp_classifier_dev &D, uint32_t addr_host) {
    int lo = 0, hi = (int)D.n_asn4 - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        const uint32_t a = rfl(D.asn4[mid].lo), b = rfl(D.asn4[mid].hi);
        if (addr_host < a) hi = mid - 1;
        else if (addr_host > b) lo = mid + 1;
        else return rfl(D.asn4[mid].asn);
    }
    return 0;
}
ADEV bool le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) { return ah < bh || (ah == bh && al <= bl); }
ADEV uint32_t asn_v6(const mfp_classifier_dev &D, uint64_t xh, uint64_t xl) {
    int lo = 0, hi = (int)D.n_asn6 - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        const mfp_asn6 r = D.asn6[mid];
        const uint64_t ah = rfl64(r.lo_hi), al = rfl64(r.lo_lo), bh = rfl64(r.hi_hi), bl = rfl64(r.hi_lo);
        if (!le128(ah, al, xh, xl)) hi = mid - 1;
        else if (!le128(xh, xl, bh, bl)) lo = mid + 1;
        else return rfl(r.asn);
    }
    return 0;
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
constexpr int LB = 8;   // words per batch

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

ADEV bool lane_eq(const uint8_t *a, const uint8_t *b, uint32_t len) {
    for (uint32_t j0 = 0; 8 * j0 < len; j0 += LB) {
        uint64_t x[LB], y[LB];
        load_words<LB>(a, len, j0, x);
        load_words<LB>(b, len, j0, y);
        bool same = true;
#pragma unroll
        for (int k = 0; k < LB; k++) same &= x[k] == y[k];
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
ADEV bool cand_feature_lane(const mfp_classifier_dev &D, uint32_t entry, uint32_t kind, uint64_t key, uint32_t len,
                            Hit &hit, uint32_t &str_off) {
    for (uint64_t k = feat_slot_hash(entry, kind, key) & D.feat_mask;; k = (k + 1) & D.feat_mask) {
        const mfp_feat_slot sl = D.feat_slots[k];
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
ADEV Hit probe_feature_lane(const mfp_classifier_dev &D, uint32_t entry, uint32_t kind, uint64_t key,
                            const uint8_t *s, uint32_t len) {
    for (uint64_t k = feat_slot_hash(entry, kind, key) & D.feat_mask;; k = (k + 1) & D.feat_mask) {
        const mfp_feat_slot sl = D.feat_slots[k];
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

ADEV uint32_t asn_v4_lane(const mfp_classifier_dev &D, uint32_t addr_host) {
    int lo = 0, hi = (int)D.n_asn4 - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const mfp_asn4 r = D.asn4[mid];
        if (addr_host < r.lo) hi = mid - 1;
        else if (addr_host > r.hi) lo = mid + 1;
        else return r.asn;
    }
    return 0;
}
ADEV uint32_t asn_v6_lane(const mfp_classifier_dev &D, uint64_t xh, uint64_t xl) {
    int lo = 0, hi = (int)D.n_asn6 - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const mfp_asn6 r = D.asn6[mid];
        if (!le128(r.lo_hi, r.lo_lo, xh, xl)) hi = mid - 1;
        else if (!le128(xh, xl, r.hi_hi, r.hi_lo)) lo = mid + 1;
        else return r.asn;
    }
    return 0;
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

// a packet k_analyze hands to k_analyze_wave, with its feature lookups done
struct Deferred {
    uint32_t i, entry, slow_sni, pad;   // slow_sni: domain / SNI lookups still to do
    uint32_t off[6], cnt[6];
};

struct AParams {
    mfp_classifier_dev D;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    const uint8_t *fp_arena;
    mfp_analysis *out;
    uint64_t *pend_bits;         // per group of 64 packets: unknown-TLS sightings (k_analyze_resolve)
    mfp_seen_tab seen;           // this batch's sightings per distinct fingerprint
    struct Deferred *deferred;   // packets scored by k_analyze_wave
    uint32_t mode;
    uint32_t lane_max_p;         // phase L takes fingerprints with P <= min(lane_max_p, PL)
    unsigned long long *stats;   // [0] analyzed, [1] pending unknown-TLS, [2] over-size P, [3] deferred
};

constexpr uint32_t NFEAT = 6;    // ASN, port, IP, UA, domain, SNI: naive_bayes.hpp:752-772 order

// k_analyze, in two phases per group of 64 fingerprint records:
//  A. lane per packet (64 packets in flight per wave): fingerprint hash,
//     verified fingerprint-table lookup and status, destination context,
//     ASN, server-name normalisation (plain names; the rest are marked for
//     phase B) and the six feature-table lookups -> per lane: entry and six
//     (update list offset, count) pairs;
//  B. wave per scored packet: prior + update lists loaded lane-parallel,
//     applied feature by feature as LDS scatters (one update per process per
//     list, so a feature is one conflict-free scatter and each process sees
//     the reference's addition order), max / second max, fp32 softmax, result.
#ifndef MFP_AN_PL
#define MFP_AN_PL 16
#endif
#ifndef MFP_AN_MINW
#define MFP_AN_MINW 4
#endif
constexpr uint32_t PL = MFP_AN_PL;   // phase L: fingerprints with at most PL processes, scored lane per packet
constexpr int AW = 2;                // waves per k_analyze block (LDS: PL * 512 bytes of score rows per wave)

__global__ __launch_bounds__(64 * AW, MFP_AN_MINW) void k_analyze(AParams P) {
    __shared__ double sc_lds[AW][64 * PL];   // per wave: phase L's lane-private score rows S[p][lane]
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    double *scl = sc_lds[wid];
    const mfp_classifier_dev &D = P.D;
    const uint64_t ngroups = (P.n + 63) / 64;
    const uint64_t nw = (uint64_t)gridDim.x * AW;
    uint32_t n_an = 0, n_pend = 0;   // per-wave counts, one atomic each at the end
    for (uint64_t g = (uint64_t)blockIdx.x * AW + wid; g < ngroups; g += nw) {
        const uint64_t i = g * 64 + lane;
        const bool live = i < P.n;
        mfp_record r;
        if (live) r = P.rec[i];
        else { r.fp_len = 0; r.fp_type = 0; r.flags = 0; }
        mfp_analysis a;   // default: no information (analysis_result())
        a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0; a.status = 0; a.flags = 0;
        // messages whose do_analysis calls the classifier: TLS ClientHello
        // (tls.h:1977), HTTP request (http.cc:571), SSH client KEXINIT
        // (ssh.h:480); their type must also be in the archive (fp_types)
        const bool typed = live && r.fp_len != 0 && (r.fp_type == 1 || r.fp_type == 3 || r.fp_type == 5);
        const bool analyzable = typed && ((D.types_mask >> r.fp_type) & 1u);
        if (typed && !analyzable) { a.status = 4; a.flags = MFP_AN_VALID; }   // fingerprint_status_unanalyzed
        const uint64_t am = __ballot(analyzable);
        if (!am) {
            if (live) P.out[i] = a;
            if (lane == 0) P.pend_bits[g] = 0;
            continue;
        }
        n_an += (uint32_t)__builtin_popcountll(am);

        // ================= phase A: lane per packet =================
        uint32_t status = 0, entry = 0xffffffffu, np = 0, po = 0, mdb = 0, dmz = 0, mbits = 0;
        bool pending = false;
        uint32_t hoff[NFEAT], hcnt[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) { hoff[f] = 0; hcnt[f] = 0; }
        // ---- 1. fingerprint lookup / status (perform_analysis_common, analysis.h:1043-1083):
        // hash and candidate slot per lane, byte-exact check by the wave
        const uint8_t *fp = P.fp_arena + r.fp_offset;
        const uint32_t fl = analyzable ? r.fp_len : 0u;
        uint64_t fh = 0, w0 = 0;
        uint32_t cid = 0xffffffffu, coff = 0;
        if (analyzable) {
#ifdef MFP_PROBE_AN_NOHASH
            fh = fl;
#else
            fh = fp_key(r, fp, fl);
#endif
            w0 = word_at(fp, fl, 0);
            cid = cand_string_lane(D.fp_slots, D.fp_mask, fh, fl, coff);
        }
        {
            const bool ok = wave_verify(cid != 0xffffffffu, fp, (const uint8_t *)D.pool + coff, fl, lane);
            if (cid != 0xffffffffu && !ok) cid = probe_string_lane(D.fp_slots, D.fp_mask, D.pool, fp, fl, fh);
        }
        entry = cid;
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
        {   // unknown-TLS sightings of this group: the per-group bitmap, and the
            // batch table per distinct fingerprint (first / last sighting, count),
            // one set of atomics per distinct hash per wave
            const uint64_t pm = __ballot(pending);
            if (lane == 0) P.pend_bits[g] = pm;
            n_pend += (uint32_t)__builtin_popcountll(pm);
            uint64_t left = pm;
            while (left) {
                const int l0 = __builtin_ctzll(left);
                const uint64_t h0 = rl64(fh, l0);
                const uint64_t same = __ballot(pending && fh == h0) & left;
                left &= ~same;
                if ((int)lane == l0) {
                    const uint32_t i_first = (uint32_t)(g * 64 + (uint64_t)__builtin_ctzll(same));
                    const uint32_t i_last = (uint32_t)(g * 64 + 63 - (uint64_t)__builtin_clzll(same));
                    const mfp_seen_tab &T = P.seen;
                    uint64_t k = h0 & T.mask;
                    for (uint32_t t = 0; t <= T.mask; t++, k = (k + 1) & T.mask) {
                        const unsigned long long prev = atomicCAS(&T.slots[k].hash, ~0ull, (unsigned long long)h0);
                        if (prev == ~0ull) {             // new in this batch: a position in the distinct list
                            const unsigned int pos = atomicAdd(&T.counters[0], 1u);
                            if (pos < T.list_cap) T.list[pos] = (uint32_t)k;
                            else atomicExch(&T.counters[1], 1u);
                        }
                        if (prev == ~0ull || prev == h0) {      // (slots start all-ones: min, min of ~last, count - 1)
                            atomicMin(&T.slots[k].first, i_first);
                            atomicMin(&T.slots[k].nlast, ~i_last);
                            atomicAdd(&T.slots[k].count_m1, (unsigned int)__builtin_popcountll(same));
                            break;
                        }
                        if (t == T.mask) atomicExch(&T.counters[1], 1u);   // table full
                    }
                }
            }
        }
        bool scored = analyzable && entry != 0xffffffffu;
        if (scored) {
            const mfp_entry E = D.entry[entry];
            np = E.nproc; po = E.proc_off; mdb = E.malware_db; dmz = E.generic_dmz; mbits = E.mal_bits;
            if (np > 64 * MAXP_CHUNKS) {
                atomicAdd(&P.stats[2], 1ull);
                scored = false;
            }
        }
        bool plain = false;
        // string features UA, domain, SNI (hoff/hcnt slots 3..5)
        const uint8_t *vs[3] = {nullptr, nullptr, nullptr};
        uint32_t vl[3] = {0, 0, 0}, voff[3] = {0, 0, 0};
        uint64_t vk[3] = {0, 0, 0};
        Hit vh[3] = {Hit{0, 0}, Hit{0, 0}, Hit{0, 0}};
        bool has[3] = {false, false, false};
        if (scored) {
            // ---- 2. destination context (destination_context::init, result.h:346)
            const uint8_t *pkt = P.arena + P.desc[i].offset;
            const uint32_t ipv = (r.net >> 16) & 15, ipo = r.net & 0xffff;
            uint32_t asn = 0;
            uint64_t ipkey = 0, v6w0 = 0, v6w1 = 0;
            if (ipv == 4) {
                const uint32_t v4 = (uint32_t)word_at(pkt + ipo + 16, 4, 0);   // network order, as bytes
                asn = asn_v4_lane(D, __builtin_bswap32(v4));
                ipkey = normalize_ipv4(v4);
            } else if (ipv == 6) {
                v6w0 = word_at(pkt + ipo + 24, 16, 0);
                v6w1 = word_at(pkt + ipo + 24, 16, 1);
                if (D.n_asn6) asn = asn_v6_lane(D, __builtin_bswap64(v6w0), __builtin_bswap64(v6w1));
                // normalize_ipv6 (mfp_common.hpp) on the two words
                const bool gu = (v6w0 & 0xe0) == 0x20;
                const bool mapped = v6w0 == 0 && (v6w1 & 0xffffffffull) == 0xffff0000ull;
                if (!(gu || mapped)) { v6w0 = 0xfd; v6w1 = 1ull << 56; }
                ipkey = hash_final(word_term(v6w0, 0) ^ word_term(v6w1, 1), 16);
            }
            // server name: TLS SNI / HTTP Host (strncpy 256, NUL stops)
            const uint32_t sl = r.sni_len == 0xffff ? 0u : r.sni_len;
            const uint8_t *sp = pkt + r.sni_off;
            uint32_t tld = 0;
            uint64_t nh = 0;
            plain = plain_server_name(sp, sl, tld, nh);   // no NUL in a plain name
            // user agent (strncpy 511, NUL stops); TLS has none
            uint32_t ul = r.ua_len == 0xffff ? 0u : r.ua_len;
            if (ul > 511) ul = 511;
            const uint8_t *up = pkt + r.ua_off;
            uint64_t uh = 0;
            ul = cstr_hash(up, ul, uh);
            const uint32_t dport = r.dst_port;

            // ---- 3. the six feature lookups
            Hit h;
            h = probe_feature_lane(D, entry, F_ASN, asn, nullptr, 0xffffffffu);
            hoff[0] = h.off; hcnt[0] = h.cnt;
            h = probe_feature_lane(D, entry, F_PORT, dport, nullptr, 0xffffffffu);
            hoff[1] = h.off; hcnt[1] = h.cnt;
            if (ipv == 4) {
                h = probe_feature_lane(D, entry, F_IPV4, ipkey, nullptr, 0xffffffffu);
                hoff[2] = h.off; hcnt[2] = h.cnt;
            } else if (ipv == 6) {
                // the 16 normalized bytes, verified against the pool
                for (uint64_t k = feat_slot_hash(entry, F_IPV6, ipkey) & D.feat_mask;; k = (k + 1) & D.feat_mask) {
                    const mfp_feat_slot s6 = D.feat_slots[k];
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
            has[0] = cand_feature_lane(D, entry, F_UA, uh, ul, vh[0], voff[0]);
            if (plain) {   // else k_analyze_wave normalises the name (wave, LDS)
                vs[1] = sp + tld; vl[1] = sl - tld; vk[1] = lane_hash(sp + tld, sl - tld);
                has[1] = cand_feature_lane(D, entry, F_DOMAIN, vk[1], vl[1], vh[1], voff[1]);
                vs[2] = sp; vl[2] = sl; vk[2] = nh;
                has[2] = cand_feature_lane(D, entry, F_SNI, nh, sl, vh[2], voff[2]);
            }
        }

#pragma unroll
        for (int v = 0; v < 3; v++) {
            const bool ok = wave_verify(has[v], vs[v], (const uint8_t *)D.pool + voff[v], vl[v], lane);
            if (has[v]) {
                // a hash collision (ok == false) takes the full probe, which keeps looking
                const Hit h = ok ? vh[v] : probe_feature_lane(D, entry, v == 0 ? F_UA : v == 1 ? F_DOMAIN : F_SNI, vk[v],
                                                              vs[v], vl[v]);
                hoff[3 + v] = h.off; hcnt[3 + v] = h.cnt;
            }
        }

        // ================= phase L: lane per packet, P <= PL =================
        // the reference's own sequential loops (naive_bayes.hpp:752-772,
        // compute_score_and_probability analysis.h:222-277, softmax
        // softmax.hpp:227-264) on lane-private LDS rows
#ifdef MFP_PROBE_AN_NOSCORE
        const bool lanep = false;
#else
        const bool lanep = scored && np <= PL && np <= P.lane_max_p && plain;
#endif
        if (lanep) {
            double *S = scl + lane;                    // S[p * 64]
            for (uint32_t p = 0; p < np; p++) S[p * 64] = D.prior[po + p];
#pragma unroll
            for (uint32_t f = 0; f < NFEAT; f++) {
                const uint32_t c = hcnt[f] & ~MFP_UPD_SERIAL;
                const mfp_update *ul = D.upd + hoff[f];
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
            double ssum = 0.0, swo = 0.0, mal = 0.0, p_imx = 0.0, p_isx = 0.0;
            for (uint32_t p = 0; p < np; p++) {
                const double e = (double)expf((float)(S[p * 64] - mx));
                ssum += e;
                if (p != imx) swo += e;
                if ((mbits >> p) & 1u) mal += e;
                if (p == imx) p_imx = e;
                if (p == isx) p_isx = e;
            }
            double max_score = p_imx;
            if (ssum > 0.0 && mdb) mal /= ssum;
            uint32_t ibest = imx;
            if (mdb && dmz == imx && !((mbits >> isx) & 1u)) {
                ibest = isx;
                ssum = swo;
                max_score = p_isx;
            }
            if (ssum > 0.0) max_score /= ssum;
            a.score = max_score;
            a.process = D.proc_id[po + ibest];
            a.attr = (uint16_t)D.proc_attr[po + ibest];
            a.malware_prob = -1.0;
            a.flags = MFP_AN_VALID;
            if (mdb) {
                a.malware_prob = mal;
                a.flags |= MFP_AN_CLASSIFY_MALWARE;
                if ((mbits >> ibest) & 1u) a.flags |= MFP_AN_MALWARE;
            }
            if ((a.flags & MFP_AN_MALWARE) && r.fp_type == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();

        // ================= the rest: queued for k_analyze_wave =================
        {
            const bool defer = scored && !lanep;
            const uint64_t dm = __ballot(defer);
            if (dm) {
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(&P.stats[3], (unsigned long long)__builtin_popcountll(dm));
                base = rfl64(base);
                if (defer) {
                    Deferred &d = P.deferred[base + __builtin_popcountll(dm & ((1ull << lane) - 1))];
                    d.i = (uint32_t)i; d.entry = entry; d.slow_sni = plain ? 0u : 1u; d.pad = 0;
#pragma unroll
                    for (uint32_t f = 0; f < NFEAT; f++) { d.off[f] = hoff[f]; d.cnt[f] = hcnt[f]; }
                }
            }
        }
        if (analyzable) {
            if (!lanep) {   // no process distribution (yet: k_analyze_wave scores the deferred ones)
                a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0; a.flags = MFP_AN_VALID;
            }
            a.status = (uint8_t)status;
            if (pending) a.flags |= MFP_AN_PENDING;
            // analyze_ip_packet: a truncated message reports "unlabeled" and
            // keeps its classification (pkt_proc.cc:1716-1719)
            if (P.mode == MFP_MODE_ANALYSIS && (r.flags & MFP_FLAG_TRUNCATED) && !pending) a.status = 3;
        }
        if (live) P.out[i] = a;   // the status lives in the analysis record only (no 1-byte record rewrite)
    }
    if (lane == 0 && n_an) atomicAdd(&P.stats[0], (unsigned long long)n_an);
    if (lane == 0 && n_pend) atomicAdd(&P.stats[1], (unsigned long long)n_pend);
}

// k_analyze_wave: the packets k_analyze deferred (more than PL processes, or a
// server name that needs the full normalisation) -- one wavefront per packet,
// lane i holds process i (up to 64 * MAXP_CHUNKS processes).  Scores live in
// LDS: the prior and the first 64 updates of every list are loaded in one
// round trip, then the lists are applied feature by feature as lane-parallel
// scatters (a list names each process at most once, so every process sees the
// reference's addition order; lists flagged MFP_UPD_SERIAL go one by one).
__global__ __launch_bounds__(256) void k_analyze_wave(AParams P) {
    __shared__ char sni_buf[4][336];
    __shared__ double sc_lds[4][64 * MAXP_CHUNKS];
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    char *nbuf = sni_buf[wid];
    double *scl = sc_lds[wid];
    const mfp_classifier_dev &D = P.D;
    const uint64_t total = P.stats[3];
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t q = (uint64_t)blockIdx.x * 4 + wid; q < total; q += nw) {
        const Deferred &dq = P.deferred[q];
        const uint32_t i = rfl(dq.i), entry = rfl(dq.entry), slow = rfl(dq.slow_sni);
        uint32_t off[NFEAT], cnt[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) { off[f] = rfl(dq.off[f]); cnt[f] = rfl(dq.cnt[f]); }
        const mfp_entry E = D.entry[entry];
        const uint32_t np = rfl(E.nproc), po = rfl(E.proc_off), mdb = rfl(E.malware_db), dmz = rfl(E.generic_dmz);
        const uint32_t ft = rfl((uint32_t)P.rec[i].fp_type);
        if (slow) {
            // server name: full normalisation on lane 0 into LDS, hashed and
            // verified lane-parallel (strncpy 256, NUL stops)
            const mfp_record r = P.rec[i];
            const uint32_t sni = rfl((uint32_t)r.sni_off | ((uint32_t)r.sni_len << 16));
            const uint32_t sl = (sni >> 16) == 0xffff ? 0 : (sni >> 16);
            const uint8_t *sp = P.arena + P.desc[i].offset + (sni & 0xffff);
            int nlen = 0;
            if (lane == 0) nlen = normalize_server_name(sp, (int)sl, nbuf);
            nlen = (int)rfl((uint32_t)nlen);
            __builtin_amdgcn_wave_barrier();
            const int tld = (int)rfl((uint32_t)(lane == 0 ? tld_domain_offset(nbuf, nlen) : 0));
            const uint8_t *dom = (const uint8_t *)nbuf + tld;
            Hit h = probe_feature(D, entry, F_DOMAIN, wave_hash(dom, (uint32_t)(nlen - tld), lane), dom,
                                  (uint32_t)(nlen - tld), true, lane);
            off[4] = h.off; cnt[4] = h.cnt;
            h = probe_feature(D, entry, F_SNI, wave_hash((const uint8_t *)nbuf, (uint32_t)nlen, lane),
                              (const uint8_t *)nbuf, (uint32_t)nlen, true, lane);
            off[5] = h.off; cnt[5] = h.cnt;
            __builtin_amdgcn_wave_barrier();
        }
        // ---- scores: prior, then the six features in the reference's order
        uint32_t anylong = 0;
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) anylong |= (cnt[f] & ~MFP_UPD_SERIAL) > 64 ? 1u : 0u;
        mfp_update u[NFEAT];
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) {
            u[f].idx = 0; u[f].value = 0.0;
            if (lane < (cnt[f] & ~MFP_UPD_SERIAL)) u[f] = D.upd[off[f] + lane];
        }
        uint32_t malbits = 0;
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++) {
            const uint32_t pi = (uint32_t)c * 64 + lane;
            if ((uint32_t)c * 64 < np) {
                scl[pi] = pi < np ? D.prior[po + pi] : 0.0;
                if (pi < np && D.proc_mal[po + pi]) malbits |= 1u << c;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t f = 0; f < NFEAT; f++) {
            const uint32_t c = cnt[f] & ~MFP_UPD_SERIAL;
            if (cnt[f] & MFP_UPD_SERIAL) {
                for (uint32_t k = 0; k < c; k++) {
                    const mfp_update x = k < 64 && !anylong ? mfp_update{(uint32_t)__shfl((int)u[f].idx, (int)k, 64), 0,
                                                                        __shfl(u[f].value, (int)k, 64)}
                                                            : D.upd[off[f] + k];
                    if (lane == 0) scl[x.idx] += x.value;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            } else {
                if (lane < c) scl[u[f].idx] += u[f].value;
                for (uint32_t b = 64; b < c; b += 64) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    if (b + lane < c) { const mfp_update x = D.upd[off[f] + b + lane]; scl[x.idx] += x.value; }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        double sc[MAXP_CHUNKS];
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++) sc[c] = (uint32_t)c * 64 < np ? scl[c * 64 + lane] : 0.0;
        __builtin_amdgcn_wave_barrier();

        // ---- max / second max (sequential first-index rule)
        double mx = -1.7976931348623157e308;
        uint32_t imx = 0xffffffffu;
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++) {
            const uint32_t pi = (uint32_t)c * 64 + lane;
            if (pi < np && (imx == 0xffffffffu || sc[c] > mx)) { mx = sc[c]; imx = pi; }
        }
        for (int d = 32; d >= 1; d >>= 1) {
            const double om = __shfl_xor(mx, d, 64);
            const uint32_t oi = (uint32_t)__shfl_xor((int)imx, d, 64);
            if (oi != 0xffffffffu && (imx == 0xffffffffu || om > mx || (om == mx && oi < imx))) { mx = om; imx = oi; }
        }
        imx = rfl(imx);
        mx = __hiloint2double((int)rfl((uint32_t)(__double_as_longlong(mx) >> 32)),
                              (int)rfl((uint32_t)__double_as_longlong(mx)));
        double sx = -1.7976931348623157e308;
        uint32_t isx = 0xffffffffu;
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++) {
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

        // ---- softmax (expf in fp32, stored as double), sums
        double ssum = 0.0, swo = 0.0, mal = 0.0, p_imx = 0.0, p_isx = 0.0;
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++) {
            const uint32_t pi = (uint32_t)c * 64 + lane;
            if (pi < np) {
                const double p = (double)expf((float)(sc[c] - mx));
                ssum += p;
                if (pi != imx) swo += p;
                if (malbits & (1u << c)) mal += p;
                if (pi == imx) p_imx = p;
                if (pi == isx) p_isx = p;
            }
        }
        ssum = sum_all(ssum); swo = sum_all(swo); mal = sum_all(mal);
        p_imx = sum_all(p_imx); p_isx = sum_all(p_isx);
        double max_score = p_imx;
        if (ssum > 0.0 && mdb) mal /= ssum;
        uint32_t ibest = imx;
        if (mdb && dmz == imx && !D.proc_mal[po + isx]) {
            ibest = isx;
            ssum = swo;
            max_score = p_isx;
        }
        if (ssum > 0.0) max_score /= ssum;
        if (lane == 0) {
            mfp_analysis a = P.out[i];   // status and pending flag from k_analyze
            a.score = max_score;
            a.process = D.proc_id[po + ibest];
            a.attr = (uint16_t)D.proc_attr[po + ibest];
            a.malware_prob = -1.0;
            a.flags = (uint8_t)(MFP_AN_VALID | (a.flags & MFP_AN_PENDING));
            if (mdb) {
                a.malware_prob = mal;
                a.flags |= MFP_AN_CLASSIFY_MALWARE;
                if (D.proc_mal[po + ibest]) a.flags |= MFP_AN_MALWARE;
            }
            // encrypted_channel (analysis.h:1161-1163)
            if ((a.flags & MFP_AN_MALWARE) && ft == 1) a.attr |= (uint16_t)(1u << D.enc_channel_idx);
            P.out[i] = a;
        }
        __builtin_amdgcn_wave_barrier();
    }
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
    const uint64_t ngroups = (P.n + 63) / 64;
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups; g += (uint64_t)gridDim.x * 256) {
    uint32_t r = seen_pos ? 0u : group_off[g];
    for (uint64_t w = P.pend_bits[g]; w; w &= w - 1) {
        const uint32_t i = (uint32_t)(g * 64 + (uint64_t)__builtin_ctzll(w));
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
            seen = seen_seq[r++] != 0;
        }
        a.flags &= (uint8_t)~MFP_AN_PENDING;
        if (seen) {
            a.status = 3;
            a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0;
            a.flags = MFP_AN_VALID;
        }
        if (P.mode == MFP_MODE_ANALYSIS && (rc.flags & MFP_FLAG_TRUNCATED)) a.status = 3;   // pkt_proc.cc:1716-1719
        P.out[i] = a;
    }
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
    P.pend_bits = (uint64_t *)pending;
    P.deferred = (mfpa::Deferred *)deferred;
    P.lane_max_p = lane_max_p;
    P.stats = stats;
    return P;
}

extern "C" int mfp_launch_analysis(const mfp_classifier_dev *D, const mfp_seen_tab *T, const uint8_t *arena,
                                   const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, const uint8_t *fp_arena,
                                   mfp_analysis *out, uint32_t *pending, void *deferred, unsigned long long *stats,
                                   uint32_t mode, uint32_t lane_max_p, hipStream_t stream, mfp_prof *prof) {
    if (n == 0) return 0;
    mfpa::AParams P = make_params(D, *T, arena, desc, n, rec, fp_arena, out, pending, deferred, stats, mode, lane_max_p);
    uint64_t groups = (n + 63) / 64, blocks = (groups + mfpa::AW - 1) / mfpa::AW;
    if (blocks > 4096) blocks = 4096;
    if (prof) mfp_prof_begin(prof, "k_analyze", stream);
    hipLaunchKernelGGL(mfpa::k_analyze, dim3((uint32_t)blocks), dim3(64 * mfpa::AW), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    if (hipGetLastError() != hipSuccess) return -1;
    if (prof) mfp_prof_begin(prof, "k_analyze_wave", stream);
    hipLaunchKernelGGL(mfpa::k_analyze_wave, dim3(1024), dim3(256), 0, stream, P);
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
    uint64_t groups = (n + 63) / 64, blocks = (groups + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (prof) mfp_prof_begin(prof, "k_analyze_resolve", stream);
    hipLaunchKernelGGL(mfpa::k_analyze_resolve, dim3((uint32_t)blocks), dim3(256), 0, stream, P, seen_pos, group_off,
                       seen_seq);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
