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
// the known set is a device table; the adaptive set is a device hash set
// whose per-fingerprint word is min((batch << 32) | packet index), so the
// first sighting in stream order is "randomized" and every later one
// "unlabeled" (k_analyze_status).
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
    for (uint32_t u = 0; u < h.cnt; u++) {
        const mfp_update up = D.upd[h.off + u];
        const uint32_t idx = rfl(up.idx);
        const double v = __hiloint2double((int)rfl((uint32_t)(__double_as_longlong(up.value) >> 32)),
                                          (int)rfl((uint32_t)__double_as_longlong(up.value)));
#pragma unroll
        for (int c = 0; c < MAXP_CHUNKS; c++)
            if ((idx >> 6) == (uint32_t)c && (idx & 63) == lane) sc[c] += v;
    }
}

struct AParams {
    mfp_classifier_dev D;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    const uint8_t *fp_arena;
    mfp_analysis *out;
    uint32_t mode;
    unsigned long long *stats;   // [0] analyzed, [1] pending unknown-TLS, [2] over-size P
};

__global__ __launch_bounds__(256) void k_analyze(AParams P) {
    __shared__ char sni_buf[4][336];
    const uint32_t lane = lane_id();
    const int wid = (int)rfl(threadIdx.x >> 6);
    char *nbuf = sni_buf[wid];
    const mfp_classifier_dev &D = P.D;
    const uint64_t ngroups = (P.n + 63) / 64;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + wid; g < ngroups; g += nw) {
        const uint64_t i = g * 64 + lane;
        const bool live = i < P.n;
        mfp_record r;
        if (live) r = P.rec[i];
        else { r.fp_len = 0; r.fp_type = 0; }
        // default result: no information (analysis_result())
        mfp_analysis a;
        a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0; a.status = 0; a.flags = 0;
        // messages whose do_analysis calls the classifier: TLS ClientHello
        // (tls.h:1977), HTTP request (http.cc:571), SSH client KEXINIT
        // (ssh.h:480); their type must also be in the archive (fp_types)
        const bool typed = live && r.fp_len != 0 && (r.fp_type == 1 || r.fp_type == 3 || r.fp_type == 5);
        const bool analyzable = typed && ((D.types_mask >> r.fp_type) & 1u);
        if (typed && !analyzable) { a.status = 4; a.flags = MFP_AN_VALID; }   // fingerprint_status_unanalyzed
        uint64_t todo = __ballot(analyzable);
        while (todo) {
            const int j = (int)__builtin_ctzll(todo);
            todo &= todo - 1;
            // ---- this packet's inputs, wave-uniform
            const uint64_t fpo = ((uint64_t)rfl(__shfl((uint32_t)(r.fp_offset >> 32), j, 64)) << 32) |
                                 rfl(__shfl((uint32_t)r.fp_offset, j, 64));
            const uint32_t fl = rfl(__shfl(r.fp_len, j, 64));
            const uint32_t ft = rfl(__shfl((uint32_t)r.fp_type, j, 64));
            const uint32_t sni = rfl(__shfl((uint32_t)r.sni_off | ((uint32_t)r.sni_len << 16), j, 64));
            const uint32_t ua = rfl(__shfl((uint32_t)r.ua_off | ((uint32_t)r.ua_len << 16), j, 64));
            const uint32_t dport = rfl(__shfl((uint32_t)r.dst_port, j, 64));
            const uint32_t net = rfl(__shfl(r.net, j, 64));
            const uint64_t pidx = g * 64 + (uint64_t)j;
            const mfp_pkt_desc dsc = P.desc[pidx];
            const uint8_t *pkt = P.arena + dsc.offset;
            const uint8_t *fp = P.fp_arena + fpo;

            // ---- 1. fingerprint lookup / status (perform_analysis_common)
            uint32_t status = 0, entry = 0xffffffffu;
            bool pending = false;
            const uint64_t fh = wave_hash(fp, fl, lane);
            entry = probe_string(D.fp_slots, D.fp_mask, D.pool, fp, fl, fh, lane);
            if (entry != 0xffffffffu) {
                status = 1;                                         // labeled
            } else if (fl >= 4 && fp[0] == 't' && fp[1] == 'l' && fp[2] == 's' && fp[3] == '/') {
                if (probe_string(D.prev_slots, D.prev_mask, D.pool, fp, fl, fh, lane) != 0xffffffffu) {
                    status = 3;                                     // unlabeled (known set; no LRU update)
                } else {
                    // adaptive set: record the sighting; k_analyze_status decides
                    pending = true;
                    status = 2;
                    if (lane == 0) {
                        uint64_t k = fh & (D.seen_cap - 1);
                        for (uint32_t t = 0; t < D.seen_cap; t++, k = (k + 1) & (D.seen_cap - 1)) {
                            unsigned long long prev = atomicCAS(&D.seen[k].hash, ~0ull, (unsigned long long)fh);
                            if (prev == ~0ull) atomicAdd(D.seen_count, 1ull);
                            if (prev == ~0ull || prev == fh) {
                                atomicMin(&D.seen[k].first, ((unsigned long long)D.batch << 32) | (uint32_t)pidx);
                                break;
                            }
                        }
                    }
                    // classify with "<prefix>randomized" when the DB has it
                    const uint32_t pre = fl > 5 && fp[4] == '1' && fp[5] == '/' ? 1u : fl > 5 && fp[4] == '2' && fp[5] == '/' ? 2u : 0u;
                    entry = D.randomized_entry[pre];
                }
            } else {
                status = 3;                                         // unlabeled
            }
            mfp_analysis res;
            res.score = 0.0; res.malware_prob = -1.0; res.process = MFP_NO_PROCESS; res.attr = 0;
            res.status = (uint8_t)status; res.flags = MFP_AN_VALID | (pending ? MFP_AN_PENDING : 0);
            if (entry != 0xffffffffu) {
                const mfp_entry E = D.entry[entry];
                const uint32_t np = rfl(E.nproc), po = rfl(E.proc_off), mdb = rfl(E.malware_db), dmz = rfl(E.generic_dmz);
                if (np > 64 * MAXP_CHUNKS) {
                    if (lane == 0) atomicAdd(&P.stats[2], 1ull);
                } else {
                    // ---- 2. destination context
                    uint32_t ipv = (net >> 16) & 15, ipo = net & 0xffff;
                    uint32_t v4 = 0, asn = 0;
                    uint8_t v6[16];
                    uint64_t v6h = 0, v6l = 0;
                    if (ipv == 4) {
                        const uint8_t *d = pkt + ipo + 16;
                        v4 = (uint32_t)d[0] | (uint32_t)d[1] << 8 | (uint32_t)d[2] << 16 | (uint32_t)d[3] << 24;
                        asn = asn_v4(D, (uint32_t)d[0] << 24 | (uint32_t)d[1] << 16 | (uint32_t)d[2] << 8 | d[3]);
                    } else if (ipv == 6) {
                        const uint8_t *d = pkt + ipo + 24;
                        for (int k = 0; k < 16; k++) v6[k] = d[k];
                        for (int k = 0; k < 8; k++) { v6h = v6h << 8 | v6[k]; v6l = v6l << 8 | v6[k + 8]; }
                        if (D.n_asn6) asn = asn_v6(D, v6h, v6l);
                    }
                    // server name: TLS SNI, HTTP Host (strncpy 256, NUL stops)
                    const uint32_t sl = (sni >> 16) == 0xffff ? 0 : (sni >> 16);
                    const uint8_t *sp = pkt + (sni & 0xffff);
                    int nlen = 0;
                    if (lane == 0) nlen = normalize_server_name(sp, (int)sl, nbuf);
                    nlen = (int)rfl((uint32_t)nlen);
                    __builtin_amdgcn_wave_barrier();
                    const int tld = (int)rfl((uint32_t)(lane == 0 ? tld_domain_offset(nbuf, nlen) : 0));
                    // user agent (strncpy 511, NUL stops); TLS has none
                    uint32_t ul = (ua >> 16) == 0xffff ? 0 : (ua >> 16);
                    const uint8_t *up = pkt + (ua & 0xffff);
                    if (ul > 511) ul = 511;
                    {
                        uint32_t z = 0xffffffffu;
                        for (uint32_t k = lane; k < ul; k += 64) if (up[k] == 0 && k < z) z = k;
                        for (int d = 32; d >= 1; d >>= 1) z = min(z, (uint32_t)__shfl_xor((int)z, d, 64));
                        z = rfl(z);
                        if (z < ul) ul = z;
                    }

                    // ---- 3. scores (lane i = process i)
                    double sc[MAXP_CHUNKS];
#pragma unroll
                    for (int c = 0; c < MAXP_CHUNKS; c++) {
                        const uint32_t pi = (uint32_t)c * 64 + lane;
                        sc[c] = pi < np ? D.prior[po + pi] : 0.0;
                    }
                    apply(D, probe_feature(D, entry, F_ASN, asn, nullptr, 0, false, lane), sc, lane);
                    apply(D, probe_feature(D, entry, F_PORT, dport, nullptr, 0, false, lane), sc, lane);
                    if (ipv == 4) {
                        apply(D, probe_feature(D, entry, F_IPV4, normalize_ipv4(v4), nullptr, 0, false, lane), sc, lane);
                    } else if (ipv == 6) {
                        normalize_ipv6(v6);
                        uint64_t k6 = str_hash(v6, 16);
                        apply(D, probe_feature(D, entry, F_IPV6, k6, v6, 16, true, lane), sc, lane);
                    }
                    apply(D, probe_feature(D, entry, F_UA, wave_hash(up, ul, lane), up, ul, true, lane), sc, lane);
                    const uint8_t *dom = (const uint8_t *)nbuf + tld;
                    apply(D, probe_feature(D, entry, F_DOMAIN, wave_hash(dom, (uint32_t)(nlen - tld), lane), dom,
                                           (uint32_t)(nlen - tld), true, lane), sc, lane);
                    apply(D, probe_feature(D, entry, F_SNI, wave_hash((const uint8_t *)nbuf, (uint32_t)nlen, lane),
                                           (const uint8_t *)nbuf, (uint32_t)nlen, true, lane), sc, lane);

                    // ---- 4. max / second max (sequential first-index rule)
                    double mx = -1.7976931348623157e308;
                    uint32_t imx = 0xffffffffu;
#pragma unroll
                    for (int c = 0; c < MAXP_CHUNKS; c++) {
                        const uint32_t pi = (uint32_t)c * 64 + lane;
                        if (pi < np && (imx == 0xffffffffu || sc[c] > mx)) { mx = sc[c]; imx = pi; }
                    }
                    for (int d = 32; d >= 1; d >>= 1) {
                        double om = __shfl_xor(mx, d, 64);
                        uint32_t oi = (uint32_t)__shfl_xor((int)imx, d, 64);
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
                        double om = __shfl_xor(sx, d, 64);
                        uint32_t oi = (uint32_t)__shfl_xor((int)isx, d, 64);
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
                            if (D.proc_mal[po + pi]) mal += p;
                            if (pi == imx) p_imx = p;
                            if (pi == isx) p_isx = p;
                        }
                    }
                    ssum = sum_all(ssum); swo = sum_all(swo); mal = sum_all(mal);
                    p_imx = sum_all(p_imx); p_isx = sum_all(p_isx);
                    double max_score = p_imx, sec_score = p_isx;
                    if (ssum > 0.0 && mdb) mal /= ssum;
                    uint32_t ibest = imx;
                    if (mdb && dmz == imx && !D.proc_mal[po + isx]) {
                        ibest = isx;
                        ssum = swo;
                        max_score = sec_score;
                    }
                    if (ssum > 0.0) max_score /= ssum;
                    res.score = max_score;
                    res.process = D.proc_id[po + ibest];
                    res.attr = (uint16_t)D.proc_attr[po + ibest];
                    if (mdb) {
                        res.malware_prob = mal;
                        res.flags |= MFP_AN_CLASSIFY_MALWARE;
                        if (D.proc_mal[po + ibest]) res.flags |= MFP_AN_MALWARE;
                    }
                    // encrypted_channel (analysis.h:1161-1163)
                    if ((res.flags & MFP_AN_MALWARE) && ft == 1) res.attr |= (uint16_t)(1u << D.enc_channel_idx);
                }
            }
            // analyze_ip_packet: a truncated message reports "unlabeled" and
            // keeps its classification (pkt_proc.cc:1716-1719)
            const uint32_t rflags = rfl(__shfl((uint32_t)r.flags, j, 64));
            if (P.mode == MFP_MODE_ANALYSIS && (rflags & MFP_FLAG_TRUNCATED) && !pending) res.status = 3;
            if (lane == 0) atomicAdd(&P.stats[0], 1ull);
            if (pending && lane == 0) atomicAdd(&P.stats[1], 1ull);
            if (lane == (uint32_t)j) a = res;
        }
        if (live) {
            P.out[i] = a;
            P.rec[i].status = a.status;
        }
    }
}

// k_analyze_status: unknown TLS fingerprints -- the first sighting in stream
// order is "randomized" (classified with the randomized entry, if any),
// every later one "unlabeled" (no process)
__global__ __launch_bounds__(256) void k_analyze_status(AParams P) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n) return;
    mfp_analysis a = P.out[i];
    if (!(a.flags & MFP_AN_PENDING)) return;
    const mfp_record r = P.rec[i];
    const uint8_t *fp = P.fp_arena + r.fp_offset;
    const uint64_t h = str_hash(fp, r.fp_len);
    const mfp_classifier_dev &D = P.D;
    uint64_t k = h & (D.seen_cap - 1);
    bool first = false;
    for (uint32_t t = 0; t < D.seen_cap; t++, k = (k + 1) & (D.seen_cap - 1)) {
        const unsigned long long sh = D.seen[k].hash;
        if (sh == h) { first = D.seen[k].first == (((unsigned long long)D.batch << 32) | (uint32_t)i); break; }
        if (sh == ~0ull) break;
    }
    a.flags &= (uint8_t)~MFP_AN_PENDING;
    if (!first) {
        a.status = 3;
        a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.attr = 0;
        a.flags = MFP_AN_VALID;
    }
    if (P.mode == MFP_MODE_ANALYSIS && (r.flags & MFP_FLAG_TRUNCATED)) a.status = 3;   // pkt_proc.cc:1716-1719
    P.out[i] = a;
    P.rec[i].status = a.status;
}

}  // namespace mfpa

extern "C" int mfp_launch_analysis(const mfp_classifier_dev *D, const uint8_t *arena, const mfp_pkt_desc *desc,
                                   uint64_t n, mfp_record *rec, const uint8_t *fp_arena, mfp_analysis *out,
                                   unsigned long long *stats, uint32_t mode, hipStream_t stream, mfp_prof *prof) {
    if (n == 0) return 0;
    mfpa::AParams P;
    P.D = *D;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.out = out; P.mode = mode;
    P.stats = stats;
    uint64_t groups = (n + 63) / 64, blocks = (groups + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (prof) mfp_prof_begin(prof, "k_analyze", stream);
    hipLaunchKernelGGL(mfpa::k_analyze, dim3((uint32_t)blocks), dim3(256), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    if (hipGetLastError() != hipSuccess) return -1;
    if (prof) mfp_prof_begin(prof, "k_analyze_status", stream);
    hipLaunchKernelGGL(mfpa::k_analyze_status, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, P);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
