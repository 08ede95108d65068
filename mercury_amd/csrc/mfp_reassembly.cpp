// mfp_reassembly.cpp -- TCP reassembly of multi-segment messages (SURVEY
// §8(f) rank 4) around the device fingerprint path.
//
// The reference's write_json path with "reassembly" configured
// (stateful_pkt_proc::process_tcp_data pkt_proc.cc:773-893 over
// tcp_reassembler / reassembly_flow_context reassembly.hpp:140-900) keeps a
// per-flow buffer for a message whose first segment says more bytes follow
// (a TLS handshake, a certificate list, an SSH banner or binary packet), adds
// the flow's later segments by sequence number, and fingerprints the buffer
// once it is complete (or truncated); the segments before that write no
// record.
//
// Here a batch runs in three steps:
//   1. the device walks every packet (mfp_process_batch_host_seg): record,
//      fingerprint, and per packet the reassembly inputs the walk already has
//      (sequence number, TCP data span, additional_bytes_needed of the parsed
//      message, supplementary / SSH-type bits: mfp_tcp_seg);
//   2. the host applies the flow-table state machine in stream order: only
//      TCP data segments are looked at, and only header fields and the
//      segment bytes of flows in reassembly are touched;
//   3. the reassembled messages are rebuilt as frames (the packet's own IP and
//      TCP headers, IP lengths patched, then the buffer; linktype RAW) and the
//      device fingerprints them in one more batch; their records replace the
//      completing packets' records.
// State persists across batches in the mfp_reassembler (the processor's
// tcp_reassembler).  Deviations, by construction: the reference reaps expired
// flows in unordered_map iteration order (passive_reap, active_reap at 10000
// flows, reassembly.hpp:597-640); here an expired flow is found expired when
// its next segment arrives, and at 10000 flows the oldest ones are dropped.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_internal.h"

namespace {

constexpr uint32_t kMaxData = 8192;       // reassembly_flow_context::max_data_size
constexpr uint32_t kMaxSegments = 20;     // max_segments
constexpr uint64_t kTimeout = 15;         // reassembly_timeout (seconds)
constexpr size_t kMaxFlows = 10000;       // tcp_reassembler::max_entries

enum Flag { F_MISSING = 0, F_TIMEOUT, F_OOO, F_OUT_OF_BUFFER, F_MAX_SEG, F_OVERLAP, F_TRUNCATED };
enum Ovl { O_BACK_PARTIAL = 0, O_BACK_SUBSET, O_FRONT_PARTIAL, O_FRONT_SUPERSET };
enum State { S_PROGRESS = 1, S_SUCCESS, S_TRUNCATED };

// ---- the host cursor (struct datum, datum.h), for the SSH re-parse
struct HC { const uint8_t *d, *e; };
long hlen(HC c) { return c.d ? (long)(c.e - c.d) : 0; }
void hnull(HC &c) { c.d = c.e = nullptr; }
bool hrd(HC &c, int n, uint64_t &v) {
    if (c.d && c.d + n <= c.e) { v = 0; for (int i = 0; i < n; i++) v = v << 8 | c.d[i]; c.d += n; return true; }
    hnull(c); v = 0; return false;
}
void hskip(HC &c, long n) { if (!c.d) return; if (n > c.e - c.d) c.d = c.e; else c.d += n; }
void hparse(HC &dst, HC &r, long n) {
    if (hlen(r) < n || n < 0) { hnull(r); hnull(dst); return; }
    dst.d = r.d; dst.e = r.d ? r.d + n : nullptr; if (r.d) r.d += n;
}

// ssh_init_packet::more_bytes_needed (ssh.h:342-376, 464-473) of the
// reassembled bytes: the binary packet's missing bytes when a KEXINIT
// (ssh_kex_init::is_not_empty: a non-empty kex_algorithms name list,
// ssh.h:104-117,200-218) follows the banner, else max_data_size
uint32_t ssh_more(const uint8_t *p, size_t n) {
    HC c{p, p + n};
    // protocol string up to '\n' or ' ' (datum::parse_up_to_delimiters)
    const uint8_t *q = c.d;
    while (q < c.e && *q != '\n' && *q != ' ') q++;
    const bool nl = q < c.e && *q == '\n';
    c.d = q;
    if (!nl) {
        hskip(c, 1);                                       // the space
        // comment up to '\n' (parse_up_to_delim: the cursor stays when absent)
        const uint8_t *r = c.d;
        if (hlen(c) > 0) { while (r < c.e && *r != '\n') r++; if (r < c.e) c.d = r; }
        else hnull(c);
    }
    hskip(c, 1);                                           // the linefeed
    if (hlen(c) <= 0) return kMaxData;
    uint64_t plen, pad;
    hrd(c, 4, plen);
    hrd(c, 1, pad);
    if (plen > 16384 || plen < 1) return kMaxData;         // set_empty: no payload, no KEXINIT
    if (hlen(c) <= 0) return kMaxData;
    const long left = (long)plen - 1;
    uint64_t more = left > hlen(c) ? (uint64_t)(left - hlen(c)) : 0;
    HC pl{c.d, c.d + (left < hlen(c) ? left : hlen(c))};   // parse_soft_fail
    if (hlen(pl) <= 0) return kMaxData;                    // binary_pkt.is_not_empty()
    HC t;
    hparse(t, pl, 1);                                      // msg_type
    hparse(t, pl, 16);                                     // cookie
    uint64_t ll;
    hrd(pl, 4, ll);                                        // kex_algorithms name_list
    if (ll > 2048) return kMaxData;
    HC kex;
    hparse(kex, pl, (long)ll);
    if (!(kex.d && kex.d < kex.e)) return kMaxData;
    return (uint32_t)more;
}

struct FlowKey {
    uint8_t v;            // 4 or 6
    uint8_t src[16], dst[16];
    uint16_t sport, dport;
    bool operator==(const FlowKey &o) const {
        return v == o.v && sport == o.sport && dport == o.dport && !memcmp(src, o.src, 16) && !memcmp(dst, o.dst, 16);
    }
};
struct FlowKeyHash {
    size_t operator()(const FlowKey &k) const {
        uint64_t h = 1469598103934665603ull ^ k.v;
        auto mix = [&](const uint8_t *p, size_t n) { for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; } };
        mix(k.src, 16); mix(k.dst, 16);
        h ^= (uint64_t)k.sport << 16 | k.dport; h *= 1099511628211ull;
        return (size_t)h;
    }
};

// reassembly_flow_context (reassembly.hpp:140-520), TCP fields only
struct Flow {
    uint8_t flags = 0, ovl = 0;      // reassembly_flag_val, reassembly_overlap_flags
    int state = S_PROGRESS;
    uint64_t init_time = 0, order = 0;
    uint32_t init_seq = 0, init_seg_len = 0, total_needed = 0;
    bool ssh_type = false;           // reassembly_type::ssh (indefinite)
    size_t contiguous = 0;
    size_t seg_count = 0;
    std::vector<std::pair<uint32_t, uint32_t>> segs;   // [first, second] relative sequence numbers
    uint8_t buf[kMaxData];

    void init(uint32_t len, uint32_t seq, uint32_t more, bool ssh, uint64_t t, const uint8_t *data, uint32_t avail) {
        init_time = t; init_seq = seq; init_seg_len = len; total_needed = len + more; ssh_type = ssh;
        contiguous = len;
        uint32_t copy = len < avail ? len : avail;
        if (copy > kMaxData) copy = kMaxData;
        if (len == 0 || copy == 0) { state = S_TRUNCATED; flags |= 1u << F_TRUNCATED; return; }
        init_seg_len = copy;
        total_needed = len + more;
        contiguous = copy;
        segs.clear();
        segs.emplace_back(seq - init_seq, seq - init_seq + init_seg_len - 1);
        seg_count = 1;
        memcpy(buf, data, init_seg_len);
    }
    // simplify_seglist reassembly.hpp:330-400
    void simplify(size_t idx) {
        if (idx) {
            if ((segs[idx].first == segs[idx - 1].first && segs[idx].second == segs[idx - 1].second) ||
                (segs[idx].first <= segs[idx - 1].second && segs[idx].second <= segs[idx - 1].second)) {
                segs.erase(segs.begin() + (long)idx);
                flags |= 1u << F_OVERLAP; ovl |= 1u << O_BACK_SUBSET;
                return;
            }
            if (segs[idx].first <= segs[idx - 1].second && segs[idx].second > segs[idx - 1].second) {
                segs[idx].first = segs[idx - 1].second + 1;
                flags |= 1u << F_OVERLAP; ovl |= 1u << O_BACK_PARTIAL;
            }
        }
        if (idx != segs.size() - 1) {
            size_t i = idx + 1;
            for (; i < segs.size() - 1; i++) {
                if (segs[i].first <= segs[idx].second && segs[i].second <= segs[idx].second) {
                    flags |= 1u << F_OVERLAP; ovl |= 1u << O_FRONT_SUPERSET;
                } else {
                    break;
                }
            }
            if (i != idx + 1) segs.erase(segs.begin() + (long)idx + 1, segs.begin() + (long)i);
        }
        if (idx != segs.size() - 1) {
            if (segs[idx].second >= segs[idx + 1].first && segs[idx].second <= segs[idx + 1].second) {
                segs[idx].second = segs[idx + 1].first - 1;
                flags |= 1u << F_OVERLAP; ovl |= 1u << O_FRONT_PARTIAL;
            }
        }
    }
    // update_contiguous_data reassembly.hpp:404-416
    void update_contiguous() {
        contiguous = init_seg_len;
        for (size_t k = 1; k < segs.size(); k++) {
            if (segs[k].first == segs[k - 1].second + 1) contiguous += segs[k].second - segs[k].first + 1;
            else break;
        }
    }
    // process_tcp_segment reassembly.hpp:456-512
    void add(uint32_t len, uint32_t seq, const uint8_t *data, uint32_t avail) {
        if (len == 0 || !data) return;
        const uint32_t st = seq >= init_seq ? seq - init_seq : (uint32_t)(0xffffffffu + seq - init_seq + 1);
        uint32_t dlen = len < avail ? len : avail;
        if (dlen == 0) return;
        const uint64_t end64 = (uint64_t)st + dlen - 1;
        const uint32_t en = end64 >= kMaxData - 1 ? kMaxData - 1 : (uint32_t)end64;
        seg_count++;
        if (seg_count > kMaxSegments) {
            flags |= (1u << F_MAX_SEG) | (1u << F_TRUNCATED);
            state = S_TRUNCATED;
            return;
        }
        if (st > kMaxData - 1) return;
        memcpy(buf + st, data, en - st + 1);
        size_t idx = segs.size();
        for (size_t k = segs.size(); k-- > 0;) {
            if (segs[k].first <= st) { segs.insert(segs.begin() + (long)k + 1, {st, en}); break; }
            idx--;
        }
        simplify(idx);
        update_contiguous();
        if (contiguous >= total_needed) state = S_SUCCESS;
        if (ssh_type) {                                    // handle_indefinite_reassembly (ssh)
            const uint32_t more = ssh_more(buf, contiguous);
            if (!more) { state = S_SUCCESS; total_needed = (uint32_t)contiguous; }
            else if (more != kMaxData) { total_needed = more + (uint32_t)contiguous; ssh_type = false; }
        }
    }
    bool truncated_flags() const {                        // was_flow_truncated reassembly.hpp:790-800
        return flags & ((1u << F_TRUNCATED) | (1u << F_TIMEOUT) | (1u << F_OUT_OF_BUFFER) | (1u << F_MAX_SEG) |
                        (1u << F_MISSING));
    }
};

}  // namespace

struct mfp_reassembler_s {
    std::unordered_map<FlowKey, Flow, FlowKeyHash> table;
    std::deque<std::pair<FlowKey, uint64_t>> age;   // insertion order (for the 10000-flow bound)
    uint64_t order = 0;
    std::vector<mfp_tcp_seg> seg;
    std::vector<mfp_record> rec2;
    std::vector<mfp_pkt_desc> desc2;
    std::vector<uint8_t> frames;
    std::vector<size_t> who;                        // packet index of each rebuilt frame
    std::vector<uint16_t> who_props;
    std::vector<uint8_t> quiet;                     // 1: a segment that writes no record (return false)
    std::vector<uint8_t> merged;                    // arena ++ frames (the classifier pass)
    std::vector<mfp_pkt_desc> desc3;
};

extern "C" MFP_EXPORT mfp_reassembler mfp_reassembler_create(void) { return new mfp_reassembler_s; }
extern "C" MFP_EXPORT void mfp_reassembler_destroy(mfp_reassembler r) { delete r; }
extern "C" MFP_EXPORT uint64_t mfp_reassembler_flows(mfp_reassembler r) { return r ? r->table.size() : 0; }
extern "C" MFP_EXPORT const uint8_t *mfp_reassembler_frames(mfp_reassembler r, size_t *len) {
    if (len) *len = r ? r->frames.size() : 0;
    return r && !r->frames.empty() ? r->frames.data() : nullptr;
}

static bool flow_key(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, FlowKey &k) {
    const uint32_t ip = r.net & 0xffff, v = (r.net >> 16) & 15;
    memset(&k, 0, sizeof k);
    k.v = (uint8_t)v; k.sport = r.src_port; k.dport = r.dst_port;
    if (v == 4 && ip + 20 <= caplen) { memcpy(k.src, pkt + ip + 12, 4); memcpy(k.dst, pkt + ip + 16, 4); return true; }
    if (v == 6 && ip + 40 <= caplen) { memcpy(k.src, pkt + ip + 8, 16); memcpy(k.dst, pkt + ip + 24, 16); return true; }
    return false;
}

// the reassembled message as a frame: the packet's IP header and TCP header
// (bytes [ip, data)), the IP length fields set for the new data, the buffer
static void rebuild(std::vector<uint8_t> &out, const uint8_t *pkt, const mfp_record &r, const mfp_tcp_seg &s,
                    const uint8_t *data, size_t len) {
    const uint32_t ip = r.net & 0xffff, v = (r.net >> 16) & 15;
    const size_t hdr = s.pay_off - ip;
    const size_t at = out.size();
    out.insert(out.end(), pkt + ip, pkt + s.pay_off);
    out.insert(out.end(), data, data + len);
    uint8_t *h = out.data() + at;
    if (v == 4) {
        const size_t tl = hdr + len;                        // ipv4_packet::parse trims to tot_len - 20 (ip.h:124-137)
        h[2] = (uint8_t)(tl >> 8); h[3] = (uint8_t)tl;
    } else {
        const size_t pl = hdr - 40 + len;                   // ipv6 payload_len (ip.h:448-474)
        h[4] = (uint8_t)(pl >> 8); h[5] = (uint8_t)pl;
    }
    while (out.size() % 8) out.push_back(0);                // keep frames 8-byte aligned
    out.resize(out.size() + 16, 0);                         // the readable tail block (include/mfp.h)
}

extern "C" MFP_EXPORT long long mfp_process_batch_reassembly(mfp_context ctx, mfp_reassembler R, const uint8_t *arena,
                                                             size_t arena_len, const mfp_pkt_desc *desc, size_t n,
                                                             const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                                                             size_t fp_cap, uint16_t *props,
                                                             mfp_pkt_desc *out_desc) {
    if (!ctx || !R) { mfp_set_error("null context or reassembler"); return -1; }
    if (!mfp_reassembly_enabled(ctx)) { mfp_set_error("the context's configuration has no \"reassembly\""); return -1; }
    if (n && (!arena || !desc || !rec || !fp_arena || !props)) { mfp_set_error("null argument"); return -1; }
    R->seg.resize(n);
    // 1. the device walk: records, fingerprints, reassembly inputs
    long long used = mfp_process_batch_host_seg(ctx, arena, arena_len, desc, n, rec, fp_arena, fp_cap, R->seg.data());
    if (used < 0) return used;
    // 2. the flow table in stream order (process_tcp_data pkt_proc.cc:773-893)
    R->frames.clear(); R->desc2.clear(); R->who.clear(); R->who_props.clear();
    R->quiet.assign(n, 0);
    for (size_t i = 0; i < n; i++) {
        props[i] = 0;
        const mfp_tcp_seg &s = R->seg[i];
        if (!(s.kind & MFP_SEG_DATA)) continue;
        mfp_record &r = rec[i];
        const uint8_t *pkt = arena + desc[i].offset;
        const uint32_t data_len = s.pay_len;
        const uint32_t more = s.more;
        const bool supp = s.kind & MFP_SEG_SUPPLEMENTARY;
        const bool mono = r.msg == 0;                       // std::monostate: no message parsed
        if (!more && !mono && !supp) continue;              // a complete message
        if (more > kMaxData || data_len > kMaxData) continue;   // cannot be reassembled
        FlowKey k;
        if (!flow_key(pkt, desc[i].caplen, r, k)) continue;
        const uint64_t sec = ts_ns ? ts_ns[i] / 1000000000ull : 0;
        auto it = R->table.find(k);
        const uint8_t *data = pkt + s.pay_off;
        const uint32_t avail = s.pay_off + (uint64_t)data_len <= desc[i].caplen ? data_len : 0;
        if (it == R->table.end()) {
            if (supp) continue;                             // not in reassembly: taken as complete
            if (!more) { r.flags &= (uint8_t)~MFP_FLAG_EMIT; r.fp_type = 0; r.fp_len = 0; R->quiet[i] = 1; continue; }
            if (R->table.size() >= kMaxFlows) {             // active_reap (two entries)
                for (int d = 0; d < 2 && !R->age.empty(); d++) {
                    auto old = R->table.find(R->age.front().first);
                    if (old != R->table.end() && old->second.order == R->age.front().second) R->table.erase(old);
                    R->age.pop_front();
                }
            }
            Flow &f = R->table[k];
            f.order = ++R->order;
            R->age.emplace_back(k, f.order);
            f.init(data_len, s.seq, more, (s.kind & MFP_SEG_SSH) != 0, sec, data, avail);
            it = R->table.find(k);
        } else {
            Flow &f = it->second;
            if (sec - f.init_time >= kTimeout) {            // continue_reassembly: set_expired
                f.state = S_TRUNCATED;
                f.flags |= 1u << F_TIMEOUT;
            } else {
                const uint32_t seq = s.seq ? s.seq : (uint32_t)f.contiguous;   // 0: in order (pkt_proc.cc:857-861)
                f.add(data_len, seq, data, avail);
            }
        }
        Flow &f = it->second;
        if (f.state == S_SUCCESS || f.state == S_TRUNCATED) {   // is_ready: fingerprint the buffer
            R->who.push_back(i);
            R->who_props.push_back((uint16_t)(1u | (uint32_t)f.flags << 1 | (uint32_t)f.ovl << 8));
            mfp_pkt_desc d2;
            d2.offset = R->frames.size();
            rebuild(R->frames, pkt, r, s, f.buf, f.contiguous);
            d2.caplen = (uint32_t)(s.pay_off - (r.net & 0xffff) + f.contiguous);
            d2.linktype = 101;                              // LINKTYPE_RAW
            d2.flags = 0;
            R->desc2.push_back(d2);
            R->table.erase(it);                             // consumed, then clean_curr_flow
        } else {
            r.flags &= (uint8_t)~MFP_FLAG_EMIT; r.fp_type = 0; r.fp_len = 0;   // no record for this segment
            R->quiet[i] = 1;
        }
    }
    // 3. the reassembled messages through the device; their records replace
    // the completing packets' (their strings follow the batch's)
    const size_t m = R->who.size();
    if (out_desc) for (size_t i = 0; i < n; i++) out_desc[i] = desc[i];
    if (m) {
        R->rec2.resize(m);
        std::vector<mfp_tcp_seg> seg2(m);
        const long long used2 = mfp_process_batch_host_seg(ctx, R->frames.data(), R->frames.size(), R->desc2.data(), m,
                                                           R->rec2.data(), fp_arena + used, fp_cap - (size_t)used,
                                                           seg2.data());
        if (used2 < 0) return used2;
        for (size_t j = 0; j < m; j++) {
            const size_t i = R->who[j];
            mfp_record r2 = R->rec2[j];
            if (r2.fp_type) r2.fp_offset += (uint64_t)used;
            // the reassembler's own "reassembly_properties" replace {"truncated":true}
            // (write_reassembly_properties reassembly.hpp:1231-1247)
            r2.flags &= (uint8_t)~MFP_FLAG_TRUNCATED;
            rec[i] = r2;
            props[i] = R->who_props[j];
            if (out_desc) {
                out_desc[i] = R->desc2[j];
                out_desc[i].offset += arena_len;            // frames follow the caller's arena
            }
        }
        used += used2;
    }
    return used;
}

// --analysis with reassembly (write_json with a classifier, pkt_proc.cc:1195-1238):
// the batch through the reassembler, then fingerprint + classify once more in
// stream order over what the reference analyses -- the packets that write a
// record, the reassembled messages in their completing packets' places, and
// nothing for the segments that only fed a buffer (zero-length descriptors),
// so the classifier's unknown-TLS sightings follow the reference's order.
extern "C" MFP_EXPORT long long mfp_process_batch_reassembly_analysis(
    mfp_context ctx, mfp_reassembler R, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc, size_t n,
    const uint64_t *ts_ns, mfp_record *rec, char *fp_arena, size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc,
    mfp_analysis *analysis, double *attr_prob) {
    if (!mfp_analysis_enabled(ctx)) { mfp_set_error("the context has no classifier"); return -1; }
    if (n && (!analysis || !out_desc)) { mfp_set_error("null argument"); return -1; }
    long long used = mfp_process_batch_reassembly(ctx, R, arena, arena_len, desc, n, ts_ns, rec, fp_arena, fp_cap, props,
                                                  out_desc);
    if (used < 0) return used;
    R->merged.assign(arena, arena + arena_len);
    R->merged.insert(R->merged.end(), R->frames.begin(), R->frames.end());
    R->merged.resize(R->merged.size() + 16, 0);
    R->desc3.assign(out_desc, out_desc + n);
    for (size_t i = 0; i < n; i++) if (R->quiet[i]) R->desc3[i].caplen = 0;
    used = mfp_process_batch_host_ex(ctx, R->merged.data(), R->merged.size(), R->desc3.data(), n, rec, fp_arena, fp_cap,
                                     analysis, attr_prob);
    if (used < 0) return used;
    for (size_t i = 0; i < n; i++) if (props[i] & 1) rec[i].flags &= (uint8_t)~MFP_FLAG_TRUNCATED;
    return used;
}
