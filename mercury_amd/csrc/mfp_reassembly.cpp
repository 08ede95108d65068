// mfp_reassembly.cpp -- reassembly of multi-segment messages (SURVEY §8(f)
// rank 4) around the device fingerprint path: TCP messages, DTLS ClientHello
// fragments, QUIC ClientHellos spread over several Initials.
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
// tcp_reassembler), in the reference's container with its hash, reaped from a
// persistent iterator exactly as passive_reap / active_reap do.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_encap.hpp"
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
    uint8_t proto;        // 6 TCP, 17 UDP (struct key's protocol)
    uint8_t src[16], dst[16];
    uint16_t sport, dport;
    bool operator==(const FlowKey &o) const {
        return v == o.v && proto == o.proto && sport == o.sport && dport == o.dport && !memcmp(src, o.src, 16) &&
               !memcmp(dst, o.dst, 16);
    }
};
// std::hash<key> (flow_key.h:257-286, 313-317): the flow table's bucket of a
// key, and so its iteration order (the reaping order), follow from it
struct FlowKeyHash {
    size_t operator()(const FlowKey &k) const {
        const uint64_t m = 2862933555777941757ull;
        uint64_t x;
        const uint16_t sp = k.sport, dp = k.dport;
        const uint8_t pr = k.proto;
        if (k.v == 4) {
            uint32_t sa, da;                            // addr.ipv4: network order, read as stored
            memcpy(&sa, k.src, 4); memcpy(&da, k.dst, 4);
            x = (uint64_t)sp * da + (uint64_t)dp * sa;
            x *= m;
            x += (uint32_t)(sa + da + sp + dp + pr);    // unsigned int arithmetic
            x *= m;
        } else {
            uint64_t sa[2], da[2];
            memcpy(sa, k.src, 16); memcpy(da, k.dst, 16);
            x = (uint64_t)sp * da[0] * da[1] + (uint64_t)dp * sa[0] * sa[1];
            x *= m;
            x += sa[0] + sa[1] + da[0] + da[1] + sp + dp + pr;
            x *= m;
        }
        return (size_t)x;
    }
};

// reassembly_flow_context (reassembly.hpp:140-520), TCP fields only
struct Flow {
    uint8_t flags = 0, ovl = 0;      // reassembly_flag_val, reassembly_overlap_flags
    int state = S_PROGRESS;
    uint64_t init_time = 0;
    uint32_t init_seq = 0, init_seg_len = 0, total_needed = 0;
    bool ssh_type = false;           // reassembly_type::ssh (indefinite)
    uint8_t cid[20] = {};            // UDP reassembly: the DTLS message_seq, the QUIC connection id
    uint32_t cid_len = 0;            // (get_cid_datum, max_cid_len 20)
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

// quic_init's cryptographic_buffer (quic.h:1203-1294) for one packet
struct QCrypto {
    uint8_t buf[kMaxData];                        // zero for every packet (a new quic_init)
    uint64_t buf_len = 0, min_off = ~0ull, min_len = ~0ull, max_off = 0, max_len = 0;
    uint32_t total = 0, count = 0, first = 0xffff; // first_frame_index (invalid_first_frame_index)
    uint64_t foff[20], flen[20];                  // crypto_frames: offset, length
    uint32_t min_crypto_offset = 0xffffffffu;     // quic_init::min_crypto_offset
    void reset() {
        memset(buf, 0, sizeof buf);
        reset_meta();
    }
    // cryptographic_buffer::reset (quic.h:1283-1292): the bookkeeping only,
    // the bytes stay
    void reset_meta() {
        buf_len = 0; min_off = ~0ull; min_len = ~0ull; max_off = 0; max_len = 0;
        total = 0; count = 0; first = 0xffff; min_crypto_offset = 0xffffffffu;
    }
    // extend + update_crypto_frames + the min offset (quic.h:1226-1265, 1541-1548)
    void add(uint64_t off, uint64_t len, const uint8_t *data) {
        if (off > kMaxData || len > kMaxData || off + len > kMaxData) return;
        memcpy(buf + off, data, len);
        if (off + len > buf_len) buf_len = off + len;
        if (off == 0) first = count;
        if (off <= min_off) { min_off = off; min_len = len; }
        if (off >= max_off) { max_off = off; max_len = len; }
        total += (uint32_t)len;
        if (count < 20) { foff[count] = off; flen[count] = len; count++; }
        if (off <= min_crypto_offset) min_crypto_offset = (uint32_t)off;
    }
    bool missing() const { return (uint64_t)total != max_off + max_len - min_off; }   // quic.h:1267-1272
    bool has_first() const { return first != 0xffff && first < count; }
};

}  // namespace

struct mfp_reassembler_s {
    // the flows in reassembly (tcp_reassembler::table, reassembly.hpp:549-568):
    // the same container, hash and reserved size as the reference, so its
    // iteration order -- which the reaping iterator walks -- is the reference's
    struct Entry { Flow f; };
    std::unordered_map<FlowKey, Entry, FlowKeyHash> table;
    decltype(table)::iterator reap_it;              // reassembly.hpp:555
    bool more_state = false;                        // analysis_context::flow_state_pkts_needed (sticky)
    std::vector<mfp_tcp_seg> seg;
    std::vector<mfp_record> rec2;
    std::vector<mfp_pkt_desc> desc2;
    std::vector<uint8_t> frames;
    std::vector<size_t> who;                        // packet index of each rebuilt frame
    std::vector<uint16_t> who_props;
    std::vector<uint8_t> quiet;                     // 1: a segment that writes no record (return false)
    std::vector<uint8_t> dump;                      // 1: the packet fed the flow table (tcp_reassembler::dump_pkt)
    uint8_t dump_carry = 0;                         // dump_pkt after the last packet of the previous batch
    std::vector<uint8_t> merged;                    // arena ++ frames (the classifier pass)
    std::vector<mfp_pkt_desc> desc3;
    QCrypto qc;                                     // the current QUIC Initial's crypto buffer
    mfp_reassembler_s() { table.reserve(kMaxFlows); reap_it = table.end(); }
};

extern "C" MFP_EXPORT mfp_reassembler mfp_reassembler_create(void) { return new mfp_reassembler_s; }
extern "C" MFP_EXPORT void mfp_reassembler_destroy(mfp_reassembler r) { delete r; }
extern "C" MFP_EXPORT uint64_t mfp_reassembler_flows(mfp_reassembler r) { return r ? r->table.size() : 0; }
// tcp_reassembler::dump_pkt after each packet of the last batch
// (stateful_pkt_proc::dump_pkt pkt_proc.cc:1842-1845): set where the reference
// hands the packet's data to process_tcp_data_pkt / process_udp_data_pkt
// (pkt_proc.cc:852-866, reassembly.hpp:931-1009,1074-1079), cleared for every
// other packet (ip_write_json pkt_proc.cc:1078-1080)
extern "C" MFP_EXPORT const uint8_t *mfp_reassembler_dumped(mfp_reassembler r, size_t *n) {
    if (n) *n = r ? r->dump.size() : 0;
    return r && !r->dump.empty() ? r->dump.data() : nullptr;
}
extern "C" MFP_EXPORT const uint8_t *mfp_reassembler_frames(mfp_reassembler r, size_t *len) {
    if (len) *len = r ? r->frames.size() : 0;
    return r && !r->frames.empty() ? r->frames.data() : nullptr;
}

static bool flow_key(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, FlowKey &k, uint8_t proto = 6) {
    const uint32_t ip = r.net & 0xffff, v = (r.net >> 16) & 15;
    memset(&k, 0, sizeof k);
    k.v = (uint8_t)v; k.proto = proto; k.sport = r.src_port; k.dport = r.dst_port;
    if (v == 4 && ip + 20 <= caplen) { memcpy(k.src, pkt + ip + 12, 4); memcpy(k.dst, pkt + ip + 16, 4); return true; }
    if (v == 6 && ip + 40 <= caplen) { memcpy(k.src, pkt + ip + 8, 16); memcpy(k.dst, pkt + ip + 24, 16); return true; }
    return false;
}

// the reassembled message as a frame: the packet's headers up to its TCP data
// (link layer, any encapsulation levels, IP, TCP), then the buffer; every IP
// length field on the way is set to reach the end of the new data, so the
// device's re-walk finds the same levels (the JSON record's
// "encapsulations" come from the current packet, pkt_proc.cc:1231-1233) and
// the message.  Returns the frame's length (its link type is the packet's).
static uint32_t rebuild(std::vector<uint8_t> &out, const uint8_t *pkt, uint32_t caplen, uint32_t linktype,
                        const mfp_record &r, const mfp_tcp_seg &s, const uint8_t *data, size_t len) {
    const uint32_t ip = r.net & 0xffff;
    uint32_t start = 0;
    mfpe::Chain chain;
    const bool levels = (r.flags & MFP_FLAG_ENCAP) && mfpe::walk(pkt, caplen, linktype, ip, chain);
    if (!levels) start = ip;                                // the inner IP header on its own (LINKTYPE_RAW)
    const size_t at = out.size();
    const bool dtls = s.kind & MFP_SEG_DTLS;
    if (!dtls) {
        out.insert(out.end(), pkt + start, pkt + s.pay_off);
    } else {
        // a DTLS ClientHello: the datagram's headers up to its first record,
        // then that record's header and the handshake header of the whole
        // message (fragment_offset 0, fragment_length = its length), so the
        // re-walk parses the reassembled body as dtls_client_hello's
        // reparse_from_buf does (dtls.h:170-173)
        const uint32_t rec_off = s.pay_off - 25, udp_off = rec_off - 8;
        out.insert(out.end(), pkt + start, pkt + rec_off + 11);            // ..., record type, version, epoch, sequence
        const uint32_t L = (uint32_t)len;
        const uint8_t hs[14] = {(uint8_t)((12 + L) >> 8), (uint8_t)(12 + L),   // record length
                                pkt[s.pay_off - 12],                          // msg_type
                                (uint8_t)(L >> 16), (uint8_t)(L >> 8), (uint8_t)L,
                                pkt[s.pay_off - 8], pkt[s.pay_off - 7],       // message_seq
                                0, 0, 0, (uint8_t)(L >> 16), (uint8_t)(L >> 8), (uint8_t)L};
        out.insert(out.end(), hs, hs + 14);
        const uint32_t ul = 8 + 25 + L;                                      // the UDP length
        out[at + (udp_off - start) + 4] = (uint8_t)(ul >> 8);
        out[at + (udp_off - start) + 5] = (uint8_t)ul;
    }
    out.insert(out.end(), data, data + len);
    const uint32_t flen = (uint32_t)(out.size() - at);
    auto patch = [&](uint32_t off, uint32_t v) {            // ipv4 tot_len (ip.h:124-137) / ipv6 payload_len (:448-474)
        uint8_t *h = out.data() + at + (off - start);
        const uint32_t rest = flen - (off - start);
        if (v == 4) { h[2] = (uint8_t)(rest >> 8); h[3] = (uint8_t)rest; }
        else { h[4] = (uint8_t)((rest - 40) >> 8); h[5] = (uint8_t)(rest - 40); }
    };
    if (levels) for (int k = 0; k < chain.n; k++) patch(chain.lv[k].ip_off, chain.lv[k].ipv);
    patch(ip, (r.net >> 16) & 15);
    while (out.size() % 8) out.push_back(0);                // keep frames 8-byte aligned
    out.resize(out.size() + 16, 0);                         // the readable tail block (include/mfp.h)
    return flen | (levels ? 0x80000000u : 0u);
}

// check_flow's connection-id test (reassembly.hpp:679-688): a flow without one
// matches any; otherwise the incoming id, cut to 20 bytes, must equal it
// (datum::cmp: same bytes and length)
static bool cid_matches(const Flow &f, const uint8_t *cid, uint32_t n) {
    if (n > 20) n = 20;
    return f.cid_len == 0 || (f.cid_len == n && !memcmp(f.cid, cid, n));
}

// check_flow's housekeeping (reassembly.hpp:596-655): at max_entries flows two
// are dropped (active_reap), otherwise up to two expired ones (passive_reap),
// from the persistent reaping iterator over the table
static void reap_step(mfp_reassembler R) {                 // increment_reap_iterator
    if (R->reap_it != R->table.end()) ++R->reap_it;
    else R->reap_it = R->table.begin();
}
static void housekeeping(mfp_reassembler R, uint64_t sec) {
    const bool active = R->table.size() >= kMaxFlows;
    for (int d = 0; d < 2; d++) {
        reap_step(R);
        if (R->reap_it != R->table.end() &&
            (active || sec - R->reap_it->second.f.init_time >= kTimeout))   // reassembly_flow_context::is_expired
            R->reap_it = R->table.erase(R->reap_it);
    }
}

static void drop(mfp_reassembler R, decltype(R->table)::iterator it) {   // clean_curr_flow (reassembly.hpp:830-835)
    R->reap_it = R->table.erase(it);
}

// a flow whose state is final: its buffer rebuilt as a frame for the
// device's re-walk (in the completing packet i's place), the flow consumed
static void complete(mfp_reassembler R, size_t i, const uint8_t *pkt, const mfp_pkt_desc &d, const mfp_record &r,
                     const mfp_tcp_seg &s, decltype(R->table)::iterator it, bool an_path) {
    Flow &f = it->second.f;
    R->who.push_back(i);
    R->who_props.push_back((uint16_t)(1u | (uint32_t)f.flags << 1 | (uint32_t)f.ovl << 8));
    mfp_pkt_desc d2;
    d2.offset = R->frames.size();
    if (s.kind & MFP_SEG_QUIC) {
        // a QUIC Initial: the packet itself, then the reassembled CRYPTO data
        // its ClientHello is parsed from (include/mfp.h MFP_DESC_QUIC_CRYPTO)
        std::vector<uint8_t> &o = R->frames;
        o.insert(o.end(), pkt, pkt + d.caplen);
        while (o.size() % 8) o.push_back(0);
        const uint32_t L = (uint32_t)f.contiguous;
        const uint8_t hdr[8] = {(uint8_t)L, (uint8_t)(L >> 8), (uint8_t)(L >> 16), (uint8_t)(L >> 24), 0, 0, 0, 0};
        o.insert(o.end(), hdr, hdr + 8);
        o.insert(o.end(), f.buf, f.buf + L);
        while (o.size() % 8) o.push_back(0);
        o.resize(o.size() + 16, 0);
        d2.caplen = d.caplen;
        d2.linktype = d.linktype;
        d2.flags = MFP_DESC_QUIC_CRYPTO;
    } else {
        const uint32_t fl = rebuild(R->frames, pkt, d.caplen, d.linktype, r, s, f.buf, f.contiguous);
        d2.caplen = fl & 0x7fffffffu;
        d2.linktype = (fl >> 31) ? d.linktype : (uint16_t)101;   // the packet's, or LINKTYPE_RAW
        d2.flags = 0;
    }
    R->desc2.push_back(d2);
    drop(R, it);                                              // consumed, then clean_curr_flow
    if (an_path) R->more_state = false;                       // finalize_reassembly_flow (reassembly.hpp:1218-1228)
}

// one DTLS ClientHello fragment (process_udp_data pkt_proc.cc:896-945 ->
// process_udp_offset_reassembly reassembly.hpp:1036-1100 ->
// tcp_reassembler::process_udp_data_pkt :748-783): the first fragment of a
// message opens a flow keyed by the 5-tuple and the message_seq; later ones
// fill it by fragment_offset; a complete (or truncated) buffer is
// fingerprinted in the completing packet's place; the fragments before write
// no record.  Fragments that cannot take part are fingerprinted on their own.
template <class NoRecord>
static void dtls_fragment(mfp_reassembler R, size_t i, const uint8_t *arena, const mfp_pkt_desc *desc,
                          const uint64_t *ts_ns, mfp_record *rec, bool an_path, NoRecord &no_record) {
    const mfp_tcp_seg &s = R->seg[i];
    const mfp_record &r = rec[i];
    const uint8_t *pkt = arena + desc[i].offset;
    const uint32_t frag_len = s.pay_len, frag_off = s.seq, more_bytes = s.more;
    if (frag_len > kMaxData || frag_len == 0) return;
    if (frag_off == 0 && !more_bytes) return;                        // a complete message
    if ((uint64_t)frag_len + more_bytes > kMaxData) return;         // beyond the buffer
    if (s.pay_off < 33 || (uint64_t)s.pay_off + frag_len > desc[i].caplen) return;
    {   // rebuild() writes a UDP length 8 bytes before the fragment's record:
        // only a handshake record right behind the UDP header takes part
        const uint32_t ip = r.net & 0xffff, ipv = (r.net >> 16) & 15;
        const uint32_t ip_end = ip + (ipv == 4 ? 4u * (pkt[ip] & 15u) : 40u);
        if (pkt[s.pay_off - 25] != 22 || s.pay_off - 33 < ip_end) return;
    }
    FlowKey k;
    if (!flow_key(pkt, desc[i].caplen, r, k, 17)) return;
    const uint8_t cid[2] = {pkt[s.pay_off - 8], pkt[s.pay_off - 7]};   // message_seq, big-endian (dtls.h:119)
    const uint64_t sec = ts_ns ? ts_ns[i] / 1000000000ull : 0;
    auto cid_ok = [&](const Flow &f) { return cid_matches(f, cid, 2); };
    housekeeping(R, sec);                                            // check_flow (reassembly.hpp:669-692)
    auto it = R->table.find(k);
    if (it != R->table.end() && !cid_ok(it->second.f)) return;      // another message on this 5-tuple: standalone
    if (it == R->table.end() && !more_bytes) return;                 // a later fragment without a flow: standalone
    const bool first = it == R->table.end();                         // udp_segment{init_seg = true} (:1071-1080)
    R->dump[i] = 1;                                                  // dump_pkt (:1074, :1079)
    housekeeping(R, sec);                                            // process_udp_data_pkt's own check_flow
    it = R->table.find(k);
    if (it != R->table.end() && !cid_ok(it->second.f)) { no_record(i); return; }
    const uint8_t *data = pkt + s.pay_off;
    if (it == R->table.end()) {                                      // init_reassembly
        auto &e = R->table[k];
        e.f.init(frag_len, frag_off, first ? more_bytes : 0, false, sec, data, frag_len);
        e.f.cid[0] = cid[0]; e.f.cid[1] = cid[1]; e.f.cid_len = 2;
        it = R->table.find(k);
    } else {
        Flow &f = it->second.f;
        if (sec - f.init_time >= kTimeout) { f.state = S_TRUNCATED; f.flags |= 1u << F_TIMEOUT; }   // set_expired
        else f.add(frag_len, frag_off, data, frag_len);
    }
    const Flow &f = it->second.f;
    if (f.state == S_SUCCESS || f.state == S_TRUNCATED) {
        complete(R, i, pkt, desc[i], r, s, it, an_path);
    } else {
        no_record(i);
        if (an_path) R->more_state = true;                          // in_progress (pkt_proc.cc:1659-1661)
    }
}

// ---- QUIC Initials whose ClientHello spans datagrams
// (process_udp_data pkt_proc.cc:933-939 -> process_quic_reassembly
// reassembly.hpp:895-1033 over the same flow table, keyed by the 5-tuple and
// the connection id)

// variable_length_integer (quic_vli.hpp), as k_quic reads it: a short read
// nulls the cursor and yields what was read
static uint64_t hvli(HC &c) {
    uint64_t b = 0;
    hrd(c, 1, b);
    const int len = (b & 0xc0) == 0xc0 ? 8 : (b & 0xc0) == 0x80 ? 4 : (b & 0xc0) == 0x40 ? 2 : 1;
    uint64_t v = b & 0x3f;
    for (int k = 1; k < len; k++) { uint64_t x = 0; hrd(c, 1, x); v = v * 256 + x; }
    return v;
}

// the frame loop (quic_init quic.h:1532-1552; strict: quic_init_decry::parse
// quic.h:1369-1390), the same walk as k_quic's quic_frames over the plaintext
// the device decrypted
static bool quic_frames_host(HC p, bool strict, QCrypto &q) {
    while (p.d && p.d < p.e) {
        uint64_t t = 0;
        hrd(p, 1, t);
        bool crypto = false;
        uint64_t off = 0, len = 0;
        HC data{nullptr, nullptr};
        if (t == 0x06) {
            off = hvli(p); len = hvli(p);
            hparse(data, p, (long)len);
            crypto = true;
        } else if (t == 0x1c) {
            hvli(p); hvli(p);
            const uint64_t rl = hvli(p);
            HC r; hparse(r, p, (long)rl);
        } else if (t == 0x02 || t == 0x03) {
            hvli(p); hvli(p);
            const uint64_t rc = hvli(p);
            hvli(p);
            if (rc > 1000) hnull(p);
            else for (uint64_t k = 0; k < rc && p.d && p.d < p.e; k++) { hvli(p); hvli(p); }
            if (t == 0x03) { hvli(p); hvli(p); hvli(p); }
        } else if (t != 0x00 && t != 0x01) {
            return !strict;
        }
        if (strict && !p.d) return false;
        if (crypto && data.d && data.d < data.e) q.add(off, len, data.d);
    }
    return true;
}

// quic_init's ctor (quic.h:1513-1528) before it decrypts: an Initial whose
// protected first byte has zero reserved bits is first parsed as already
// decrypted (quic_init_decry::parse, strict), over the payload after the
// packet-number length the protected byte names; when that parse fails, the
// CRYPTO frames it read stay in the buffer (crypto_buffer.reset() keeps the
// bytes) and show through the gaps the decrypted frames leave.  The header is
// quic_initial_packet::parse (quic.h:421-522), as k_quic's quic_hdr reads it.
static void quic_stale_bytes(const uint8_t *pay, uint32_t n, QCrypto &q) {
    if (n < 1184) return;                                     // min_len_pdu quic.h:525
    HC d{pay, pay + n};
    uint64_t ci = 0, v = 0;
    hrd(d, 1, ci);
    HC x; hparse(x, d, 4);
    hrd(d, 1, v);
    if (v > 20 || !d.d) return;
    hparse(x, d, (long)v);
    hrd(d, 1, v);
    if (v > 20 || !d.d) return;
    hparse(x, d, (long)v);
    const uint64_t tl = hvli(d);
    hparse(x, d, (long)tl);
    const uint64_t len = hvli(d);
    if (!d.d || (uint64_t)(d.e - d.d) < len || len < 64) return;   // min_len_pn_and_payload quic.h:524
    HC payload; hparse(payload, d, (long)len);
    if (!payload.d || payload.d >= payload.e || (ci & 0x0c)) return;
    quic_frames_host(HC{payload.d + (ci & 3) + 1, payload.e}, true, q);
}

// the long header's connection ids (quic_initial_packet::parse quic.h:421-522);
// get_cid: the DCID when not empty, else the SCID (quic.h:1611-1617)
static bool quic_cid(const uint8_t *pay, uint32_t n, const uint8_t *&cid, uint32_t &cid_len) {
    HC d{pay, pay + n};
    uint64_t v;
    hrd(d, 1, v);
    HC ver; hparse(ver, d, 4);
    hrd(d, 1, v);
    if (v > 20 || !d.d) return false;
    HC dcid; hparse(dcid, d, (long)v);
    hrd(d, 1, v);
    if (v > 20 || !d.d) return false;
    HC scid; hparse(scid, d, (long)v);
    if (!dcid.d || !scid.d) return false;
    if (dcid.e > dcid.d) { cid = dcid.d; cid_len = (uint32_t)(dcid.e - dcid.d); }
    else { cid = scid.d; cid_len = (uint32_t)(scid.e - scid.d); }
    return true;
}

// one QUIC Initial through process_quic_reassembly: its CRYPTO data opens or
// feeds the flow of its 5-tuple and connection id; a complete (or truncated)
// buffer is fingerprinted in the completing packet's place, the Initials
// before it write no record, the rest are taken on their own
template <class NoRecord>
static void quic_initial(mfp_reassembler R, size_t i, const uint8_t *arena, const mfp_pkt_desc *desc,
                         const uint64_t *ts_ns, mfp_record *rec, const char *fp_arena, bool an_path,
                         NoRecord &no_record) {
    const mfp_tcp_seg &s = R->seg[i];
    const mfp_record &r = rec[i];
    const uint8_t *pkt = arena + desc[i].offset;
    const uint32_t more_bytes = s.more;                      // udp_pkt.additional_bytes_needed()
    if (more_bytes > kMaxData) return;                       // pkt_proc.cc:935-937
    // the plaintext from the record's sidecar (JSON block flag bit 2)
    if (!(r.flags & MFP_FLAG_SIDECAR)) return;
    const uint8_t *sc = (const uint8_t *)fp_arena + r.fp_offset + ((r.fp_len + 7) & ~7u) + 8;
    const uint32_t jo = (uint32_t)sc[6] | (uint32_t)sc[7] << 8;
    if (!jo) return;
    const uint8_t *j = sc + jo;
    if (!(j[10] & 4)) return;                                // no CRYPTO data that could need reassembly
    const uint32_t pt_len = (uint32_t)j[4] | (uint32_t)j[5] << 8;
    const bool pre = j[10] & 1;
    QCrypto &q = R->qc;
    q.reset();
    if (!pre) {                                              // the failed already-decrypted parse's bytes
        quic_stale_bytes(pkt + s.pay_off, s.pay_len, q);
        q.reset_meta();
    }
    quic_frames_host(HC{j + 16, j + 16 + pt_len}, pre, q);
    // get_crypto_buf (quic.h:1600-1609): the bytes from the smallest CRYPTO offset
    const uint32_t crypto_offset = q.min_crypto_offset;
    const uint32_t crypto_len = (!q.buf_len || crypto_offset == 0xffffffffu || crypto_offset > q.buf_len)
                                    ? 0u : (uint32_t)(q.buf_len - crypto_offset);
    if (crypto_len > kMaxData) return;
    if (!crypto_len || (!crypto_offset && !more_bytes)) return;          // a complete Initial
    if ((uint64_t)crypto_len + more_bytes > kMaxData) return;
    if (s.pay_off + (uint64_t)s.pay_len > desc[i].caplen) return;
    const uint8_t *cid = nullptr;
    uint32_t cid_len = 0;
    if (!quic_cid(pkt + s.pay_off, s.pay_len, cid, cid_len)) return;
    FlowKey k;
    if (!flow_key(pkt, desc[i].caplen, r, k, 17)) return;
    const uint64_t sec = ts_ns ? ts_ns[i] / 1000000000ull : 0;
    const bool missing = q.missing();
    // check_flow (reassembly.hpp:669-692)
    housekeeping(R, sec);
    auto it = R->table.find(k);
    if (it != R->table.end() && !cid_matches(it->second.f, cid, cid_len)) return;   // another connection: standalone
    const bool fresh = it == R->table.end();
    if (fresh && !more_bytes) return;
    // process_udp_data_pkt (reassembly.hpp:748-783) for one segment of the
    // packet's crypto buffer: open the flow, or add to it while in progress
    bool lost = false;                                       // curr_flow reset by a connection-id mismatch
    auto segment = [&](bool init, uint64_t off, uint64_t len) {
        housekeeping(R, sec);
        auto f = R->table.find(k);
        if (f != R->table.end() && !cid_matches(f->second.f, cid, cid_len)) { lost = true; return; }
        lost = false;
        const uint8_t *data = q.buf + off;
        if (f == R->table.end()) {                           // init_reassembly (UDP ctor reassembly.hpp:224-275)
            auto &e = R->table[k];
            e.f.init((uint32_t)len, (uint32_t)off, init ? more_bytes : 0, false, sec, data, (uint32_t)len);
            e.f.cid_len = cid_len;
            memcpy(e.f.cid, cid, cid_len);
        } else if (f->second.f.state == S_PROGRESS) {        // continue_reassembly
            Flow &fl = f->second.f;
            if (sec - fl.init_time >= kTimeout) { fl.state = S_TRUNCATED; fl.flags |= 1u << F_TIMEOUT; }
            else fl.add((uint32_t)len, (uint32_t)off, data, (uint32_t)len);
        }
    };
    const uint64_t max_end = (uint64_t)crypto_offset + crypto_len;
    auto usable = [&](uint32_t x) {
        return q.flen[x] && q.foff[x] + q.flen[x] <= max_end && q.foff[x] <= 0xffffffffu && q.flen[x] <= 0xffffffffu;
    };
    if (fresh) {
        if (!missing) {
            segment(true, crypto_offset, crypto_len);
            R->dump[i] = 1;                                  // dump_pkt (reassembly.hpp:931)
        } else {
            if (q.count == 0 || q.first == 0xffff) return;
            if (q.first >= q.count) return;                  // frames[first_frame_idx] past the list: not restated
            R->dump[i] = 1;                                  // dump_pkt (reassembly.hpp:981)
            const uint32_t ff = q.first;
            if (q.flen[ff] < 10) {                           // min_crypto_data (quic.h:1571-1578)
                const uint64_t fo = q.foff[ff];
                if (fo < max_end && fo <= 0xffffffffu) {
                    uint64_t sl = 10;
                    if (max_end - fo < sl) sl = max_end - fo;
                    if (sl) segment(true, fo, sl);
                }
            } else if (usable(ff)) {
                segment(true, q.foff[ff], q.flen[ff]);
            }
            for (uint32_t x = 0; x < q.count; x++)
                if (x != ff && usable(x)) segment(false, q.foff[x], q.flen[x]);
        }
    } else {
        if (it->second.f.state != S_PROGRESS) { no_record(i); return; }   // success / truncated: return false
        if (!missing) {
            segment(false, crypto_offset, crypto_len);
            R->dump[i] = 1;                                  // dump_pkt (reassembly.hpp:988)
        } else {
            if (q.count == 0) return;
            R->dump[i] = 1;                                  // dump_pkt (reassembly.hpp:1009)
            for (uint32_t x = 0; x < q.count; x++)
                if (usable(x)) segment(false, q.foff[x], q.flen[x]);
        }
    }
    it = R->table.find(k);
    if (!lost && it != R->table.end() && (it->second.f.state == S_SUCCESS || it->second.f.state == S_TRUNCATED)) {
        complete(R, i, pkt, desc[i], r, s, it, an_path);     // reparse_crypto_buf, set_completed
    } else {
        no_record(i);
        if (an_path && !lost && it != R->table.end()) R->more_state = true;   // in_progress (pkt_proc.cc:1660-1662)
    }
}

// the flow table over one batch, in stream order (process_tcp_data
// pkt_proc.cc:773-893).  an_path: the analysis_context path
// (analyze_ip_packet pkt_proc.cc:1624-1646): SYN, SYN/ACK and RST are skipped
// and every IP packet resets flow_state_pkts_needed (more[i]; non-IP packets keep it).
static long long reassemble(mfp_context ctx, mfp_reassembler R, const uint8_t *arena, size_t arena_len,
                            const mfp_pkt_desc *desc, size_t n, const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                            size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc, bool an_path, uint8_t *more) {
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
    R->dump.assign(n, 0);
    auto no_record = [&](size_t i) {                        // process_tcp_data returned false
        rec[i].flags &= (uint8_t)~MFP_FLAG_EMIT; rec[i].fp_type = 0; rec[i].fp_len = 0; R->quiet[i] = 1;
    };
    for (size_t i = 0; i < n; i++) {
        props[i] = 0;
        const mfp_tcp_seg &s = R->seg[i];
        if (an_path && (s.kind & MFP_SEG_IP)) R->more_state = false;   // analysis.reinit() (pkt_proc.cc:1609)
        if (an_path && (s.kind & MFP_SEG_TCP)) {
            if (s.kind & MFP_SEG_SYN_RST) {                 // handshake control packets (pkt_proc.cc:1631-1633)
                no_record(i);
                if (more) more[i] = 0;
                continue;
            }
        }
        if (more) more[i] = R->more_state;
        if (s.kind & MFP_SEG_DTLS) {
            dtls_fragment(R, i, arena, desc, ts_ns, rec, an_path, no_record);
            if (more) more[i] = R->more_state;
            continue;
        }
        if (s.kind & MFP_SEG_QUIC) {
            quic_initial(R, i, arena, desc, ts_ns, rec, fp_arena, an_path, no_record);
            if (more) more[i] = R->more_state;
            continue;
        }
        if (!(s.kind & MFP_SEG_DATA)) {
            if (an_path && (s.kind & MFP_SEG_TCP)) no_record(i);   // empty data: process_tcp_data returns false
            continue;
        }
        mfp_record &r = rec[i];
        const uint8_t *pkt = arena + desc[i].offset;
        const uint32_t data_len = s.pay_len;
        const uint32_t more_bytes = s.more;
        const bool supp = s.kind & MFP_SEG_SUPPLEMENTARY;
        const bool mono = r.msg == 0;                       // std::monostate: no message parsed
        if (!more_bytes && !mono && !supp) continue;        // a complete message
        if (more_bytes > kMaxData || data_len > kMaxData) continue;   // cannot be reassembled
        FlowKey k;
        if (!flow_key(pkt, desc[i].caplen, r, k)) continue;
        const uint64_t sec = ts_ns ? ts_ns[i] / 1000000000ull : 0;
        housekeeping(R, sec);                               // check_flow (pkt_proc.cc:840)
        auto it = R->table.find(k);
        const uint8_t *data = pkt + s.pay_off;
        const uint32_t avail = s.pay_off + (uint64_t)data_len <= desc[i].caplen ? data_len : 0;
        const bool had = it != R->table.end();
        if (!had) {
            if (supp) continue;                             // not in reassembly: taken as complete
            if (!more_bytes) { no_record(i); continue; }
        }
        R->dump[i] = 1;                                     // dump_pkt (pkt_proc.cc:852, 862, 866)
        // 0: in order, after the flow's contiguous bytes (pkt_proc.cc:856-861)
        const uint32_t seq = had && !s.seq ? (uint32_t)it->second.f.contiguous : s.seq;
        // process_tcp_data_pkt (reassembly.hpp:717-746): its own check_flow, then
        // open the flow (again, if that check reaped it) or continue it
        housekeeping(R, sec);
        it = R->table.find(k);
        if (it == R->table.end()) {
            auto &e = R->table[k];
            e.f.init(data_len, seq, had ? 0 : more_bytes, (s.kind & MFP_SEG_SSH) != 0, sec, data, avail);
            it = R->table.find(k);
        } else if (it->second.f.state == S_PROGRESS) {
            Flow &f = it->second.f;
            if (sec - f.init_time >= kTimeout) {            // continue_reassembly: set_expired
                f.state = S_TRUNCATED;
                f.flags |= 1u << F_TIMEOUT;
            } else {
                f.add(data_len, seq, data, avail);
            }
        }
        Flow &f = it->second.f;
        if (f.state == S_SUCCESS || f.state == S_TRUNCATED) {   // is_ready: fingerprint the buffer
            complete(R, i, pkt, desc[i], r, s, it, an_path);
        } else {
            no_record(i);                                   // no record for this segment
            if (an_path) R->more_state = true;              // in_progress (pkt_proc.cc:1636-1638)
        }
        if (more) more[i] = R->more_state;
    }
    // dump_pkt is cleared only by packets that reach the IP layer
    // (ip_write_json pkt_proc.cc:1078-1080, analyze_ip_packet :1611-1613); a
    // packet that does not (ARP, an unsupported ethertype) keeps the value the
    // packet before it left
    for (size_t i = 0; i < n; i++) {
        if (R->seg[i].kind & MFP_SEG_IP) R->dump_carry = R->dump[i];
        else R->dump[i] = R->dump_carry;
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
            if (r2.fp_type || (r2.flags & MFP_FLAG_SIDECAR)) r2.fp_offset += (uint64_t)used;
            // the reassembler's own "reassembly_properties" replace {"truncated":true}
            // (write_reassembly_properties reassembly.hpp:1231-1247)
            if (!an_path) r2.flags &= (uint8_t)~MFP_FLAG_TRUNCATED;
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

extern "C" MFP_EXPORT long long mfp_process_batch_reassembly(mfp_context ctx, mfp_reassembler R, const uint8_t *arena,
                                                             size_t arena_len, const mfp_pkt_desc *desc, size_t n,
                                                             const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                                                             size_t fp_cap, uint16_t *props,
                                                             mfp_pkt_desc *out_desc) {
    return reassemble(ctx, R, arena, arena_len, desc, n, ts_ns, rec, fp_arena, fp_cap, props, out_desc, false, nullptr);
}

// the packets the reference analyses -- those with a record, the reassembled
// messages in their completing packets' places, nothing for the segments that
// only fed a buffer (zero-length descriptors) -- fingerprinted and classified
// once more in stream order, so the unknown-TLS sightings keep the
// reference's order
static long long classify_pass(mfp_context ctx, mfp_reassembler R, const uint8_t *arena, size_t arena_len, size_t n,
                               mfp_record *rec, char *fp_arena, size_t fp_cap, const mfp_pkt_desc *out_desc,
                               mfp_analysis *analysis, double *attr_prob) {
    R->merged.assign(arena, arena + arena_len);
    R->merged.insert(R->merged.end(), R->frames.begin(), R->frames.end());
    R->merged.resize(R->merged.size() + 16, 0);
    R->desc3.assign(out_desc, out_desc + n);
    for (size_t i = 0; i < n; i++) if (R->quiet[i]) R->desc3[i].caplen = 0;
    return mfp_process_batch_host_ex(ctx, R->merged.data(), R->merged.size(), R->desc3.data(), n, rec, fp_arena, fp_cap,
                                     analysis, attr_prob);
}

// --analysis with reassembly (write_json with a classifier, pkt_proc.cc:1195-1238)
extern "C" MFP_EXPORT long long mfp_process_batch_reassembly_analysis(
    mfp_context ctx, mfp_reassembler R, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc, size_t n,
    const uint64_t *ts_ns, mfp_record *rec, char *fp_arena, size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc,
    mfp_analysis *analysis, double *attr_prob) {
    if (!mfp_analysis_enabled(ctx)) { mfp_set_error("the context has no classifier"); return -1; }
    if (n && (!analysis || !out_desc)) { mfp_set_error("null argument"); return -1; }
    long long used = reassemble(ctx, R, arena, arena_len, desc, n, ts_ns, rec, fp_arena, fp_cap, props, out_desc, false,
                                nullptr);
    if (used < 0) return used;
    used = classify_pass(ctx, R, arena, arena_len, n, rec, fp_arena, fp_cap, out_desc, analysis, attr_prob);
    if (used < 0) return used;
    for (size_t i = 0; i < n; i++) if (props[i] & 1) rec[i].flags &= (uint8_t)~MFP_FLAG_TRUNCATED;
    return used;
}

// the analysis_context path with reassembly (analyze_ip_packet pkt_proc.cc:1597-1662)
extern "C" MFP_EXPORT long long mfp_process_batch_reassembly_context(
    mfp_context ctx, mfp_reassembler R, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc, size_t n,
    const uint64_t *ts_ns, mfp_record *rec, char *fp_arena, size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc,
    mfp_analysis *analysis, double *attr_prob, uint8_t *more_pkts) {
    if (!ctx || !R) { mfp_set_error("null context or reassembler"); return -1; }
    if (mfp_context_mode(ctx) != MFP_MODE_ANALYSIS) {
        mfp_set_error("mfp_process_batch_reassembly_context needs a context created with MFP_MODE_ANALYSIS");
        return -1;
    }
    if (analysis && !mfp_analysis_enabled(ctx)) { mfp_set_error("the context has no classifier"); return -1; }
    if (n && !out_desc) { mfp_set_error("null argument"); return -1; }
    long long used = reassemble(ctx, R, arena, arena_len, desc, n, ts_ns, rec, fp_arena, fp_cap, props, out_desc, true,
                                more_pkts);
    if (used < 0 || !analysis) return used;
    used = classify_pass(ctx, R, arena, arena_len, n, rec, fp_arena, fp_cap, out_desc, analysis, attr_prob);
    if (used < 0) return used;
    // detect_truncation (reassembly.hpp:1183-1196): a reassembled message whose
    // flow was truncated is a truncated fingerprint -> unlabeled (pkt_proc.cc:1716-1719)
    const uint16_t trunc_bits = (uint16_t)(((1u << F_TRUNCATED) | (1u << F_TIMEOUT) | (1u << F_OUT_OF_BUFFER) |
                                            (1u << F_MAX_SEG) | (1u << F_MISSING)) << 1);
    for (size_t i = 0; i < n; i++)
        if ((props[i] & 1) && (props[i] & trunc_bits) && (analysis[i].flags & MFP_AN_VALID)) analysis[i].status = 3;
    return used;
}
