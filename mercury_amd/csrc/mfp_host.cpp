// mfp_host.cpp -- host side of libmercury_amd.so: context, configuration
// (the reference's packet_filter_cfg syntax, global_config.h:143-153,
// 246-275, 348-368), device buffers and the C-ABI batch entry points of
// include/mfp.h.  There is no CPU fallback: without a HIP device the calls
// fail with an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_analysis.h"
#include "mfp_common.hpp"
#include "mfp_internal.h"

extern "C" int mfp_launch_analysis(const mfp_classifier_dev *D, const mfp_seen_tab *T, const uint8_t *arena,
                                   const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, const uint8_t *fp_arena,
                                   mfp_analysis *out, double *attr_prob, uint32_t *pending, void *work, void *lanel,
                                   void *deferred, uint32_t *seg_n, unsigned long long *stats, uint32_t mode,
                                   uint32_t lane_max_p, void *huge_rows, hipStream_t stream, mfp_prof *prof);
extern "C" size_t mfp_analysis_huge_bytes(uint32_t max_nproc);
extern "C" void mfp_analysis_segments(uint64_t n, uint32_t *nseg, uint32_t *seg_cap);
extern "C" int mfp_launch_seen_export(const mfp_seen_tab *T, uint32_t u, mfp_sighting *out, hipStream_t stream);
extern "C" int mfp_launch_seen_sequence(const mfp_classifier_dev *D, const mfp_seen_tab *T, uint64_t n,
                                        const mfp_record *rec, const uint8_t *fp_arena, uint32_t *pending,
                                        const uint32_t *group_off, uint64_t *seq, hipStream_t stream);
extern "C" int mfp_launch_analysis_resolve(const mfp_classifier_dev *D, const mfp_seen_tab *T, uint64_t n,
                                           const mfp_record *rec, const uint8_t *fp_arena, mfp_analysis *out,
                                           uint32_t *pending, uint32_t mode, const uint8_t *seen_pos,
                                           const uint32_t *group_off, const uint8_t *seen_seq, hipStream_t stream,
                                           mfp_prof *prof);

extern "C" int mfp_launch_fingerprint(uint32_t select, uint32_t block, uint32_t tls_format, uint32_t mode,
                                      const uint8_t *arena,
                                      const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, mfp_tcp_seg *seg,
                                      uint8_t *fp_arena,
                                      uint64_t fp_cap, unsigned long long *fp_used, uint32_t *work,
                                      unsigned long long *bin_count, int strategy, uint32_t bin_seg_mask,
                                      uint32_t bin_lds_mask, uint32_t quic_format, uint8_t *quic_scratch,
                                      uint32_t quic_grid, hipStream_t stream, mfp_prof *prof,
                                      unsigned long long *fin = nullptr, unsigned long long *host_out = nullptr);
extern "C" size_t mfp_quic_scratch_bytes(uint32_t grid);

extern "C" int mfp_launch_compact(mfp_record *rec, uint64_t n, const uint8_t *src, uint8_t *dst, uint32_t *local,
                                  unsigned long long *block_sum, unsigned long long *total, hipStream_t stream,
                                  mfp_prof *prof);


extern "C" int mfp_launch_compact_small(const mfp_record *rec, uint64_t n, const uint8_t *src, uint8_t *dst_host,
                                        uint64_t cap, mfp_record *rec_host, const unsigned long long *used,
                                        unsigned long long *used_host, const mfp_analysis *an, mfp_analysis *an_host,
                                        const double *ap, double *ap_host, hipStream_t stream, mfp_prof *prof);

static thread_local std::string g_err;

void mfp_set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

extern "C" MFP_EXPORT const char *mfp_last_error(void) { return g_err.c_str(); }
extern "C" MFP_EXPORT uint32_t mfp_reference_version(void) { return (2u << 16) | (18u << 8) | 0u; }

// selection bits, mirrored in mfp_device.hpp (SEL_*) and oracle/mfp_oracle.h
enum : uint32_t {
    SEL_TLS_CH = 1u << 0, SEL_TLS_SH = 1u << 1, SEL_TLS_CERT = 1u << 2, SEL_SSH_CLIENT = 1u << 3,
    SEL_SSH_SERVER = 1u << 4, SEL_HTTP_REQ = 1u << 5, SEL_HTTP_RESP = 1u << 6, SEL_TCP_SYN = 1u << 7,
    SEL_TCP_SYNACK = 1u << 8, SEL_DTLS = 1u << 9, SEL_QUIC = 1u << 10,
    SEL_GRE = 1u << 11, SEL_VXLAN = 1u << 12, SEL_GENEVE = 1u << 13,
    SEL_STUN = 1u << 14, SEL_OPENVPN = 1u << 15,
    SEL_ALL = (1u << 16) - 1,
};

static std::string strip(const std::string &s) {
    std::string o;
    for (char c : s) if (!isspace((unsigned char)c)) o += c;
    return o;
}
static std::string trim(const std::string &s) {
    size_t a = 0, b = s.size();
    while (a < b && isspace((unsigned char)s[a])) a++;
    while (b > a && isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

// global_config::set_protocols (global_config.h:246-276) over the reference's
// protocol names (global_config.h:163-227).  This path's protocols set
// `sel`; the others write no record, and those whose matchers or ports the
// reference consults before one of this path's set their BLK_* bits in
// `block` (traffic_selector proto_identify.h:620-895; mirrored in
// mfp_device.hpp).  "all" sets everything; "none" clears everything
// (proto_identify.h:623-627); a name the reference does not know is refused,
// as set_protocols refuses it.
enum : uint32_t {
    BLK_SMTP = 1u << 0, BLK_DNS_TCP = 1u << 1, BLK_DNS_UDP = 1u << 2, BLK_SMB = 1u << 3, BLK_BT = 1u << 4,
    BLK_MYSQL = 1u << 5, BLK_SOCKS = 1u << 6, BLK_IEC = 1u << 7, BLK_DNP3 = 1u << 8, BLK_LDAP = 1u << 9,
    BLK_NBSS = 1u << 10, BLK_FTP_RESP = 1u << 11, BLK_TACACS = 1u << 12, BLK_RDP = 1u << 13, BLK_KRB5 = 1u << 14,
    BLK_REDIS_REQ = 1u << 15, BLK_REDIS_RESP = 1u << 16, BLK_IMAP_REQ = 1u << 17, BLK_IMAP_RESP = 1u << 18,
    BLK_TELNET = 1u << 19, BLK_IPSEC = 1u << 20, BLK_WIREGUARD = 1u << 21, BLK_SSDP = 1u << 22, BLK_NBDS = 1u << 23,
    BLK_TFTP = 1u << 24, BLK_SNMP = 1u << 25, BLK_SYSLOG = 1u << 26, BLK_ALL = (1u << 27) - 1,
};
struct SelState {
    uint32_t sel = 0, block = 0;
    bool none = false;          // protocols["none"]: cleared at the end (proto_identify.h:623-627)
    std::string warn;           // what the reference logs (printf_err) and goes on from
};
static void add_warning(SelState &st, const std::string &w) { st.warn += (st.warn.empty() ? "" : "; ") + w; }

// set_protocols (global_config.h:246-276), literally: the list is split at
// ','; every token but the last has its spaces removed (the last keeps them:
// the function strips the rest of the string, not the token); the first
// unknown token is logged and ends the list, what was set stays
static void parse_select(const std::string &data, SelState &st) {
    static const std::map<std::string, uint32_t> known = {
        {"none", 0},
        {"tls", SEL_TLS_CH | SEL_TLS_SH | SEL_TLS_CERT}, {"tls.client_hello", SEL_TLS_CH},
        {"tls.server_hello", SEL_TLS_SH}, {"tls.server_certificate", SEL_TLS_CERT},
        {"ssh", SEL_SSH_CLIENT | SEL_SSH_SERVER}, {"ssh.client", SEL_SSH_CLIENT}, {"ssh.server", SEL_SSH_SERVER},
        {"http", SEL_HTTP_REQ | SEL_HTTP_RESP}, {"http.request", SEL_HTTP_REQ}, {"http.response", SEL_HTTP_RESP},
        {"tcp", SEL_TCP_SYN}, {"tcp.syn_ack", SEL_TCP_SYNACK}, {"dtls", SEL_DTLS}, {"quic", SEL_QUIC},
        {"gre", SEL_GRE}, {"vxlan", SEL_VXLAN}, {"geneve", SEL_GENEVE},
        {"stun", SEL_STUN}, {"openvpn_tcp", SEL_OPENVPN},
    };
    static const std::map<std::string, uint32_t> other = {
        {"arp", 0}, {"bittorrent", BLK_BT}, {"cdp", 0}, {"dhcp", 0}, {"dnp3", BLK_DNP3},
        {"dns", BLK_DNS_TCP | BLK_DNS_UDP}, {"icmp", 0}, {"iec", BLK_IEC}, {"kerberos", BLK_KRB5}, {"ldap", BLK_LDAP},
        {"imap", BLK_IMAP_REQ | BLK_IMAP_RESP}, {"imap.request", BLK_IMAP_REQ}, {"imap.response", BLK_IMAP_RESP},
        {"ipsec", BLK_IPSEC}, {"lldp", 0}, {"mdns", BLK_DNS_UDP}, {"nbns", BLK_DNS_UDP}, {"nbds", BLK_NBDS},
        {"nbss", BLK_NBSS}, {"ospf", 0}, {"rdp", BLK_RDP}, {"rfb", 0}, {"sctp", 0}, {"smb", BLK_SMB}, {"smtp", BLK_SMTP},
        {"snmp", BLK_SNMP}, {"ssdp", BLK_SSDP}, {"syslog", BLK_SYSLOG}, {"tacacs", BLK_TACACS}, {"tcp.message", 0},
        {"telnet", BLK_TELNET}, {"tftp", BLK_TFTP}, {"wireguard", BLK_WIREGUARD}, {"mysql", BLK_MYSQL},
        {"tofsee", 0}, {"socks", BLK_SOCKS}, {"ftp", BLK_FTP_RESP}, {"ftp.response", BLK_FTP_RESP},
        {"ftp.request", 0}, {"redis", BLK_REDIS_REQ | BLK_REDIS_RESP}, {"redis.request", BLK_REDIS_REQ},
        {"redis.response", BLK_REDIS_RESP},
    };
    const std::string list = data.empty() ? std::string("all") : data;   // global_config.h:248
    size_t pos = 0;
    while (true) {
        const size_t c = list.find(',', pos);
        const std::string tok = c == std::string::npos ? list.substr(pos) : strip(list.substr(pos, c - pos));
        if (tok == "all") {
            st.sel |= SEL_ALL;
            st.block |= BLK_ALL;
        } else if (auto it = known.find(tok); it != known.end()) {
            if (tok == "none") st.none = true;
            st.sel |= it->second;
        } else if (auto jt = other.find(tok); jt != other.end()) {
            st.block |= jt->second;
        } else {
            add_warning(st, "unrecognized filter command \"" + tok + "\"");
            return;
        }
        if (c == std::string::npos) break;
        pos = c + 1;
    }
}

// fingerprint_format::set_fingerprint_format (global_config.h:55-121),
// literally: a token is substr(start, current_pos) -- a count, not an end --
// with its spaces removed, the last token keeps its spaces; an unknown format
// is logged and ends the list ("using default instead").  The result packs
// the TLS format in bits 0-7 and the QUIC format in bits 8-15.
static void parse_format(const std::string &s, uint32_t &tls_format, SelState &st) {
    auto one = [&](const std::string &tok) -> bool {
        const size_t sl = tok.find('/');
        const std::string proto = tok.substr(0, sl), ver = sl == std::string::npos ? "" : tok.substr(sl + 1);
        if (proto == "tls" && (ver == "" || ver == "1" || ver == "2")) {
            tls_format = (tls_format & ~0xffu) | (ver == "" ? 0u : ver == "1" ? 1u : 2u);
            return true;
        }
        if (proto == "quic" && (ver == "" || ver == "1")) {
            tls_format = (tls_format & ~0xff00u) | (ver == "1" ? 1u << 8 : 0u);
            return true;
        }
        add_warning(st, "unknown fingerprint format: " + tok + "; using default instead");
        return false;
    };
    if (s.empty()) return;
    size_t start = 0, cur;
    while ((cur = s.find(',', start)) != std::string::npos) {
        const std::string tok = strip(s.substr(start, cur));
        start = cur + 1;
        if (!one(tok)) return;
    }
    if (start < s.size()) one(s.substr(start));
}

// global_config(const libmerc_config&) (global_config.h:143-153): a string
// without ';' is the protocol list; otherwise parse_additional_options
// (config_generator.cc:115-162): ';'-separated tokens, trimmed, key=value or a
// bare key; a key no option recognises is taken as a protocol list.  Warnings
// (what the reference logs and goes on from) land in *warn.
//
// The reference's other options (config_generator.cc:28-44,
// global_config.h:350-365) fall in three groups here:
//  * no effect on the records this path writes -- accepted: stats-blocking,
//    max_stats_entries (the stats aggregator, off), dns-json (DNS/mDNS
//    records only, pkt_proc_util.h:284-313: this path writes none),
//    raw-features naming only bittorrent/smb/ssdp (or none), http-body-max=0,
//    and any boolean option set to a value other than "" or "1" (off);
//  * report_os: honoured (*report_os = 1 / 0; -1 when absent);
//  * options that change the records (metadata, certs-json, raw-features of
//    tls/stun/all, crypto-assess, network-behavioral-detections,
//    exposed-creds, http-headers, http-body-max > 0, nonselected-tcp-data,
//    nonselected-udp-data, quic-trial-decryption, minimize-ram,
//    fp_proc_threshold / proc_dst_threshold > 0, stats): REFUSED -- false with
//    the reason in mfp_last_error(), so no caller gets records that differ
//    from the reference's without being told.
bool mfp_parse_config(const char *cfg, uint32_t &sel, uint32_t &tls_format, std::string *resources, bool *analysis,
                      bool *reassembly, uint32_t *block_out, std::string *warn, int *report_os) {
    tls_format = 0;
    if (report_os) *report_os = -1;
    SelState st;
    std::string s = cfg ? cfg : "";
    if (s.find(';') == std::string::npos) {
        parse_select(s, st);
    } else {
        static const char *const no_effect[] = {"stats-blocking", "max_stats_entries", "dns-json"};
        // boolean setters of config_mapper: on for "" or "1" (config_generator.cc:31-43)
        static const char *const refused_on[] = {"metadata", "certs-json", "network-behavioral-detections",
                                                 "nonselected-tcp-data", "nonselected-udp-data", "stats"};
        // extended setters that turn their feature on whatever the value (global_config.h:356-364)
        static const char *const refused_any[] = {"crypto-assess", "exposed-creds", "http-headers",
                                                  "quic-trial-decryption", "minimize-ram"};
        auto refuse = [&](const std::string &key, const std::string &why) {
            mfp_set_error("packet_filter_cfg option \"%s\" %s; libmercury_amd writes the reference's records with it "
                          "off only, and refuses it rather than ignore it", key.c_str(), why.c_str());
            return false;
        };
        auto in = [](const char *const *b, const char *const *e, const std::string &k) { return std::find(b, e, k) != e; };
        size_t pos = 0;
        while (pos <= s.size()) {
            size_t c = s.find(';', pos);
            std::string tok = trim(s.substr(pos, c == std::string::npos ? std::string::npos : c - pos));
            if (!tok.empty()) {
                size_t eq = tok.find('=');
                std::string key = trim(tok.substr(0, eq)), val = eq == std::string::npos ? "" : trim(tok.substr(eq + 1));
                const bool on = val.empty() || val == "1";
                if (key == "select" || key == "-s" || key == "--select") parse_select(val, st);
                else if (key == "format") parse_format(val, tls_format, st);
                else if (key == "resources") { if (resources) *resources = val; }
                else if (key == "analysis" || key == "-a" || key == "--analysis") {
                    if (analysis) *analysis = on;
                } else if (key == "reassembly" || key == "tcp-reassembly") {   // global_config.h:354-355
                    if (reassembly) *reassembly = true;
                } else if (key == "report_os") {                              // config_generator.cc:35
                    if (report_os) *report_os = on ? 1 : 0;
                } else if (in(std::begin(no_effect), std::end(no_effect), key)) {
                } else if (in(std::begin(refused_on), std::end(refused_on), key)) {
                    if (on) return refuse(key, "changes the JSON records (write_metadata pkt_proc_util.h:264-333, "
                                               "pkt_proc.cc:1157-1253)");
                } else if (in(std::begin(refused_any), std::end(refused_any), key)) {
                    return refuse(key, "changes the records or the classifier (global_config.h:356-364)");
                } else if (key == "raw-features") {                           // global_config.h:277-294
                    for (const char *p : {"all", "tls", "stun"}) {
                        size_t at = 0;
                        std::string v = val;
                        v.erase(std::remove_if(v.begin(), v.end(), ::isspace), v.end());
                        while ((at = v.find(p, at)) != std::string::npos) {
                            const size_t end = at + strlen(p);
                            if ((at == 0 || v[at - 1] == ',') && (end == v.size() || v[end] == ','))
                                return refuse(key + "=" + val, "adds the \"features\" string to TLS/STUN records "
                                                               "(tls.h:1909-1913)");
                            at = end;
                        }
                    }
                } else if (key == "http-body-max") {                          // global_config.h:327-345
                    if (val != "0") return refuse(key + "=" + val, "adds HTTP bodies to the records");
                } else if (key == "fp_proc_threshold" || key == "proc_dst_threshold") {
                    if (strtof(val.c_str(), nullptr) > 0.0f)                  // analysis.h:836: fingerprint_db_lite.json
                        return refuse(key + "=" + val, "switches the classifier's database");
                } else {
                    parse_select(key, st);   // config_generator.cc:156-160
                }
            }
            if (c == std::string::npos) break;
            pos = c + 1;
        }
    }
    sel = st.none ? 0 : st.sel;
    if (block_out) *block_out = st.none ? 0 : st.block;
    if (warn) *warn = st.warn;
    return true;
}

extern "C" MFP_EXPORT int mfp_parse_filter(const char *cfg, uint32_t *select, uint32_t *tls_format) {
    return mfp_parse_filter_ex(cfg, select, tls_format, nullptr);
}

extern "C" MFP_EXPORT int mfp_parse_filter_ex(const char *cfg, uint32_t *select, uint32_t *tls_format,
                                              uint32_t *other) {
    uint32_t sel = 0, fmt = 0, blk = 0;
    std::string warn;
    if (!mfp_parse_config(cfg, sel, fmt, nullptr, nullptr, nullptr, &blk, &warn)) return -1;
    if (select) *select = sel;
    if (tls_format) *tls_format = fmt;
    if (other) *other = blk;
    if (!warn.empty()) { mfp_set_error("%s", warn.c_str()); return 1; }
    return 0;
}

// ---------------------------------------------------------------------------
// per-kernel timing: HIP events recorded on the launch stream around every
// kernel launch of a context (mfp_profile_enable); read back by name
// ---------------------------------------------------------------------------
struct mfp_prof {
    struct Pending { const char *name; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    std::vector<std::string> names;                  // first-launch order
    std::map<std::string, std::pair<uint64_t, double>> acc;   // launches, total ms

    hipEvent_t get() {
        hipEvent_t e = nullptr;
        if (!pool.empty()) { e = pool.back(); pool.pop_back(); return e; }
        (void)hipEventCreate(&e);
        return e;
    }
    int collect() {
        int rc = 0;
        for (auto &p : pending) {
            float ms = 0.f;
            if (hipEventSynchronize(p.b) != hipSuccess || hipEventElapsedTime(&ms, p.a, p.b) != hipSuccess) rc = -1;
            auto it = acc.find(p.name);
            if (it == acc.end()) { names.push_back(p.name); it = acc.emplace(p.name, std::make_pair(0ull, 0.0)).first; }
            it->second.first++;
            it->second.second += ms;
            pool.push_back(p.a); pool.push_back(p.b);
        }
        pending.clear();
        return rc;
    }
    void reset() { (void)collect(); acc.clear(); names.clear(); }
    ~mfp_prof() {
        (void)collect();
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

void mfp_prof_begin(mfp_prof *p, const char *kernel, hipStream_t s) {
    hipEvent_t a = p->get();
    (void)hipEventRecord(a, s);
    p->pending.push_back({kernel, a, nullptr});
}

void mfp_prof_end(mfp_prof *p, hipStream_t s) {
    hipEvent_t b = p->get();
    (void)hipEventRecord(b, s);
    p->pending.back().b = b;
}

// device scratch of one batch in flight: classify bins, classifier lists and
// counters, and for host batches the staging copies of the batch itself.
// Slot 0 serves the synchronous calls; slots 1 and 2 alternate in
// mfp_process_pipelined, so two batches can be in flight on two streams.
struct Slot {
    unsigned long long *d_used = nullptr;   // fp arena counters of host batches
    unsigned long long *d_bins = nullptr;   // per-bin packet counts of the classify pass (9 bins)
    uint8_t *d_quic = nullptr;              // k_quic's per-lane scratch (decrypted payload, CRYPTO buffer)
    uint32_t *d_work = nullptr; size_t cap_work = 0;   // bin index lists / fallback list / bin ids
    unsigned long long *d_an_stats = nullptr;
    uint32_t *d_pending = nullptr; size_t cap_pending = 0;   // unknown-TLS sightings (bitmap)
    // the classifier's per-wave segments (mfp_analysis_segments): work items
    // (16 B), lane-scored and wave-scored packets (64 B each), counts
    uint4 *d_work_items = nullptr; size_t cap_work_items = 0;
    uint4 *d_lanel = nullptr; size_t cap_lanel = 0;
    uint4 *d_deferred = nullptr; size_t cap_deferred = 0;
    uint4 *d_huge = nullptr; size_t cap_huge = 0;     // k_analyze_huge's score rows (archives with P > 4096)
    uint32_t *d_segn = nullptr; size_t cap_segn = 0;
    mfp_analysis *d_an = nullptr; size_t cap_an = 0;
    double *d_ap = nullptr; size_t cap_ap = 0;               // archive-tag probabilities of host batches
    // the unknown-TLS sightings of the batch analysed in this slot (mfp_prevalence)
    mfp_seen_tab seen;
    mfp_sighting *d_sight = nullptr;                          // distinct list export
    uint8_t *d_seen_bits = nullptr; size_t cap_seen_bits = 0; // decisions per distinct / per sighting
    uint32_t *d_group_off = nullptr; size_t cap_group_off = 0;
    uint64_t *d_seq = nullptr; size_t cap_seq = 0;
    // pinned host side of the decision round trip: the sightings in stream
    // order (D2H), the per-group sighting bitmap (D2H), the decisions (H2D)
    uint64_t *h_seq = nullptr; size_t cap_h_seq = 0;
    uint64_t *h_gbits = nullptr; size_t cap_h_gbits = 0;
    uint8_t *h_dec = nullptr; size_t cap_h_dec = 0;
    // the batch whose statuses wait for a decision (deferred, or pipelined until retire)
    struct Pending {
        bool live = false;
        uint64_t n = 0;
        const mfp_record *rec = nullptr; const char *fp = nullptr; mfp_analysis *out = nullptr;
        hipStream_t stream = nullptr;
        // the last mfp_analysis_sequence / _distinct result of this batch (the
        // count query and the export that follows it share one device pass)
        long long seq_m = -1;
        std::vector<mfp_sighting> dist;
        long long dist_u = -5;
    } pend;
    uint8_t *d_arena = nullptr; size_t cap_arena = 0;
    mfp_pkt_desc *d_desc = nullptr; size_t cap_desc = 0;
    mfp_record *d_rec = nullptr; size_t cap_rec = 0;
    mfp_tcp_seg *d_seg = nullptr; size_t cap_seg = 0;   // reassembly inputs (when seg_on)
    bool seg_on = false;
    char *d_fp = nullptr; size_t cap_fp = 0;
    char *d_fp2 = nullptr; size_t cap_fp2 = 0;   // dense (compacted) fingerprints of a host batch
    unsigned long long *h_used = nullptr;   // pinned copy of d_used ([4]: k_compact_small's done flag)
    // the small-batch staging copy (mfp_process_small_pinned): counters
    // (zeroed), descriptors and packets in one host-to-device transfer
    uint8_t *d_small = nullptr; size_t cap_small = 0;
    uint8_t *h_small = nullptr; size_t cap_h_small = 0;
    // the direct small batch's device counters (fp_used 4, bins 16, waves
    // done 1), zero between batches: the batch's last wave resets them;
    // cnt_dirty after a batch that may not have finished them
    unsigned long long *d_cnt = nullptr;
    bool cnt_dirty = false;
    hipStream_t stream = nullptr;
    // pipelined device batches (mfp_analyze_batch_device_pipelined): the
    // batch's kernels done (on the caller's stream), the decision applied (on
    // this slot's stream)
    hipEvent_t ev_kernels = nullptr, ev_resolved = nullptr;
    bool resolved_recorded = false;
    // the last device-pointer call that used this slot's scratch on the
    // caller's stream (mfp_process_batch_device, mfp_analyze_batch_device*):
    // a host batch staged on the slot's own stream waits for it
    hipEvent_t ev_dev = nullptr;
    // host pipeline: the chunk's copy in done (on the copy stream), and the
    // slot's chunk done with its packet buffers (on the slot's stream)
    hipEvent_t ev_in = nullptr, ev_free = nullptr;
    bool free_recorded = false;
    bool dev_recorded = false;

    bool init() {
        return hipMalloc(&d_used, 4 * sizeof(unsigned long long)) == hipSuccess &&
               hipMalloc(&d_bins, 16 * sizeof(unsigned long long)) == hipSuccess &&
               hipMalloc(&d_an_stats, MFP_AN_STATS_WORDS * sizeof(unsigned long long)) == hipSuccess &&
               hipMemset(d_an_stats, 0, MFP_AN_STATS_WORDS * sizeof(unsigned long long)) == hipSuccess &&
               hipMalloc(&d_cnt, 24 * sizeof(unsigned long long)) == hipSuccess &&
               hipMemset(d_cnt, 0, 24 * sizeof(unsigned long long)) == hipSuccess &&
               hipHostMalloc((void **)&h_used, 8 * sizeof(unsigned long long), hipHostMallocDefault) == hipSuccess &&
               hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess &&
               hipEventCreateWithFlags(&ev_kernels, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_resolved, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_dev, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_in, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_free, hipEventDisableTiming) == hipSuccess;
    }
    void release() {
        void *p[] = {d_used, d_bins, d_quic, d_work, d_an_stats, d_pending, d_work_items, d_lanel, d_deferred, d_huge, d_segn,
                     d_an, d_ap, d_arena, d_desc, d_rec, d_seg, d_fp, d_fp2, d_small, d_cnt,
                     seen.slots, seen.list, seen.counters, d_sight, d_seen_bits, d_group_off, d_seq};
        for (void *x : p) if (x) (void)hipFree(x);
        for (void *x : {(void *)h_used, (void *)h_seq, (void *)h_gbits, (void *)h_dec, (void *)h_small})
            if (x) (void)hipHostFree(x);
        if (stream) (void)hipStreamDestroy(stream);
        for (hipEvent_t e : {ev_kernels, ev_resolved, ev_dev, ev_in, ev_free}) if (e) (void)hipEventDestroy(e);
    }
};

struct mfp_context_s {
    int device = 0;
    uint32_t select = SEL_ALL, tls_format = 0, mode = 0;
    uint32_t block = 0;                  // BLK_*: selected protocols outside this path (mfp_device.hpp)
    uint32_t quic_format = 0;            // fingerprint_format::quic_fingerprint_format (global_config.h:41)
    uint32_t quic_grid = 512;            // k_quic workgroups (x 128 lanes, each with a scratch slot)
    int strategy = MFP_STRATEGY_BINNED;  // MFP_STRATEGY=binned|lane (A/B, debugging)
    // batches of at most this many packets take MFP_STRATEGY_SMALL (the
    // LDS-staged walker, no classify pass: the per-packet API's latency);
    // MFP_SMALL_BATCH
    size_t small_batch = 256;
    // bin b -> kernel: k_fp_lds (LDS-staged walk) if bit b of bin_lds_mask
    // (MFP_BIN_LDS_MASK), else the HBM lane walker; the bins of bin_seg_mask
    // (MFP_BIN_SEG_MASK; default the two HTTP bins) use segment expansion
    uint32_t bin_seg_mask = 0x4a;        // HTTP request/response and SSH: segment lists + lane emission (r04g)
    uint32_t bin_lds_mask = 0xa0;        // TLS server, DTLS: measured faster from LDS (r02c/d)
    uint32_t an_lane_max_p = ~0u;        // classifier: lane-per-packet scoring up to this P (MFP_AN_LANE_MAX_P, tests)
    mfp_classifier *clf = nullptr;       // --analysis classifier (resources=...;analysis)
    mfp_prevalence own_prev = nullptr;   // the context's fingerprint_prevalence LRU
    mfp_prevalence prev = nullptr;       // the one its sightings are decided against (own or shared)
    bool defer = false;                  // mfp_analysis_defer
    bool report_os = false;              // libmerc_config.report_os (mfp_analysis_report_os)
    bool reassembly = false;             // "reassembly" in the config: mfp_process_batch_reassembly
    Slot slot[4];                        // 0: synchronous calls (and 3: pipelined device batches); 1, 2: host pipeline
    hipStream_t in_stream = nullptr;        // the host pipeline's copy stream
    // the per-packet shim's concurrent small batches (mfp_process_small_pinned):
    // each on a slot of its own, so batches of different callers overlap on the
    // device; taken and returned under mu, waited for outside it
    static constexpr int NSMALL = 8;
    Slot small[NSMALL];
    bool small_init[NSMALL] = {}, small_busy[NSMALL] = {};
    int pipe_next = 0;                   // mfp_analyze_batch_device_pipelined: the slot of the next batch (0 or 3)
    bool pipe_active = false;            // a pipelined batch may be pending in slot 0 or 3
    std::atomic<size_t> attr_names_len{SIZE_MAX};   // mfp_attribute_names_len
    int an_slot = 0;                     // slot of the last classified batch (mfp_analysis_stats)
    mfp_prof *prof = nullptr;            // mfp_profile_enable
    std::mutex mu;
};

#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            mfp_set_error("%s failed: %s", #x, hipGetErrorString(e_));              \
            return -2;                                                              \
        }                                                                           \
    } while (0)

extern "C" MFP_EXPORT mfp_context mfp_init(const char *packet_filter_cfg, int device, int mode) {
    return mfp_init_ex(packet_filter_cfg, device, mode, nullptr);
}

extern "C" MFP_EXPORT mfp_context mfp_init_ex(const char *packet_filter_cfg, int device, int mode,
                                               const uint8_t *enc_key) {
    uint32_t sel, fmt, blk = 0;
    std::string resources;
    bool analysis = false, reassembly = false;
    int report_os = -1;
    if (!mfp_parse_config(packet_filter_cfg, sel, fmt, &resources, &analysis, &reassembly, &blk, nullptr, &report_os))
        return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        mfp_set_error("no HIP device available: the mercury_amd fingerprint path runs only on the GPU");
        return nullptr;
    }
    if (device < 0 || device >= ndev) { mfp_set_error("bad device %d", device); return nullptr; }
    auto *c = new mfp_context_s;
    c->device = device; c->select = sel; c->block = blk; c->tls_format = fmt & 0xff; c->quic_format = (fmt >> 8) & 0xff; c->mode = mode;
    c->reassembly = reassembly;
    c->report_os = report_os == 1;
    const char *st = getenv("MFP_STRATEGY");
    if (st && !strcmp(st, "lane")) c->strategy = MFP_STRATEGY_LANE;
    if (const char *sb = getenv("MFP_SMALL_BATCH")) c->small_batch = (size_t)strtoull(sb, nullptr, 0);
    const char *sm = getenv("MFP_BIN_SEG_MASK");
    if (sm) c->bin_seg_mask = (uint32_t)strtoul(sm, nullptr, 0);
    const char *dm = getenv("MFP_BIN_LDS_MASK");
    if (dm) c->bin_lds_mask = (uint32_t)strtoul(dm, nullptr, 0);
    const char *lm = getenv("MFP_AN_LANE_MAX_P");
    if (lm) c->an_lane_max_p = (uint32_t)strtoul(lm, nullptr, 0);
    bool ok = hipSetDevice(device) == hipSuccess;
    for (Slot &S : c->slot) ok = ok && S.init();
    if (!ok) {
        mfp_set_error("device init failed");
        mfp_finalize(c);
        return nullptr;
    }
    if (analysis && !resources.empty()) {
        // mercury ctor (pkt_proc.h:76-110): load the archive, force the TLS
        // fingerprint format to the database's, keep parsing if the
        // classifier is disabled
        mfp_classifier *clf = mfp_classifier_load(resources.c_str(), enc_key);
        if (!clf) { mfp_finalize(c); return nullptr; }
        // the formats follow the archive even when its classifier is then
        // disabled (missing members, VERSION qualifiers): pkt_proc.h:92-104
        c->tls_format = (uint32_t)mfp_classifier_tls_format(clf);
        c->quic_format = (uint32_t)mfp_classifier_quic_format(clf);
        if (mfp_classifier_disabled(clf)) {
            mfp_classifier_free(clf);
        } else {
            if (mfp_classifier_upload(clf, device) != 0) {
                mfp_classifier_free(clf);
                mfp_finalize(c);
                return nullptr;
            }
            c->clf = clf;
            c->own_prev = c->prev = mfp_prevalence_create(100000);   // analysis.h:433
        }
    }
    return c;
}

extern "C" MFP_EXPORT void mfp_finalize(mfp_context c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->clf) mfp_classifier_free(c->clf);
    if (c->own_prev) mfp_prevalence_destroy(c->own_prev);
    for (Slot &S : c->slot) S.release();
    for (int j = 0; j < mfp_context_s::NSMALL; j++) if (c->small_init[j]) c->small[j].release();
    if (c->in_stream) (void)hipStreamDestroy(c->in_stream);
    delete c->prof;
    delete c;
}

extern "C" MFP_EXPORT size_t mfp_fp_arena_bound(size_t n, size_t total_caplen) {
    // every byte of a captured frame yields at most 4 fingerprint characters
    // (TCP NOP option "(01)"), plus the type prefix; each string owns a
    // 64-byte aligned slot that also holds its 8-byte hash
    return 4 * total_caplen + 176 * n + 4096;
}

int mfp_set_config(mfp_context c, uint32_t select, uint32_t tls_format, uint32_t mode) {
    c->select = select; c->tls_format = tls_format & 0xff; c->quic_format = (tls_format >> 8) & 0xff; c->mode = mode;
    return 0;
}

template <class T>
static int grow(T *&p, size_t &cap, size_t need) {
    if (need <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    size_t nc = std::max(need, cap * 2);
    if (hipMalloc(&p, nc * sizeof(T)) != hipSuccess) { cap = 0; return -1; }
    cap = nc;
    return 0;
}

template <class T>
static int grow_pinned(T *&p, size_t &cap, size_t need) {
    if (need <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    size_t nc = std::max(need, cap + cap / 2);
    if (hipHostMalloc((void **)&p, nc * sizeof(T), hipHostMallocDefault) != hipSuccess) { cap = 0; return -1; }
    cap = nc;
    return 0;
}

extern "C" MFP_EXPORT int mfp_reserve(mfp_context c, size_t n) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (grow(c->slot[0].d_work, c->slot[0].cap_work, 11 * n + 2)) { mfp_set_error("device allocation failed"); return -2; }
    return 0;
}

// d_bins: the classify pass's bin counts, already zeroed together with
// d_fp_used (the small-batch staging copy); nullptr: the slot's, cleared here
static int process_device_locked(mfp_context c, Slot &S, const uint8_t *d_arena, const mfp_pkt_desc *d_desc, size_t n,
                                 mfp_record *d_rec, char *d_fp_arena, size_t fp_cap, uint64_t *d_fp_used,
                                 hipStream_t s, unsigned long long *d_bins = nullptr, unsigned long long *fin = nullptr,
                                 unsigned long long *host_out = nullptr) {
    HIPCHK(hipSetDevice(c->device));
    if (grow(S.d_work, S.cap_work, 11 * n + 2)) { mfp_set_error("device allocation failed"); return -2; }
    if ((c->select & (SEL_QUIC | SEL_OPENVPN)) && !S.d_quic &&
        hipMalloc(&S.d_quic, mfp_quic_scratch_bytes(c->quic_grid)) != hipSuccess) {
        S.d_quic = nullptr;
        mfp_set_error("device allocation failed (QUIC scratch)");
        return -2;
    }
    if (!d_bins) {
        HIPCHK(hipMemsetAsync(d_fp_used, 0, 4 * sizeof(unsigned long long), s));
        HIPCHK(hipMemsetAsync(S.d_bins, 0, 16 * sizeof(unsigned long long), s));
        d_bins = S.d_bins;
    }
    mfp_tcp_seg *d_seg = nullptr;
    if (S.seg_on) {
        if (grow(S.d_seg, S.cap_seg, n + 1)) { mfp_set_error("device allocation failed"); return -2; }
        d_seg = S.d_seg;
    }
    if (mfp_launch_fingerprint(c->select, c->block, c->tls_format, c->mode, d_arena, d_desc, n, d_rec, d_seg, (uint8_t *)d_fp_arena,
                               fp_cap, (unsigned long long *)d_fp_used, S.d_work, d_bins,
                               c->strategy == MFP_STRATEGY_BINNED && n <= c->small_batch ? (int)MFP_STRATEGY_SMALL
                                                                                         : c->strategy,
                               c->bin_seg_mask, c->bin_lds_mask, c->quic_format, S.d_quic, c->quic_grid, s,
                               c->prof, fin, host_out) != 0) {
        mfp_set_error("kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -3;
    }
    return 0;
}

// the slot's sighting table, sized for a batch of n packets (reset per batch)
static int seen_reserve(Slot &S, size_t n, hipStream_t s) {
    uint64_t want = 4096;
    const uint64_t target = 2 * std::min<uint64_t>(n, (uint64_t)1 << 21);
    while (want < target) want <<= 1;
    if (S.seen.slots == nullptr || S.seen.mask + 1 < want) {
        if (S.seen.slots) (void)hipFree(S.seen.slots);
        if (S.seen.list) (void)hipFree(S.seen.list);
        if (S.d_sight) (void)hipFree(S.d_sight);
        S.seen.slots = nullptr; S.seen.list = nullptr; S.d_sight = nullptr;
        if (hipMalloc(&S.seen.slots, want * sizeof(mfp_seen_slot)) != hipSuccess ||
            hipMalloc(&S.seen.list, want / 2 * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&S.d_sight, want / 2 * sizeof(mfp_sighting)) != hipSuccess)
            return -2;
        S.seen.mask = (uint32_t)(want - 1);
        S.seen.list_cap = (uint32_t)(want / 2);
    }
    if (!S.seen.counters && hipMalloc(&S.seen.counters, 4 * sizeof(unsigned int)) != hipSuccess) return -2;
    if (hipMemsetAsync(S.seen.slots, 0xff, (S.seen.mask + 1ull) * sizeof(mfp_seen_slot), s) != hipSuccess ||
        hipMemsetAsync(S.seen.counters, 0, 4 * sizeof(unsigned int), s) != hipSuccess)
        return -2;
    return 0;
}

// d_stats: the batch's counters, already zeroed (the small-batch staging
// copy), and no sighting table -- the batch is decided on the host from its
// records (resolve_on_host); nullptr: the slot's counters and table
static int analyze_slot(mfp_context c, Slot &S, const uint8_t *d_arena, const mfp_pkt_desc *d_desc, size_t n,
                        mfp_record *d_rec, const char *d_fp_arena, mfp_analysis *d_out, double *d_attr_prob,
                        hipStream_t s, unsigned long long *d_stats) {
    HIPCHK(hipSetDevice(c->device));
    uint32_t nseg = 0, seg_cap = 0;
    mfp_analysis_segments(n, &nseg, &seg_cap);
    const size_t items = (size_t)nseg * seg_cap + 1;
    if (grow(S.d_pending, S.cap_pending, n + 1) || grow(S.d_work_items, S.cap_work_items, items) ||
        grow(S.d_lanel, S.cap_lanel, 4 * items) || grow(S.d_deferred, S.cap_deferred, 5 * items) ||
        grow(S.d_segn, S.cap_segn, 3 * (size_t)nseg + 1) || (!d_stats && seen_reserve(S, n, s))) {
        mfp_set_error("device allocation failed");
        return -2;
    }
    mfp_classifier_dev *D = mfp_classifier_device_mut(c->clf);
    const size_t huge = mfp_analysis_huge_bytes(D->max_nproc);
    if (huge && grow(S.d_huge, S.cap_huge, (huge + 15) / 16)) {
        mfp_set_error("device allocation failed");
        return -2;
    }
    if (!d_stats) HIPCHK(hipMemsetAsync(S.d_an_stats, 0, MFP_AN_STATS_WORDS * sizeof(unsigned long long), s));
    if (mfp_launch_analysis(D, d_stats ? nullptr : &S.seen, d_arena, d_desc, n, d_rec, (const uint8_t *)d_fp_arena, d_out,
                            d_attr_prob, S.d_pending, S.d_work_items, S.d_lanel, S.d_deferred, S.d_segn,
                            d_stats ? d_stats : S.d_an_stats, c->mode,
                            c->an_lane_max_p, S.d_huge, s, c->prof) != 0) {
        mfp_set_error("analysis kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -3;
    }
    return 0;
}
static int analyze_locked(mfp_context c, int slot, const uint8_t *d_arena, const mfp_pkt_desc *d_desc, size_t n,
                          mfp_record *d_rec, const char *d_fp_arena, mfp_analysis *d_out, double *d_attr_prob,
                          hipStream_t s) {
    Slot &S = c->slot[slot];
    const int r = analyze_slot(c, S, d_arena, d_desc, n, d_rec, d_fp_arena, d_out, d_attr_prob, s, nullptr);
    if (r) return r;
    c->an_slot = slot;
    S.pend.live = true;
    S.pend.seq_m = -1;
    S.pend.dist_u = -5;
    S.pend.n = n; S.pend.rec = d_rec; S.pend.fp = d_fp_arena; S.pend.out = d_out; S.pend.stream = s;
    return 0;
}

// ---- deciding a batch's unknown-TLS sightings (mfp_prevalence) ----
// the distinct list of the slot's pending batch; -3 when its table overflowed
// `bound`: return -4 without exporting when the batch has more distinct
// fingerprints than the bound (the LRU's capacity: the distinct form cannot
// be exact then, mfp_prevalence_resolve_distinct)
static long long slot_distinct(mfp_context c, Slot &S, std::vector<mfp_sighting> &d, uint64_t bound = ~0ull) {
    hipStream_t s = S.pend.stream;
    unsigned int cnt[4];
    HIPCHK(hipMemcpyAsync(cnt, S.seen.counters, sizeof cnt, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (cnt[1] || cnt[0] > S.seen.list_cap) return -3;
    if (cnt[0] > bound) return -4;
    d.resize(cnt[0]);
    if (cnt[0]) {
        if (mfp_launch_seen_export(&S.seen, cnt[0], S.d_sight, s) != 0) { mfp_set_error("export launch failed"); return -3; }
        HIPCHK(hipMemcpyAsync(d.data(), S.d_sight, cnt[0] * sizeof(mfp_sighting), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    (void)c;
    return (long long)cnt[0];
}

// the slot's pending sightings in stream order (hashes), and the per-group
// offsets the resolve kernel indexes them with (left in S.d_group_off)
// (S.h_seq, pinned: valid until the slot's next sequence)
static long long slot_sequence(mfp_context c, Slot &S) {
    hipStream_t s = S.pend.stream;
    const uint64_t groups = (S.pend.n + 63) / 64;
    if (grow_pinned(S.h_gbits, S.cap_h_gbits, groups + 1)) { mfp_set_error("host allocation failed"); return -2; }
    if (groups) HIPCHK(hipMemcpyAsync(S.h_gbits, S.d_pending, groups * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<uint32_t> off(groups + 1, 0);
    for (uint64_t g = 0; g < groups; g++) off[g + 1] = off[g] + (uint32_t)__builtin_popcountll(S.h_gbits[g]);
    const uint64_t m = off[groups];
    if (grow(S.d_group_off, S.cap_group_off, groups + 1) || grow(S.d_seq, S.cap_seq, m + 1)) {
        mfp_set_error("device allocation failed");
        return -2;
    }
    if (grow_pinned(S.h_seq, S.cap_h_seq, m + 1)) { mfp_set_error("host allocation failed"); return -2; }
    if (groups) HIPCHK(hipMemcpyAsync(S.d_group_off, off.data(), (groups + 1) * 4, hipMemcpyHostToDevice, s));
    if (mfp_launch_seen_sequence(mfp_classifier_device(c->clf), &S.seen, S.pend.n, S.pend.rec,
                                 (const uint8_t *)S.pend.fp, S.d_pending, S.d_group_off, S.d_seq, s) != 0) {
        mfp_set_error("sequence launch failed");
        return -3;
    }
    if (m) HIPCHK(hipMemcpyAsync(S.h_seq, S.d_seq, m * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return (long long)m;
}

// apply decisions to the slot's pending batch: per distinct entry (pos order)
// or per sighting (seq), on the device records
// (bits may be S.h_dec, pinned, or any host memory: staged through S.h_dec)
static int slot_apply(mfp_context c, Slot &S, const uint8_t *bits, size_t nbits, bool per_sighting) {
    hipStream_t s = S.pend.stream;
    if (grow(S.d_seen_bits, S.cap_seen_bits, nbits + 1)) { mfp_set_error("device allocation failed"); return -2; }
    if (bits != S.h_dec) {
        if (grow_pinned(S.h_dec, S.cap_h_dec, nbits + 1)) { mfp_set_error("host allocation failed"); return -2; }
        if (nbits) memcpy(S.h_dec, bits, nbits);
    }
    if (nbits) HIPCHK(hipMemcpyAsync(S.d_seen_bits, S.h_dec, nbits, hipMemcpyHostToDevice, s));
    if (mfp_launch_analysis_resolve(mfp_classifier_device(c->clf), &S.seen, S.pend.n, S.pend.rec,
                                    (const uint8_t *)S.pend.fp, S.pend.out, S.d_pending, c->mode,
                                    per_sighting ? nullptr : S.d_seen_bits, S.d_group_off,
                                    per_sighting ? S.d_seen_bits : nullptr, s, c->prof) != 0) {
        mfp_set_error("resolve launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -3;
    }
    HIPCHK(hipEventRecord(S.ev_resolved, s));   // (a pipelined slot's next batch waits for it)
    S.resolved_recorded = true;
    S.pend.live = false;
    return 0;
}

// decide the slot's pending batch against c->prev and apply: the distinct
// form when it is exact, else the sighting sequence
static int slot_resolve(mfp_context c, Slot &S) {
    if (!S.pend.live) return 0;
    std::vector<mfp_sighting> d;
    const long long u = slot_distinct(c, S, d, mfp_prevalence_capacity(c->prev));
    if (u == -2) return -2;
    if (u >= 0) {
        // the device's distinct list is in insertion order: positions are
        // what k_seen_export stored in the slots (index = pos)
        const int r = mfp_prevalence_resolve_distinct(c->prev, d.data(), d.size());
        if (r == 0) {
            std::vector<uint8_t> bits(d.size());
            for (size_t i = 0; i < d.size(); i++) bits[i] = (uint8_t)d[i].first_seen;
            return slot_apply(c, S, bits.data(), bits.size(), false);
        }
        if (r != -2) return r;
    }
    const long long m = slot_sequence(c, S);
    if (m < 0) return (int)m;
    if (grow_pinned(S.h_dec, S.cap_h_dec, (size_t)m + 1)) { mfp_set_error("host allocation failed"); return -2; }
    if (mfp_prevalence_resolve_sequence(c->prev, S.h_seq, (size_t)m, S.h_dec) != 0) return -1;
    return slot_apply(c, S, S.h_dec, (size_t)m, true);
}

// Decide the pipelined device batches still pending (slots 0 and 3, the
// older first) before any other analysis call takes slot 0 or the LRU: a
// synchronous batch between pipelined ones must neither overwrite slot 0's
// undecided batch nor decide its own sightings ahead of earlier ones (the LRU
// follows stream order, analysis.h:362-421).
static int flush_pipelined_locked(mfp_context c) {
    if (!c->pipe_active) return 0;
    for (int k = 0; k < 2; k++) {
        Slot &S = c->slot[(k == 0) == (c->pipe_next == 0) ? 0 : 3];
        if (!S.pend.live) continue;
        const int r = slot_resolve(c, S);
        if (r) return r;
        HIPCHK(hipEventRecord(S.ev_resolved, S.stream));
        S.resolved_recorded = true;
        // the decision's kernels finish before the caller's next work reuses
        // the slot's tables (on whichever stream) or reads the records
        HIPCHK(hipStreamSynchronize(S.stream));
    }
    c->pipe_active = false;
    return 0;
}

extern "C" MFP_EXPORT int mfp_process_batch_device(mfp_context c, const uint8_t *d_arena, const mfp_pkt_desc *d_desc,
                                                   size_t n, mfp_record *d_rec, char *d_fp_arena, size_t fp_cap,
                                                   uint64_t *d_fp_used, void *stream) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot &S = c->slot[0];
    const int r = process_device_locked(c, S, d_arena, d_desc, n, d_rec, d_fp_arena, fp_cap, d_fp_used,
                                        (hipStream_t)stream);
    if (r) return r;
    HIPCHK(hipEventRecord(S.ev_dev, (hipStream_t)stream));
    S.dev_recorded = true;
    return 0;
}

// decide the slot's pending batch against c->prev and patch the host copies
// of its records (the pipeline retires chunks in order, after their D2H)
static void host_patch(mfp_context c, mfp_analysis &a, const mfp_record &r, bool seen) {
    a.flags &= (uint8_t)~MFP_AN_PENDING;
    if (seen) {   // as k_analyze_resolve: unlabeled keeps encrypted_dns / domain_faking only
        const mfp_classifier_dev *D = mfp_classifier_device(c->clf);
        a.status = 3;
        a.score = 0.0; a.malware_prob = -1.0; a.process = MFP_NO_PROCESS; a.proc_slot = MFP_NO_PROCESS;
        a.attr &= (uint16_t)((1u << D->doh_idx) | (1u << D->domain_faking_idx));
        a.flags = MFP_AN_VALID;
    }
    if (c->mode == MFP_MODE_ANALYSIS && (r.flags & MFP_FLAG_TRUNCATED)) a.status = 3;   // pkt_proc.cc:1716-1719
}
static int slot_resolve_host(mfp_context c, Slot &S, mfp_analysis *an, const mfp_record *rec) {
    if (!S.pend.live) return 0;
    S.pend.live = false;
    const size_t m = S.pend.n;
    std::vector<mfp_sighting> d;
    const long long u = slot_distinct(c, S, d, mfp_prevalence_capacity(c->prev));
    if (u == -2) return -2;
    if (u >= 0) {
        const int r = mfp_prevalence_resolve_distinct(c->prev, d.data(), d.size());
        if (r == 0) {
            std::vector<uint8_t> randomized(m, 0);
            for (const auto &x : d) if (!x.first_seen && x.first < m) randomized[x.first] = 1;
            for (size_t i = 0; i < m; i++)
                if (an[i].flags & MFP_AN_PENDING) host_patch(c, an[i], rec[i], !randomized[i]);
            return 0;
        }
        if (r != -2) return r;
    }
    const long long ms = slot_sequence(c, S);
    if (ms < 0) return (int)ms;
    if (grow_pinned(S.h_dec, S.cap_h_dec, (size_t)ms + 1)) { mfp_set_error("host allocation failed"); return -2; }
    const uint8_t *seen = S.h_dec;
    if (mfp_prevalence_resolve_sequence(c->prev, S.h_seq, (size_t)ms, S.h_dec) != 0) return -1;
    size_t k = 0;
    for (size_t i = 0; i < m && k < (size_t)ms; i++)
        if (an[i].flags & MFP_AN_PENDING) host_patch(c, an[i], rec[i], seen[k++] != 0);
    return 0;
}

// the bytes a host batch's descriptors span: [lo, hi) (lo 256-byte aligned)
// and the packet bytes in it (a QUIC packet's reassembled CRYPTO data included)
static int batch_span(const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc, size_t n, uint64_t &lo,
                      uint64_t &hi, uint64_t &total) {
    lo = UINT64_MAX; hi = 0; total = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t end = desc[i].offset + desc[i].caplen;
        if (desc[i].flags & MFP_DESC_QUIC_CRYPTO) {
            // the reassembled CRYPTO data behind the packet travels with it
            const uint64_t at = desc[i].offset + ((desc[i].caplen + 7) & ~7ull);
            if (at + 8 > arena_len) { mfp_set_error("reassembled QUIC data past the end of the arena"); return -1; }
            const uint32_t L = (uint32_t)arena[at] | (uint32_t)arena[at + 1] << 8 | (uint32_t)arena[at + 2] << 16 |
                               (uint32_t)arena[at + 3] << 24;
            if (L > 8192) { mfp_set_error("reassembled QUIC data longer than the 8192-byte buffer"); return -1; }
            end = at + 8 + L;
            total += 8 + L;
        }
        lo = std::min<uint64_t>(lo, desc[i].offset);
        hi = std::max<uint64_t>(hi, end);
        total += desc[i].caplen;
    }
    if (n == 0) lo = hi = 0;   // (a capture ring hands packets in arena order; this scan is a few ms per 1M)
    lo &= ~(uint64_t)255;
    if (hi > arena_len) { mfp_set_error("descriptor past the end of the arena"); return -1; }
    return 0;
}

// copy a host batch into slot `slot` (grown as needed) and launch its kernels
// on the slot's stream; descriptors keep their offsets: the device arena
// pointer handed to the kernels is the staging buffer minus the (256-byte
// aligned) start of the copied span
static int stage_and_launch(mfp_context c, int slot, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                            size_t n, size_t fp_cap, bool analysis, bool attr_prob, bool host_resolve = false,
                            const uint64_t *staged = nullptr) {
    Slot &S = c->slot[slot];
    // device-pointer calls may still be using this slot's scratch on the caller's stream
    if (S.dev_recorded) { HIPCHK(hipStreamWaitEvent(S.stream, S.ev_dev, 0)); S.dev_recorded = false; }
    uint64_t lo, hi, total;
    if (staged) {   // (stage_copy ran: {lo, hi, total}, the copies queued behind ev_in)
        lo = staged[0]; hi = staged[1]; total = staged[2];
    } else if (batch_span(arena, arena_len, desc, n, lo, hi, total)) {
        return -1;
    }
    // the device arena holds the strings at their reserved slots (the TLS
    // ClientHello bin reserves by an upper bound, k_fp_tls1): sized by the
    // bound, whatever the caller's dense capacity; the callers check that the
    // packed strings fit theirs
    const size_t dcap = std::max(fp_cap, mfp_fp_arena_bound(n, total));
    const uint64_t span = hi - lo;
    // 64 bytes of padding after the span: the kernels read the aligned block
    // that holds a packet's last byte
    if ((!staged && (grow(S.d_arena, S.cap_arena, span + 64) || grow(S.d_desc, S.cap_desc, n + 1))) ||
        grow(S.d_rec, S.cap_rec, n + 1) ||
        grow(S.d_fp, S.cap_fp, dcap + 64) || grow(S.d_fp2, S.cap_fp2, dcap + 64) ||
        (analysis && grow(S.d_an, S.cap_an, n + 1)) ||
        (analysis && attr_prob && grow(S.d_ap, S.cap_ap, MFP_ATTR_DB_TAGS * (n + 1)))) {
        mfp_set_error("device allocation failed");
        return -2;
    }
    if (staged) {
        HIPCHK(hipStreamWaitEvent(S.stream, S.ev_in, 0));
    } else {
        const uint64_t copy = std::min<uint64_t>(span + 16, arena_len - lo);
        if (copy) HIPCHK(hipMemcpyAsync(S.d_arena, arena + lo, copy, hipMemcpyHostToDevice, S.stream));
        if (n) HIPCHK(hipMemcpyAsync(S.d_desc, desc, n * sizeof(mfp_pkt_desc), hipMemcpyHostToDevice, S.stream));
    }
    const uint8_t *d_base = S.d_arena - lo;
    int r = process_device_locked(c, S, d_base, S.d_desc, n, S.d_rec, S.d_fp, dcap, (uint64_t *)S.d_used, S.stream);
    if (r) return r;
    if (analysis) {
        r = analyze_locked(c, slot, d_base, S.d_desc, n, S.d_rec, S.d_fp, S.d_an, attr_prob ? S.d_ap : nullptr, S.stream);
        if (r) return r;
        // the synchronous host batch decides its unknown-TLS sightings now;
        // pipeline slots when they retire (chunk order), on the host copies
        if (slot == 0 && !c->defer && !host_resolve) { r = slot_resolve(c, S); if (r) return r; }
    }
    if (staged) {   // the packets and descriptors are read by now: the copy of the slot's next chunk may start
        HIPCHK(hipEventRecord(S.ev_free, S.stream));
        S.free_recorded = true;
    }
    // strings to a dense arena in packet order (d_fp2, d_used[2] bytes), records re-pointed;
    // the bin lists in d_work are dead by now and hold the scan scratch
    // (the packed total, strings and QUIC sidecars, replaces d_used[2])
    if (n && mfp_launch_compact(S.d_rec, n, (const uint8_t *)S.d_fp, (uint8_t *)S.d_fp2, S.d_work,
                                (unsigned long long *)(S.d_work + ((n + 3) & ~(size_t)1)), S.d_used + 2, S.stream,
                                c->prof) != 0) {
        mfp_set_error("compaction launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -3;
    }
    // the records now point into the dense arena (a fingerprint-only batch in
    // slot 0 leaves a pipelined batch pending there untouched)
    if (analysis) S.pend.fp = S.d_fp2;
    return 0;
}

// A small synchronous batch (the per-packet API) decides its unknown-TLS
// sightings on the host from the copies it returns -- the string hashes of the
// pending records, in packet order, against the LRU -- instead of the device
// round trips of slot_resolve (the same decisions: both are the sequence form)
static int resolve_on_host(mfp_context c, Slot &S, mfp_analysis *an, const mfp_record *rec, const char *fp, size_t n) {
    S.pend.live = false;
    std::vector<uint64_t> keys;
    std::vector<size_t> idx;
    for (size_t i = 0; i < n; i++)
        if (an[i].flags & MFP_AN_PENDING) {
            keys.push_back(mfpc::str_hash((const uint8_t *)fp + rec[i].fp_offset, rec[i].fp_len));
            idx.push_back(i);
        }
    if (keys.empty()) return 0;
    std::vector<uint8_t> seen(keys.size());
    if (mfp_prevalence_resolve_sequence(c->prev, keys.data(), keys.size(), seen.data()) != 0) return -1;
    for (size_t k = 0; k < keys.size(); k++) host_patch(c, an[idx[k]], rec[idx[k]], seen[k] != 0);
    return 0;
}

extern "C" MFP_EXPORT long long mfp_process_batch_host_ex(mfp_context c, const uint8_t *arena, size_t arena_len,
                                                          const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                                          char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                                          double *attr_prob) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (analysis && !c->clf) { mfp_set_error("analysis is not enabled (config needs resources=<archive>;analysis)"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (fp_cap < mfp_fp_arena_bound(0, 0)) { mfp_set_error("fp_cap below mfp_fp_arena_bound"); return -1; }
    Slot &S = c->slot[0];
    if (analysis) { const int fr = flush_pipelined_locked(c); if (fr) return fr; }
    const bool host_resolve = analysis && n <= c->small_batch && !c->defer;
    int r = stage_and_launch(c, 0, arena, arena_len, desc, n, fp_cap, analysis != nullptr, attr_prob != nullptr,
                             host_resolve);
    if (r) return r;
    if (analysis && n) HIPCHK(hipMemcpyAsync(analysis, S.d_an, n * sizeof(mfp_analysis), hipMemcpyDeviceToHost, S.stream));
    if (analysis && attr_prob && n)
        HIPCHK(hipMemcpyAsync(attr_prob, S.d_ap, n * MFP_ATTR_DB_TAGS * sizeof(double), hipMemcpyDeviceToHost, S.stream));
    if (n) HIPCHK(hipMemcpyAsync(rec, S.d_rec, n * sizeof(mfp_record), hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipMemcpyAsync(S.h_used, S.d_used, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, S.stream));
    // small batches (the per-packet API): the packed strings' likely extent
    // comes back with the records, one round trip instead of two
    const size_t spec = n <= c->small_batch ? std::min<size_t>(fp_cap, (size_t)256 << 10) : 0;
    if (spec) HIPCHK(hipMemcpyAsync(fp_arena, S.d_fp2, spec, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    const unsigned long long used = S.h_used[2];   // dense bytes
    if (S.h_used[1] || used > fp_cap) { mfp_set_error("fingerprint arena overflow (cap %zu)", fp_cap); return -4; }
    if (used > spec) HIPCHK(hipMemcpy(fp_arena + spec, S.d_fp2 + spec, used - spec, hipMemcpyDeviceToHost));
    if (host_resolve) {
        const int rr = resolve_on_host(c, S, analysis, rec, fp_arena, n);
        if (rr) return rr;
    }
    return (long long)used;
}

// A small batch is done when its last kernel's flag (S.h_used[4]) lands in
// host memory, its writes before it: no wake-up through the runtime; a batch
// not done within 2 ms waits on the stream, which also reports a failed launch
static int wait_done_flag(Slot &S) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; spin++) {
        if (__atomic_load_n(&S.h_used[4], __ATOMIC_ACQUIRE) != 0) return 0;
        if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    HIPCHK(hipStreamSynchronize(S.stream));
    return 0;
}

// The per-packet shim's batch (mfp_libmerc.cpp run_batch): every buffer is
// page-locked host memory (hipHostMalloc), so the batch is one transfer in --
// counters (zeroed by the copy itself), descriptors and packets staged
// together -- the walker, the classifier when asked, and one kernel that writes
// the packed strings, the records and the results straight into the caller's
// buffers: one host-to-device copy, no memsets, no copies back, one wait.
// Same results as mfp_process_batch_host_ex, which it defers to for anything
// else (larger batches, deferred decisions, reassembly contexts).
long long mfp_process_small_pinned(mfp_context c, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                                   size_t n, mfp_record *rec, char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                   double *attr_prob) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (n == 0 || n > c->small_batch || n > 1024 || c->defer || (analysis && !c->clf))
        return mfp_process_batch_host_ex(c, arena, arena_len, desc, n, rec, fp_arena, fp_cap, analysis, attr_prob);
    if (fp_cap < mfp_fp_arena_bound(0, 0)) { mfp_set_error("fp_cap below mfp_fp_arena_bound"); return -1; }
    uint64_t lo, hi, total;
    if (batch_span(arena, arena_len, desc, n, lo, hi, total)) return -1;
    int k = -1;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        HIPCHK(hipSetDevice(c->device));
        if (analysis) { const int fr = flush_pipelined_locked(c); if (fr) return fr; }
        for (int j = 0; j < mfp_context_s::NSMALL && k < 0; j++) {
            if (c->small_busy[j]) continue;
            if (!c->small_init[j]) {
                if (!c->small[j].init()) {
                    c->small[j].release();        // what init() allocated before it failed
                    c->small[j] = Slot{};
                    mfp_set_error("small-batch slot: HIP allocation failed");
                    return -2;
                }
                c->small_init[j] = true;
            }
            c->small_busy[j] = true;
            k = j;
        }
    }
    // every slot taken (more concurrent callers than NSMALL): the copying path
    if (k < 0) return mfp_process_batch_host_ex(c, arena, arena_len, desc, n, rec, fp_arena, fp_cap, analysis, attr_prob);
    struct Give {   // the slot goes back on every exit (its next batch is ordered behind this one on its stream)
        mfp_context c; int k;
        ~Give() {
            std::lock_guard<std::mutex> lk(c->mu);
            c->small_busy[k] = false;
        }
    } give{c, k};
    Slot &S = c->small[k];
    // Fingerprints only (no classifier, no k_quic): the walker reads the
    // caller's page-locked packets in place and writes records and strings
    // straight into the caller's buffers -- one launch, no copies at all
    // (strings at their reserved, not packed, offsets; at least 64 bytes
    // after the last packet, which the walker may read)
    // Only the SMALL strategy's last wave copies the counters out, resets them
    // and sets the done flag (process_device_locked picks it for binned
    // contexts at n <= small_batch); any other strategy takes the staged path,
    // whose k_compact_small does that work
    const bool direct = !analysis && !(c->select & (SEL_QUIC | SEL_OPENVPN)) && hi + 64 <= arena_len &&
                        c->strategy == MFP_STRATEGY_BINNED && fp_cap >= mfp_fp_arena_bound(n, total);
    if (direct) {
        {
            std::lock_guard<std::mutex> lk(c->mu);
            HIPCHK(hipSetDevice(c->device));
            if (S.cnt_dirty) HIPCHK(hipMemsetAsync(S.d_cnt, 0, 24 * sizeof(unsigned long long), S.stream));
            S.cnt_dirty = true;   // until the batch's last wave has reset them
            __atomic_store_n(&S.h_used[4], 0ull, __ATOMIC_RELAXED);
            const int r = process_device_locked(c, S, arena, desc, n, rec, fp_arena, fp_cap, (uint64_t *)S.d_cnt, S.stream,
                                                S.d_cnt + 4, S.d_cnt + 20, S.h_used);
            if (r) return r;
        }
        if (wait_done_flag(S)) return -2;
        if (__atomic_load_n(&S.h_used[4], __ATOMIC_ACQUIRE) == 0) {
            // the stream drained without the walker's done flag: the counters
            // were neither copied out nor reset (cnt_dirty stays set, so the
            // next batch clears them)
            mfp_set_error("small batch finished without its done flag");
            return -3;
        }
        S.cnt_dirty = false;
        const unsigned long long used = S.h_used[0];   // reserved bytes: strings at their slots
        if (S.h_used[1] || used > fp_cap) { mfp_set_error("fingerprint arena overflow (cap %zu)", fp_cap); return -4; }
        return (long long)used;
    }
    const size_t dcap = std::max(fp_cap, mfp_fp_arena_bound(n, total));
    // staging layout: [fp counters 4 | bin counts 16 | classifier counters] [descriptors] [packets + 64]
    constexpr size_t W = 8;
    const size_t n_cnt = 4 + 16 + MFP_AN_STATS_WORDS;
    const size_t at_desc = (n_cnt * W + 255) & ~(size_t)255;
    const size_t at_pkt = (at_desc + n * sizeof(mfp_pkt_desc) + 255) & ~(size_t)255;
    const uint64_t copy = std::min<uint64_t>(hi - lo + 16, arena_len - lo);
    const size_t bytes = at_pkt + copy;
    {
        // launches under mu: the classifier tables and the context's
        // configuration are shared with the other slots' calls
        std::lock_guard<std::mutex> lk(c->mu);
        HIPCHK(hipSetDevice(c->device));
        if (grow(S.d_small, S.cap_small, bytes + 64) || grow(S.d_rec, S.cap_rec, n + 1) ||
            grow(S.d_fp, S.cap_fp, dcap + 64) || (analysis && grow(S.d_an, S.cap_an, n + 1)) ||
            (analysis && attr_prob && grow(S.d_ap, S.cap_ap, MFP_ATTR_DB_TAGS * (n + 1)))) {
            mfp_set_error("device allocation failed");
            return -2;
        }
        if (grow_pinned(S.h_small, S.cap_h_small, bytes + 64)) { mfp_set_error("host allocation failed"); return -2; }
        memset(S.h_small, 0, at_desc);
        __atomic_store_n(&S.h_used[4], 0ull, __ATOMIC_RELAXED);   // set by k_compact_small when all is written
        memcpy(S.h_small + at_desc, desc, n * sizeof(mfp_pkt_desc));
        memcpy(S.h_small + at_pkt, arena + lo, copy);
        HIPCHK(hipMemcpyAsync(S.d_small, S.h_small, bytes, hipMemcpyHostToDevice, S.stream));
        auto *d_used = (unsigned long long *)S.d_small;
        const mfp_pkt_desc *d_desc = (const mfp_pkt_desc *)(S.d_small + at_desc);
        const uint8_t *d_base = S.d_small + at_pkt - lo;
        int r = process_device_locked(c, S, d_base, d_desc, n, S.d_rec, S.d_fp, dcap, (uint64_t *)d_used, S.stream,
                                      d_used + 4);
        if (r) return r;
        if (analysis) {
            r = analyze_slot(c, S, d_base, d_desc, n, S.d_rec, S.d_fp, S.d_an, attr_prob ? S.d_ap : nullptr, S.stream,
                             d_used + 20);
            if (r) return r;
        }
        if (mfp_launch_compact_small(S.d_rec, n, (const uint8_t *)S.d_fp, (uint8_t *)fp_arena, fp_cap, rec, d_used,
                                     S.h_used, analysis ? S.d_an : nullptr, analysis,
                                     analysis && attr_prob ? S.d_ap : nullptr, attr_prob, S.stream, c->prof) != 0) {
            mfp_set_error("compaction launch failed: %s", hipGetErrorString(hipGetLastError()));
            return -3;
        }
    }
    if (wait_done_flag(S)) return -2;
    const unsigned long long used = S.h_used[2];
    if (S.h_used[1] || used > fp_cap) { mfp_set_error("fingerprint arena overflow (cap %zu)", fp_cap); return -4; }
    // decided on the host from the records (the prevalence LRU has its own
    // lock; concurrent callers' batches are decided in the order they finish)
    if (analysis) {
        const int rr = resolve_on_host(c, S, analysis, rec, fp_arena, n);
        if (rr) return rr;
    }
    return (long long)used;
}

extern "C" MFP_EXPORT long long mfp_process_batch_host_seg(mfp_context c, const uint8_t *arena, size_t arena_len,
                                                           const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                                           char *fp_arena, size_t fp_cap, mfp_tcp_seg *seg) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (!seg && n) { mfp_set_error("null segment array"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (fp_cap < mfp_fp_arena_bound(0, 0)) { mfp_set_error("fp_cap below mfp_fp_arena_bound"); return -1; }
    Slot &S = c->slot[0];
    S.seg_on = true;
    int r = stage_and_launch(c, 0, arena, arena_len, desc, n, fp_cap, false, false);
    S.seg_on = false;
    if (r) return r;
    if (n) HIPCHK(hipMemcpyAsync(rec, S.d_rec, n * sizeof(mfp_record), hipMemcpyDeviceToHost, S.stream));
    if (n) HIPCHK(hipMemcpyAsync(seg, S.d_seg, n * sizeof(mfp_tcp_seg), hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipMemcpyAsync(S.h_used, S.d_used, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    const unsigned long long used = S.h_used[2];
    if (S.h_used[1] || used > fp_cap) { mfp_set_error("fingerprint arena overflow (cap %zu)", fp_cap); return -4; }
    if (used) HIPCHK(hipMemcpy(fp_arena, S.d_fp2, used, hipMemcpyDeviceToHost));
    return (long long)used;
}

extern "C" MFP_EXPORT int mfp_reassembly_enabled(mfp_context c) { return c && c->reassembly ? 1 : 0; }
uint32_t mfp_context_mode(mfp_context c) { return c ? c->mode : 0; }

extern "C" MFP_EXPORT long long mfp_process_batch_host(mfp_context c, const uint8_t *arena, size_t arena_len,
                                                       const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                                       char *fp_arena, size_t fp_cap) {
    return mfp_process_batch_host_ex(c, arena, arena_len, desc, n, rec, fp_arena, fp_cap, nullptr, nullptr);
}

static long long pipelined_locked(mfp_context c, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                                  size_t n, mfp_record *rec, char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                  double *attr_prob, size_t chunk);

extern "C" MFP_EXPORT long long mfp_process_pipelined(mfp_context c, const uint8_t *arena, size_t arena_len,
                                                      const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                                      char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                                      double *attr_prob, size_t chunk) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (analysis && !c->clf) { mfp_set_error("analysis is not enabled (config needs resources=<archive>;analysis)"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) { mfp_set_error("hipSetDevice failed"); return -2; }
    if (analysis) { const int fr = flush_pipelined_locked(c); if (fr) return fr; }
    const long long r = pipelined_locked(c, arena, arena_len, desc, n, rec, fp_arena, fp_cap, analysis, attr_prob, chunk);
    if (r < 0) {
        // an error path may leave copies into the caller's buffers queued on
        // either pipeline stream: drain both before the caller reuses them
        // (the error string of the failure is kept)
        for (int s : {1, 2}) (void)hipStreamSynchronize(c->slot[s].stream);
        if (c->in_stream) (void)hipStreamSynchronize(c->in_stream);   // chunk copies still reading the arena
    }
    return r;
}

// a pipeline chunk's copy in, queued on the copy stream `cs` as soon as the
// slot's previous chunk has read its packets (ev_free) -- before the host waits
// for that chunk -- so consecutive chunks' copies follow each other on the
// link; span = {lo, hi, total} for stage_and_launch
static int stage_copy(mfp_context c, Slot &S, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                      size_t n, hipStream_t cs, uint64_t span[3]) {
    if (batch_span(arena, arena_len, desc, n, span[0], span[1], span[2])) return -1;
    const uint64_t lo = span[0], sp = span[1] - span[0];
    if (S.free_recorded) { HIPCHK(hipStreamWaitEvent(cs, S.ev_free, 0)); S.free_recorded = false; }
    // (growing frees the old buffers: hipFree waits for the device)
    if (grow(S.d_arena, S.cap_arena, sp + 64) || grow(S.d_desc, S.cap_desc, n + 1)) {
        mfp_set_error("device allocation failed");
        return -2;
    }
    const uint64_t copy = std::min<uint64_t>(sp + 16, arena_len - lo);
    if (copy) HIPCHK(hipMemcpyAsync(S.d_arena, arena + lo, copy, hipMemcpyHostToDevice, cs));
    if (n) HIPCHK(hipMemcpyAsync(S.d_desc, desc, n * sizeof(mfp_pkt_desc), hipMemcpyHostToDevice, cs));
    HIPCHK(hipEventRecord(S.ev_in, cs));
    (void)c;
    return 0;
}

static long long pipelined_locked(mfp_context c, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                                  size_t n, mfp_record *rec, char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                  double *attr_prob, size_t chunk) {
    if (chunk == 0) chunk = (size_t)1 << 20;
    // two chunks in flight on pipeline slots 1 and 2 (three were slower, r05_e2e); the
    // host-to-device copies go one after the other on the copy stream, so the
    // first chunk's kernels start after its own copy, not after a share of all
    constexpr int NP = 2;
    static constexpr int slot_of[NP] = {1, 2};
    if (!c->in_stream) HIPCHK(hipStreamCreateWithFlags(&c->in_stream, hipStreamNonBlocking));
    struct Inflight { bool live; size_t lo, hi; };
    Inflight inf[NP] = {};
    uint64_t fp_base = 0;
    // wait for the chunk in pipeline slot s, queue the copy of its packed
    // fingerprints to the caller's arena (chunk order; the slot's next chunk
    // queues behind it on the same stream) and rebase its records
    auto retire = [&](int s) -> int {
        Slot &S = c->slot[slot_of[s]];
        HIPCHK(hipStreamSynchronize(S.stream));
        if (analysis) {   // (the pipeline always decides its chunks itself, in order)
            const int r = slot_resolve_host(c, S, analysis + inf[s].lo, rec + inf[s].lo);
            if (r) return r;
        }
        const unsigned long long used = S.h_used[2];   // dense bytes
        if (S.h_used[1] || fp_base + used > fp_cap) { mfp_set_error("fingerprint arena overflow (cap %zu)", fp_cap); return -4; }
        if (used) HIPCHK(hipMemcpyAsync(fp_arena + fp_base, S.d_fp2, used, hipMemcpyDeviceToHost, S.stream));
        for (size_t i = inf[s].lo; i < inf[s].hi; i++) rec[i].fp_offset += fp_base;
        fp_base += used;
        inf[s].live = false;
        return 0;
    };
    const size_t nch = (n + chunk - 1) / chunk;
    for (size_t k = 0; k < nch; k++) {
        const int s = (int)(k % NP);
        Slot &S = c->slot[slot_of[s]];
        const size_t lo = k * chunk, hi = std::min(n, lo + chunk), m = hi - lo;
        uint64_t span[3];
        {   // the copy in first, then the wait for the slot's previous chunk
            const int r = stage_copy(c, S, arena, arena_len, desc + lo, m, c->in_stream, span);
            if (r) return r;
        }
        if (inf[s].live) { int r = retire(s); if (r) return r; }
        uint64_t bytes = 0;
        for (size_t i = lo; i < hi; i++) bytes += desc[i].caplen;
        const size_t cap = mfp_fp_arena_bound(m, bytes);
        int r = stage_and_launch(c, slot_of[s], arena, arena_len, desc + lo, m, cap, analysis != nullptr,
                                 attr_prob != nullptr, false, span);
        if (r) return r;
        if (analysis) HIPCHK(hipMemcpyAsync(analysis + lo, S.d_an, m * sizeof(mfp_analysis), hipMemcpyDeviceToHost, S.stream));
        if (analysis && attr_prob && m)
            HIPCHK(hipMemcpyAsync(attr_prob + lo * MFP_ATTR_DB_TAGS, S.d_ap, m * MFP_ATTR_DB_TAGS * sizeof(double),
                                  hipMemcpyDeviceToHost, S.stream));
        HIPCHK(hipMemcpyAsync(rec + lo, S.d_rec, m * sizeof(mfp_record), hipMemcpyDeviceToHost, S.stream));
        HIPCHK(hipMemcpyAsync(S.h_used, S.d_used, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, S.stream));
        inf[s] = {true, lo, hi};
    }
    for (size_t k = nch > (size_t)NP ? nch - NP : 0; k < nch; k++) {   // the chunks still in flight, oldest first
        const int s = (int)(k % NP);
        if (inf[s].live) { int r = retire(s); if (r) return r; }
    }
    for (int s = 0; s < NP; s++) HIPCHK(hipStreamSynchronize(c->slot[slot_of[s]].stream));   // the last string copies
    return (long long)fp_base;
}

// ---------------------------------------------------------------------------
// --analysis (process classifier) entry points
// ---------------------------------------------------------------------------
extern "C" MFP_EXPORT int mfp_analysis_enabled(mfp_context c) { return c && c->clf ? 1 : 0; }

extern "C" MFP_EXPORT int mfp_analyze_batch_device(mfp_context c, const uint8_t *d_arena, const mfp_pkt_desc *d_desc,
                                                   size_t n, mfp_record *d_rec, const char *d_fp_arena,
                                                   mfp_analysis *d_out, double *d_attr_prob, void *stream) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (!c->clf) { mfp_set_error("analysis is not enabled (config needs resources=<archive>;analysis)"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    if (const int fr = flush_pipelined_locked(c)) return fr;
    const int r = analyze_locked(c, 0, d_arena, d_desc, n, d_rec, d_fp_arena, d_out, d_attr_prob, (hipStream_t)stream);
    if (r) return r;
    HIPCHK(hipEventRecord(c->slot[0].ev_dev, (hipStream_t)stream));
    c->slot[0].dev_recorded = true;
    if (c->defer) return 0;
    // the batch's unknown-TLS sightings are decided now, in stream order: the
    // call waits for its kernels (a few microseconds of host time per batch)
    return slot_resolve(c, c->slot[0]);
}

// Pipelined device batches: batch k's kernels are launched, then batch k-1's
// unknown-TLS sightings are decided (in stream order, on the host) and applied
// while the device runs batch k.  Batches alternate between slots 0 and 3 (each
// has its own sighting table and work lists); a slot's decision work runs on
// the slot's own stream, after the batch's kernels (an event on the caller's
// stream), and the caller's stream waits for it before the slot is reused.
// The batch's analysis records are final after the next call, or
// mfp_analysis_flush, for work the caller enqueues on its stream afterwards.
extern "C" MFP_EXPORT int mfp_analyze_batch_device_pipelined(mfp_context c, const uint8_t *d_arena,
                                                             const mfp_pkt_desc *d_desc, size_t n, mfp_record *d_rec,
                                                             const char *d_fp_arena, mfp_analysis *d_out,
                                                             double *d_attr_prob, void *stream) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (!c->clf) { mfp_set_error("analysis is not enabled (config needs resources=<archive>;analysis)"); return -1; }
    if (c->defer) {   // the deferred (shard-merge) mode decides its batches through mfp_analysis_resolve*
        mfp_set_error("mfp_analyze_batch_device_pipelined: the context defers its prevalence decisions "
                      "(mfp_analysis_defer); use mfp_analyze_batch_device");
        return -1;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t us = (hipStream_t)stream;
    const int slot = c->pipe_next ? 3 : 0, other = c->pipe_next ? 0 : 3;
    Slot &S = c->slot[slot];
    // a deferred or failed synchronous batch left in slot 0 is decided first
    if (S.pend.live) { int r = slot_resolve(c, S); if (r) return r; }
    if (S.resolved_recorded) HIPCHK(hipStreamWaitEvent(us, S.ev_resolved, 0));
    int r = analyze_locked(c, slot, d_arena, d_desc, n, d_rec, d_fp_arena, d_out, d_attr_prob, us);
    if (r) return r;
    HIPCHK(hipEventRecord(S.ev_kernels, us));
    HIPCHK(hipEventRecord(S.ev_dev, us));
    S.dev_recorded = true;
    HIPCHK(hipStreamWaitEvent(S.stream, S.ev_kernels, 0));
    S.pend.stream = S.stream;
    c->pipe_next ^= 1;
    c->pipe_active = true;
    Slot &O = c->slot[other];
    if (O.pend.live) {
        r = slot_resolve(c, O);
        if (r) {
            // the older batch's statuses stay undecided; the new batch stays
            // pending (the next call or mfp_analysis_flush decides it), so the
            // context remains usable -- the error says which records are unfinished
            O.pend.live = false;
            mfp_set_error("mfp_analyze_batch_device_pipelined: deciding the previous batch's prevalence failed "
                          "(its unknown-TLS statuses are undecided): %s", mfp_last_error());
            return r;
        }
        HIPCHK(hipEventRecord(O.ev_resolved, O.stream));
        O.resolved_recorded = true;
        HIPCHK(hipStreamWaitEvent(us, O.ev_resolved, 0));   // later work on the caller's stream sees its records
    }
    return 0;
}

// The deferred (shard-merge) form of the pipeline: batch k's kernels are
// launched on slot 0 or 3 (alternating) and batch k-1, if it is still
// pending, becomes the batch the mfp_analysis_distinct / _sequence /
// _resolve* calls act on -- so the ranks' ordered merge of batch k-1
// (shard.ordered_prevalence_merge) runs on the host while the device runs
// batch k.  The slot is reused two calls later, after its decision was
// applied (the caller's stream waits for it); mfp_analysis_defer_newest makes
// the last batch the one the calls act on.
extern "C" MFP_EXPORT int mfp_analyze_batch_device_deferred_pipelined(mfp_context c, const uint8_t *d_arena,
                                                                      const mfp_pkt_desc *d_desc, size_t n,
                                                                      mfp_record *d_rec, const char *d_fp_arena,
                                                                      mfp_analysis *d_out, double *d_attr_prob,
                                                                      void *stream) {
    if (!c) { mfp_set_error("null context"); return -1; }
    if (!c->clf) { mfp_set_error("analysis is not enabled (config needs resources=<archive>;analysis)"); return -1; }
    if (!c->defer) {
        mfp_set_error("mfp_analyze_batch_device_deferred_pipelined: the context decides its own batches "
                      "(mfp_analysis_defer is off); use mfp_analyze_batch_device_pipelined");
        return -1;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t us = (hipStream_t)stream;
    const int slot = c->pipe_next ? 3 : 0, other = c->pipe_next ? 0 : 3;
    Slot &S = c->slot[slot];
    if (S.pend.live) {
        mfp_set_error("mfp_analyze_batch_device_deferred_pipelined: the batch two calls back was not decided "
                      "(mfp_analysis_resolve / mfp_analysis_resolve_sequence)");
        return -1;
    }
    if (S.resolved_recorded) HIPCHK(hipStreamWaitEvent(us, S.ev_resolved, 0));
    int r = analyze_locked(c, slot, d_arena, d_desc, n, d_rec, d_fp_arena, d_out, d_attr_prob, us);
    if (r) return r;
    HIPCHK(hipEventRecord(S.ev_kernels, us));
    HIPCHK(hipEventRecord(S.ev_dev, us));
    S.dev_recorded = true;
    HIPCHK(hipStreamWaitEvent(S.stream, S.ev_kernels, 0));
    S.pend.stream = S.stream;
    c->pipe_next ^= 1;
    Slot &O = c->slot[other];
    if (O.pend.live) c->an_slot = other;   // the calls decide the older batch first
    return 0;
}

// the deferred calls act on the newest analysed batch (after the last
// pipelined call, to decide it)
extern "C" MFP_EXPORT int mfp_analysis_defer_newest(mfp_context c) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    const int newest = c->pipe_next ? 0 : 3;   // the slot the last pipelined call used
    if (c->slot[newest].pend.live) c->an_slot = newest;
    return 0;
}

// decide the pipelined batch still pending and wait for its records
extern "C" MFP_EXPORT int mfp_analysis_flush(mfp_context c) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    c->pipe_active = true;                    // whatever is pending in 0 / 3, the older first
    if (const int r = flush_pipelined_locked(c)) return r;
    for (int k : {0, 3}) HIPCHK(hipStreamSynchronize(c->slot[k].stream));
    return 0;
}

// ---- the prevalence LRU: sharing across the shards of one stream ----
extern "C" MFP_EXPORT mfp_prevalence mfp_analysis_prevalence(mfp_context c) { return c ? c->prev : nullptr; }

extern "C" MFP_EXPORT int mfp_analysis_set_prevalence(mfp_context c, mfp_prevalence p) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    c->prev = p ? p : c->own_prev;
    return 0;
}

extern "C" MFP_EXPORT int mfp_analysis_defer(mfp_context c, int on) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    c->defer = on != 0;
    return 0;
}

static Slot *deferred_slot(mfp_context c) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return nullptr; }
    Slot &S = c->slot[c->an_slot];
    if (!S.pend.live) { mfp_set_error("no analysed batch waits for its prevalence decisions"); return nullptr; }
    return &S;
}

extern "C" MFP_EXPORT long long mfp_analysis_distinct(mfp_context c, mfp_sighting *out, size_t cap) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot *S = deferred_slot(c);
    if (!S) return -1;
    HIPCHK(hipSetDevice(c->device));
    if (!out && S->pend.dist_u == -5) {   // the count alone: the table's counters, no export
        unsigned int cnt[4];
        HIPCHK(hipMemcpyAsync(cnt, S->seen.counters, sizeof cnt, hipMemcpyDeviceToHost, S->pend.stream));
        HIPCHK(hipStreamSynchronize(S->pend.stream));
        return cnt[1] || cnt[0] > S->seen.list_cap ? -3 : (long long)cnt[0];
    }
    if (S->pend.dist_u == -5) {   // once per pending batch
        S->pend.dist_u = slot_distinct(c, *S, S->pend.dist);
        if (S->pend.dist_u == -2) { const long long e = S->pend.dist_u; S->pend.dist_u = -5; return e; }
    }
    const long long u = S->pend.dist_u;
    if (u < 0) return u;
    if (out) memcpy(out, S->pend.dist.data(), std::min<size_t>(cap, S->pend.dist.size()) * sizeof(mfp_sighting));
    return u;
}

extern "C" MFP_EXPORT long long mfp_analysis_sequence(mfp_context c, uint64_t *hash, size_t cap) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot *S = deferred_slot(c);
    if (!S) return -1;
    HIPCHK(hipSetDevice(c->device));
    long long m = S->pend.seq_m;
    if (m < 0) {   // once per pending batch (h_seq keeps it until the slot's next sequence)
        m = slot_sequence(c, *S);
        if (m < 0) return m;
        S->pend.seq_m = m;
    }
    if (hash) memcpy(hash, S->h_seq, std::min<size_t>(cap, (size_t)m) * 8);
    return m;
}

extern "C" MFP_EXPORT int mfp_analysis_resolve(mfp_context c, const mfp_sighting *d, size_t u) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot *S = deferred_slot(c);
    if (!S) return -1;
    HIPCHK(hipSetDevice(c->device));
    if (u && !d) { mfp_set_error("mfp_analysis_resolve: null decisions"); return -1; }
    {   // one decision per distinct entry of the pending batch (the resolve kernel
        // indexes them by position): the sighting table's counters say how many
        unsigned int cnt[4];
        HIPCHK(hipMemcpyAsync(cnt, S->seen.counters, sizeof cnt, hipMemcpyDeviceToHost, S->pend.stream));
        HIPCHK(hipStreamSynchronize(S->pend.stream));
        if (cnt[1] || cnt[0] > S->seen.list_cap) {
            mfp_set_error("mfp_analysis_resolve: the batch's sighting table overflowed (use the sequence form)");
            return -3;
        }
        if ((size_t)cnt[0] != u) {
            mfp_set_error("mfp_analysis_resolve: %zu decisions, the batch has %u distinct fingerprints", u, cnt[0]);
            return -1;
        }
    }
    if (grow_pinned(S->h_dec, S->cap_h_dec, u + 1)) { mfp_set_error("host allocation failed"); return -2; }
    for (size_t i = 0; i < u; i++) S->h_dec[i] = (uint8_t)d[i].first_seen;
    const int r = slot_apply(c, *S, S->h_dec, u, false);
    if (r == 0) HIPCHK(hipStreamSynchronize(S->pend.stream));
    return r;
}

extern "C" MFP_EXPORT long long mfp_analysis_last(mfp_context c, mfp_analysis *out, size_t cap) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot &S = c->slot[c->an_slot];
    if (!S.pend.out) { mfp_set_error("no analysed batch"); return -1; }
    HIPCHK(hipSetDevice(c->device));
    const size_t m = std::min<size_t>(cap, S.pend.n);
    if (m) HIPCHK(hipMemcpyAsync(out, S.pend.out, m * sizeof(mfp_analysis), hipMemcpyDeviceToHost, S.pend.stream));
    HIPCHK(hipStreamSynchronize(S.pend.stream));
    return (long long)S.pend.n;
}

extern "C" MFP_EXPORT int mfp_analysis_resolve_sequence(mfp_context c, const uint8_t *seen, size_t m) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    Slot *S = deferred_slot(c);
    if (!S) return -1;
    HIPCHK(hipSetDevice(c->device));
    // the group offsets the resolve kernel reads: left on the device by this
    // batch's sequence (mfp_analysis_sequence), or computed now
    long long ms = S->pend.seq_m;
    if (ms < 0) ms = slot_sequence(c, *S);
    if (ms < 0) return (int)ms;
    S->pend.seq_m = ms;
    if ((size_t)ms != m) { mfp_set_error("sequence length %zu, batch has %lld sightings", m, ms); return -1; }
    const int r = slot_apply(c, *S, seen, m, true);
    if (r == 0) HIPCHK(hipStreamSynchronize(S->pend.stream));
    return r;
}

extern "C" MFP_EXPORT const char *mfp_process_name(mfp_context c, uint32_t id) {
    return c && c->clf ? mfp_classifier_process_name(c->clf, id) : nullptr;
}

extern "C" MFP_EXPORT const char *mfp_attribute_name(mfp_context c, uint32_t bit) {
    return c && c->clf ? mfp_classifier_attr_name(c->clf, bit) : nullptr;
}

extern "C" MFP_EXPORT const char *mfp_resource_version(mfp_context c) {
    return c && c->clf ? mfp_classifier_version(c->clf) : nullptr;
}

extern "C" MFP_EXPORT int mfp_attribute_count(mfp_context c) {
    return c && c->clf ? mfp_classifier_attr_count(c->clf) : 0;
}

// the attribute names' total length (the JSON writer's per-record bound), once per context
size_t mfp_attribute_names_len(mfp_context c) {
    if (!c || !c->clf) return 0;
    size_t v = c->attr_names_len.load(std::memory_order_relaxed);
    if (v != SIZE_MAX) return v;
    v = 0;
    const int na = mfp_classifier_attr_count(c->clf);
    for (int k = 0; k < na; k++) {
        const char *nm = mfp_classifier_attr_name(c->clf, (uint32_t)k);
        v += nm ? strlen(nm) : 0;
    }
    c->attr_names_len.store(v, std::memory_order_relaxed);
    return v;
}

extern "C" MFP_EXPORT int mfp_analysis_report_os(mfp_context c, int on) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    c->report_os = on != 0;
    return 0;
}

extern "C" MFP_EXPORT int mfp_process_os_info(mfp_context c, uint32_t proc_slot, uint32_t k, const char **name,
                                              uint64_t *prevalence) {
    if (!c || !c->clf) { mfp_set_error("analysis is not enabled"); return -1; }
    const int cnt = mfp_classifier_os_info(c->clf, proc_slot, k, name, prevalence);
    if (cnt < 0) { mfp_set_error("bad process slot %u", proc_slot); return -1; }
    return c->report_os ? cnt : 0;
}

extern "C" MFP_EXPORT int mfp_analysis_stats(mfp_context c, uint64_t out[4]) {
    if (!c || !c->clf) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    unsigned long long h[4];
    HIPCHK(hipMemcpy(h, c->slot[c->an_slot].d_an_stats, sizeof h, hipMemcpyDeviceToHost));
    out[0] = h[0]; out[1] = h[1]; out[2] = h[2]; out[3] = mfp_prevalence_size(c->prev);
    return 0;
}

extern "C" MFP_EXPORT int mfp_analysis_counters(mfp_context c, uint64_t *out, size_t n) {
    if (!c || !c->clf || (n && !out)) { mfp_set_error("analysis is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    unsigned long long h[MFP_AN_STATS_WORDS];
    HIPCHK(hipMemcpy(h, c->slot[c->an_slot].d_an_stats, sizeof h, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < n && k < MFP_AN_STATS_WORDS; k++) out[k] = h[k];   // (words past the counters: probe builds)
    return 0;
}

extern "C" MFP_EXPORT uint64_t mfp_analysis_device_bytes(mfp_context c) {
    return c && c->clf ? mfp_classifier_device_bytes(c->clf) : 0;
}

// host-only: load a resource archive and report its size (no device needed)
extern "C" MFP_EXPORT int mfp_resource_stats(const char *path, uint64_t out[8]) {
    return mfp_resource_stats_ex(path, nullptr, out);
}

extern "C" MFP_EXPORT int mfp_resource_stats_ex(const char *path, const uint8_t *enc_key, uint64_t out[8]) {
    mfp_classifier *clf = mfp_classifier_load(path, enc_key);
    if (!clf) return -1;
    mfp_classifier_stats(clf, out);
    mfp_classifier_free(clf);
    return 0;
}

extern "C" MFP_EXPORT int mfp_profile_enable(mfp_context c, int on) {
    if (!c) { mfp_set_error("null context"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (on) {
        if (!c->prof) c->prof = new mfp_prof;
        c->prof->reset();
    } else {
        delete c->prof;
        c->prof = nullptr;
    }
    return 0;
}

extern "C" MFP_EXPORT int mfp_profile_read(mfp_context c, uint32_t i, char *name, size_t cap, uint64_t *launches,
                                           double *total_ms) {
    if (!c || !c->prof) { mfp_set_error("profiling is not enabled"); return -1; }
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (c->prof->collect() != 0) { mfp_set_error("event timing failed"); return -2; }
    if (i >= c->prof->names.size()) return 1;
    const std::string &k = c->prof->names[i];
    if (name && cap) snprintf(name, cap, "%s", k.c_str());
    const auto &v = c->prof->acc[k];
    if (launches) *launches = v.first;
    if (total_ms) *total_ms = v.second;
    return 0;
}
