// mfp_libmerc.cpp -- the reference's per-packet libmerc C API
// (include/mercury_amd_libmerc.h) over the batch path of include/mfp.h.
// Every call is a one-packet batch on the GPU; the high-throughput
// interface is the batch API.  File:line cites are relative to
// /root/reference/src/libmerc/.
#include <algorithm>
#include <new>

#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mercury_amd_libmerc.h"
#include "../../include/mfp.h"
#include "mfp_common.hpp"
#include "mfp_internal.h"

struct mercury {
    std::string cfg;              // packet_filter_cfg as mfp_init takes it
    bool analysis = false;
    bool report_os = false;
    std::mutex mu;
    mfp_context ctx[2] = {nullptr, nullptr};   // per reference entry point (write_json / analysis)
    // one fingerprint_prevalence for the mercury context (the reference's
    // classifier owns one, shared by every processor and entry point)
    mfp_prevalence prev = nullptr;
    uint8_t enc_key[16] = {0};    // libmerc_config.enc_key (encrypted resource archive)
    bool keyed = false;
    // packets identified as a selected protocol outside the device path
    // (MFP_MSG_OTHER, e.g. under "all"): they write no record; counted, and
    // logged once per context
    std::atomic<uint64_t> other{0};
    // concurrent per-packet calls on this context are combined into one device
    // batch per entry point (see submit())
    struct Combiner *comb[2] = {nullptr, nullptr};
};

struct analysis_context {       // the fields libmerc's accessors read (result.h:174-420)
    char fp[8193];
    uint32_t fp_type = 0;
    uint32_t status = 0;
    char sn[257];               // destination_context::sn_str (MAX_SNI_LEN)
    char ua[512];               // destination_context::ua_str (MAX_USER_AGENT_LEN)
    uint8_t alpn[128];          // destination_context::alpn_array (MAX_ALPN_STR_LEN)
    size_t alpn_len = 0;
    std::string process;
    double score = 0, malware_prob = -1;
    bool malware = false, classify_malware = false, has_process = false;
    std::vector<os_information> os;             // analysis_result::os_info
    uint32_t attr = 0;                          // attribute_result tags
    long double prob[MFP_ATTR_MAX_TAGS];        // attribute_result::prob_score
    const char *tag_names[MFP_ATTR_MAX_TAGS];
    size_t n_tags = 0;
    attribute_context actx;
};

struct mercury_packet_processor_s {
    mercury *mc;
    analysis_context ac;
    std::vector<uint8_t> arena;
    std::vector<char> fp;
    mfp_reassembler reasm = nullptr;   // the processor's tcp_reassembler ("reassembly" configured)
    bool more_pkts = false;            // analysis_context::flow_state_pkts_needed (result.h:386)
    ~mercury_packet_processor_s() { if (reasm) mfp_reassembler_destroy(reasm); }
};

// printf_err_func (printf_err.hpp:22-45): the default emitter, a level prefix
// and the message on stderr
static int stderr_err(enum log_level level, const char *format, va_list args) {
    static const char *pfx[] = {"emergency: ", "alert: ", "critical: ", "error: ", "warning: ",
                                "notice: ", "informational: ", "debug: ", ""};
    const int r = std::fprintf(stderr, "%s", pfx[(unsigned)level <= log_none ? (unsigned)level : (unsigned)log_none]);
    if (r < 0) return r;
    const int s = std::vfprintf(stderr, format, args);
    return s < 0 ? s : r + s;
}
static int silent_err(enum log_level, const char *, va_list) { return 0; }
static void free_combiners(mercury *m);   // silent_err_func printf_err.hpp:47
static void print_kernel_stats(mfp_context c);

static printf_err_ptr g_printf_err = stderr_err;

static void log_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    g_printf_err(log_err, fmt, ap);
    va_end(ap);
}
static void log_warn(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    g_printf_err(log_warning, fmt, ap);
    va_end(ap);
}
// a message of a selected protocol this path does not parse: no record
static void note_other(mercury *m, const mfp_record &rec) {
    if (rec.msg != MFP_MSG_OTHER) return;
    if (m->other.fetch_add(1, std::memory_order_relaxed) == 0)
        log_warn("the selection names protocols outside the MI355X device path (tls, dtls, ssh, http, tcp, "
                    "quic, stun, openvpn_tcp, gre, vxlan, geneve); their messages write no record\n");
}

#ifndef MFP_GIT_COMMIT
#define MFP_GIT_COMMIT "commit unknown"   // libmerc.cc:29-36
#endif

extern "C" {

// register_printf_err_callback libmerc.cc:473-475: NULL silences the library
MFP_EXPORT void register_printf_err_callback(printf_err_ptr callback) {
    g_printf_err = callback ? callback : silent_err;
}

// mercury_init libmerc.cc:92-128 / struct mercury pkt_proc.h:56-114
MFP_EXPORT mercury_context mercury_init(const struct libmerc_config *vars, int verbosity) {
    (void)verbosity;
    if (!vars) return nullptr;
    // libmerc_config fields that change the records (pkt_proc.cc:1157-1253,
    // write_metadata pkt_proc_util.h:264-333, analysis.h:836): refused at init
    // with the reason, as unsupported configurations are refused, rather than
    // silently giving records that differ from the reference's.  dns_json_output
    // changes DNS records only, which this path does not write: accepted.
    const struct { bool on; const char *what; } refused[] = {
        {vars->do_stats, "do_stats: fingerprint/destination statistics (stats.h)"},
        {vars->metadata_output, "metadata_output: the metadata JSON fields (write_metadata pkt_proc_util.h:264)"},
        {vars->certs_json_output, "certs_json_output: certificates as parsed JSON (tls.h, x509.h)"},
        {vars->output_tcp_initial_data, "output_tcp_initial_data: tcp.data records for unselected TCP payloads"},
        {vars->output_udp_initial_data, "output_udp_initial_data: udp.data records for unselected UDP payloads"},
        {vars->fp_proc_threshold > 0.0f || vars->proc_dst_threshold > 0.0f,
         "fp_proc_threshold / proc_dst_threshold: the thresholded database (analysis.h:836)"},
    };
    for (const auto &r : refused)
        if (r.on) {
            log_error("%s is not provided by libmercury_amd\n", r.what);
            return nullptr;
        }
    auto *m = new mercury;
    // the archive key: 16 bytes whatever key_type says (analysis.h:1211,
    // "TODO: key type"; cryptovar<16>)
    if (vars->enc_key) { memcpy(m->enc_key, vars->enc_key, 16); m->keyed = true; }
    std::string filt = vars->packet_filter_cfg ? vars->packet_filter_cfg : "";
    // global_config.h:148-152: "key=value;..." only when the string holds ';'
    // a bare list stays bare (mfp_init parses it the same way); key=value options are added in the ';' form
    std::string cfg = filt.empty() ? std::string("all") : filt;
    if (vars->do_analysis && vars->resources) {
        if (cfg.find(';') == std::string::npos) cfg = "select=" + cfg;
        cfg += std::string(";resources=") + vars->resources + ";analysis";
        m->analysis = true;
    }
    m->cfg = cfg;
    // validate now, so a bad configuration fails at init as in the reference
    uint32_t sel, fmt;
    int ros = -1;
    std::string warn;
    if (!mfp_parse_config(cfg.c_str(), sel, fmt, nullptr, nullptr, nullptr, nullptr, &warn, &ros)) {
        log_error("%s\n", mfp_last_error());
        delete m;
        return nullptr;
    }
    if (!warn.empty()) log_error("%s\n", warn.c_str());   // printf_err(log_err, ...) as set_protocols does, and go on
    // the config string's report_os setter overrides the field (config_generator.cc:35)
    m->report_os = ros < 0 ? vars->report_os : ros == 1;
    return m;
}

MFP_EXPORT int mercury_finalize(mercury_context mc) {
    if (!mc) return -1;
    if (const char *e = getenv("MFP_SHIM_STATS"); e && atoi(e) >= 2)
        for (auto &c : mc->ctx) if (c) print_kernel_stats(c);
    for (auto &c : mc->ctx) if (c) mfp_finalize(c);
    free_combiners(mc);
    if (mc->prev) mfp_prevalence_destroy(mc->prev);
    delete mc;
    return 0;
}

static mfp_context get_ctx(mercury *m, int mode) {
    std::lock_guard<std::mutex> lk(m->mu);
    if (!m->ctx[mode]) {
        mfp_context c = mfp_init_ex(m->cfg.c_str(), 0, mode, m->keyed ? m->enc_key : nullptr);
        if (!c) { log_error("%s\n", mfp_last_error()); return nullptr; }
        if (mfp_analysis_enabled(c)) {
            if (!m->prev) m->prev = mfp_prevalence_create(100000);   // analysis.h:433
            mfp_analysis_set_prevalence(c, m->prev);
            mfp_analysis_report_os(c, m->report_os ? 1 : 0);
        }
        // MFP_SHIM_STATS=2: kernel times too (two events per launch: not for timing runs)
        if (const char *e = getenv("MFP_SHIM_STATS"); e && atoi(e) >= 2) mfp_profile_enable(c, 1);
        m->ctx[mode] = c;
    }
    return m->ctx[mode];
}

// MFP_SHIM_STATS: the device time of each kernel the per-packet calls launched
static void print_kernel_stats(mfp_context c) {
    char name[64];
    uint64_t launches = 0;
    double ms = 0;
    fprintf(stderr, "{\"shim_kernels\": {");
    for (uint32_t i = 0; mfp_profile_read(c, i, name, sizeof name, &launches, &ms) == 0; i++)
        fprintf(stderr, "%s\"%s\": [%llu, %.3f]", i ? ", " : "", name, (unsigned long long)launches, ms);
    fprintf(stderr, "}}\n");
}

MFP_EXPORT mercury_packet_processor mercury_packet_processor_construct(mercury_context mc) {
    if (!mc) return nullptr;
    auto *p = new mercury_packet_processor_s;
    p->mc = mc;
    return p;
}

MFP_EXPORT void mercury_packet_processor_destruct(mercury_packet_processor mpp) { delete mpp; }

static void copy_cstr(char *dst, size_t cap, const uint8_t *src, size_t len) {   // datum::strncpy
    size_t n = len < cap - 1 ? len : cap - 1;
    size_t k = 0;
    for (; k < n && src[k]; k++) dst[k] = (char)src[k];
    dst[k] = 0;
}

// the processor's analysis_context from one classified packet (the state the
// reference's accessors read after write_json or get_analysis_context)
static void fill_context(mfp_context ctx, analysis_context &ac, const uint8_t *pkt, uint32_t caplen,
                         const mfp_record &rec, const char *fp, const mfp_analysis *an, const double *ap) {
    ac.fp_type = rec.fp_type;
    copy_cstr(ac.fp, sizeof ac.fp, (const uint8_t *)fp + rec.fp_offset, rec.fp_type ? rec.fp_len : 0);
    // the sni slot holds the certificate_list (TLS server), the STUN message or
    // the OpenVPN payload for those messages; the ua slot holds the ALPN list
    // of (D)TLS ClientHellos; QUIC spans index the sidecar behind the string
    const bool no_sn = rec.msg == MFP_MSG_TLS_SH || rec.msg == MFP_MSG_TLS_CERT || rec.msg == MFP_MSG_STUN ||
                       rec.msg == MFP_MSG_OPENVPN;
    const bool hello = rec.msg == MFP_MSG_TLS_CH || rec.msg == MFP_MSG_DTLS_CH;
    const uint8_t *sb = (rec.flags & MFP_FLAG_SIDECAR)
                            ? (const uint8_t *)fp + rec.fp_offset + ((rec.fp_len + 7) & ~7u) + 8 : pkt;
    copy_cstr(ac.sn, sizeof ac.sn, sb + rec.sni_off, rec.sni_len == 0xffff || no_sn ? 0 : rec.sni_len);
    if (rec.msg == MFP_MSG_SSH_INIT && rec.ua_len != 0xffff) {
        // protocol + comment (ssh.h:480-487): the span's first space is the
        // delimiter; a data_buffer<512> that does not hold both is null
        std::string u;
        bool skipped = false;
        for (uint32_t j = 0; j < rec.ua_len; j++) {
            if (!skipped && pkt[rec.ua_off + j] == ' ') { skipped = true; continue; }
            u.push_back((char)pkt[rec.ua_off + j]);
        }
        if (u.size() > 512) u.clear();
        copy_cstr(ac.ua, sizeof ac.ua, (const uint8_t *)u.data(), u.size());
    } else if (rec.msg == MFP_MSG_STUN) {
        // utf8_safe_string<512> of the SOFTWARE value (stun.h:1024-1027)
        const uint32_t n = rec.ua_len == 0xffff ? 0 : mfpc::utf8_safe_512(pkt + rec.ua_off, rec.ua_len, ac.ua);
        ac.ua[n] = 0;
    } else {
        // a (D)TLS hello's ua span is its ALPN list, unless it holds the user
        // agent of a draft transport-parameter extension (MFP_XF_TLS_UA)
        const bool alpn_span = hello && !(rec.xflags & MFP_XF_TLS_UA);
        copy_cstr(ac.ua, sizeof ac.ua, sb + rec.ua_off, rec.ua_len == 0xffff || alpn_span ? 0 : rec.ua_len);
    }
    ac.alpn_len = 0;
    ac.alpn[0] = 0;
    if (hello) {   // alpn.write_to_buffer(alpn_array, 128) (result.h:352-353)
        const uint8_t *a = nullptr;
        uint32_t al = 0;
        if (!(rec.xflags & MFP_XF_TLS_UA)) {
            if (rec.ua_len != 0xffff) { a = pkt + rec.ua_off; al = rec.ua_len; }
        } else {
            mfp_hello_alpn(pkt, caplen, rec, &a, &al);
        }
        if (a) {
            ac.alpn_len = al;
            memcpy(ac.alpn, a, std::min<size_t>(al, sizeof ac.alpn));
        }
    }
    ac.status = 0; ac.has_process = false; ac.process.clear(); ac.score = 0; ac.malware = false;
    ac.classify_malware = false; ac.malware_prob = -1; ac.os.clear(); ac.attr = 0; ac.n_tags = 0;
    if (!an) return;
    ac.status = an->status;
    ac.has_process = an->process != MFP_NO_PROCESS;
    ac.process = ac.has_process ? mfp_process_name(ctx, an->process) : "";
    if (ac.process.size() > 255) ac.process.resize(255);   // max_proc (result.h:176,198)
    ac.score = an->score;
    ac.malware = an->flags & MFP_AN_MALWARE;
    ac.classify_malware = an->flags & MFP_AN_CLASSIFY_MALWARE;
    ac.malware_prob = an->malware_prob;
    if (an->proc_slot != MFP_NO_PROCESS) {
        const int cnt = mfp_process_os_info(ctx, an->proc_slot, 0, nullptr, nullptr);
        for (int k = 0; k < cnt; k++) {
            const char *nm = nullptr;
            uint64_t prev = 0;
            mfp_process_os_info(ctx, an->proc_slot, (uint32_t)k, &nm, &prev);
            ac.os.push_back(os_information{(char *)nm, prev});
        }
    }
    ac.attr = an->attr;
    ac.n_tags = (size_t)mfp_attribute_count(ctx);
    for (size_t k = 0; k < MFP_ATTR_MAX_TAGS; k++) {
        ac.tag_names[k] = k < ac.n_tags ? mfp_attribute_name(ctx, (uint32_t)k) : nullptr;
        long double p = 0;
        if ((ac.attr >> k) & 1u) {
            if (k >= MFP_ATTR_DB_FIRST) p = ap ? ap[k - MFP_ATTR_DB_FIRST] : 0;
            else if (k == 7) p = an->malware_prob;   // encrypted_channel
            else p = 1.0;                            // encrypted_dns, domain_faking, faketls
        }
        ac.prob[k] = p;
    }
}

// ts->tv_sec == 0: the reference writes the time of tsc_clock, the TSC in
// seconds (pkt_proc.cc:1086-1089, 1619-1622; tsc_clock.hpp:64-70) -- the
// seconds since the counter started, not wall time; tv_nsec is left alone.
// CLOCK_MONOTONIC counts from the same start (boot).
static void fill_zero_ts(struct timespec *ts) {
    if (!ts || ts->tv_sec != 0) return;
    struct timespec m;
    clock_gettime(CLOCK_MONOTONIC, &m);
    ts->tv_sec = (time_t)((double)m.tv_sec + 1e-9 * (double)m.tv_nsec + 0.5);
}

// ---------------------------------------------------------------------------
// Combining: libmerc's API is one packet per call, one processor per thread
// (libmerc.h:227-231).  Each call on the device path is a batch of its own --
// a copy in, a few kernel launches, one wait -- so concurrent calls of
// different processors are combined: a call queues its packet; a caller that
// finds fewer than max_leaders batches in flight becomes a leader, takes every
// queued packet (its own included), runs them as one batch on a small-batch
// slot of the shared context and completes each caller's result; callers that
// arrive meanwhile wait and form the next batch, which may run beside it.  One
// thread calling alone pays one batch per packet, N threads share batches.  A
// batch keeps its packets' arrival order, and each thread's calls are decided
// against the fingerprint-prevalence LRU in its own call order; batches in
// flight together are decided in the order they finish, as the reference's
// shared classifier sees concurrent threads in whichever order they reach it.
// (Processors with "reassembly" keep their own flow table and run their
// packets one by one.)
// ---------------------------------------------------------------------------
struct Req {
    const uint8_t *pkt;
    size_t len;
    uint16_t linktype;
    uint64_t t_ns;
    analysis_context *ac;       // the processor's context, filled by the leader
    void *buf;                  // write_json: the caller's buffer (nullptr: analysis entry)
    size_t buf_size;
    size_t out_len = 0;         // write_json: bytes written (0: none)
    bool valid = false;         // analysis entry: MFP_AN_VALID
    bool err = false;
    bool done = false;
};

// a growable host buffer in page-locked memory: the batch's copies to and
// from the device are then DMA transfers the stream queues, not staged
// through a driver bounce buffer with a wait per copy (pageable memory)
extern "C++" {
template <class T>
struct PinnedVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    PinnedVec() = default;
    PinnedVec(const PinnedVec &) = delete;
    PinnedVec &operator=(const PinnedVec &) = delete;
    ~PinnedVec() { release(); }
    void release() {
        if (p) { if (pinned) (void)hipHostFree(p); else free(p); }
        p = nullptr; cap = 0;
    }
    void reserve(size_t c) {
        if (c <= cap) return;
        const size_t nc = std::max(c, cap * 2 + 64);
        T *q = nullptr;
        bool pq = hipHostMalloc((void **)&q, nc * sizeof(T), hipHostMallocDefault) == hipSuccess;
        if (!pq) { q = static_cast<T *>(malloc(nc * sizeof(T))); if (!q) throw std::bad_alloc(); }
        if (n) memcpy(q, p, n * sizeof(T));
        release();
        p = q; cap = nc; pinned = pq;
    }
    void resize(size_t k) { reserve(k); n = k; }
    void clear() { n = 0; }
    void append(const T *x, size_t k) { reserve(n + k); memcpy(p + n, x, k * sizeof(T)); n += k; }
    size_t size() const { return n; }
    T *data() { return p; }
    T &operator[](size_t i) { return p[i]; }
};
}  // extern "C++"

// one leader's batch buffers, page-locked
struct Bufs {
    PinnedVec<uint8_t> arena;
    PinnedVec<mfp_pkt_desc> desc;
    PinnedVec<mfp_record> rec;
    PinnedVec<char> fp;
    PinnedVec<mfp_analysis> an;
    PinnedVec<double> ap;
    std::vector<uint64_t> ts, ends;
    std::vector<char> out;
};

struct Combiner {
    std::mutex m;
    std::condition_variable cv;
    std::vector<Req *> q;
    // leaders running a batch now: up to max_leaders at once, each on a
    // small-batch slot of its own (mfp_process_small_pinned), so the batches
    // of concurrent callers overlap on the device instead of queueing behind
    // one batch in flight (MFP_SHIM_LEADERS)
    int active = 0, max_leaders = 4;
    std::vector<Bufs *> pool;       // idle leaders' buffers
    // MFP_SHIM_STATS: batches, packets, nanoseconds in the device batch / the
    // records and JSON text (printed by mercury_finalize)
    uint64_t st_batches = 0, st_pkts = 0, st_dev_ns = 0, st_host_ns = 0;
    Combiner() {
        if (const char *e = getenv("MFP_SHIM_LEADERS")) max_leaders = std::max(1, atoi(e));
    }
    ~Combiner() { for (Bufs *b : pool) delete b; }
};

struct BatchTimes { uint64_t dev_ns = 0, host_ns = 0; };

static void run_batch(mercury *m, mfp_context ctx, Bufs &C, std::vector<Req *> &batch, bool json_entry,
                      BatchTimes &bt) {
    const size_t n = batch.size();
    C.arena.clear();
    C.desc.resize(n);
    C.ts.resize(n);
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        const Req &r = *batch[i];
        C.desc[i] = mfp_pkt_desc{(uint64_t)C.arena.size(), (uint32_t)r.len, r.linktype, 0};
        C.arena.append(r.pkt, r.len);
        const size_t at = C.arena.size();
        C.arena.resize((at + 15) & ~(size_t)15);               // 16-byte aligned packets
        memset(C.arena.data() + at, 0, C.arena.size() - at);
        C.ts[i] = r.t_ns;
        total += r.len;
    }
    {   // zero padding the device may read past the last packet (mfp_process_small_pinned)
        const size_t at = C.arena.size();
        C.arena.resize(at + 64);
        memset(C.arena.data() + at, 0, 64);
    }
    const bool want_an = mfp_analysis_enabled(ctx);
    const size_t cap = mfp_fp_arena_bound(n, total);
    C.rec.resize(n);
    C.fp.resize(cap);
    if (want_an) {
        C.an.resize(n);
        C.ap.resize(n * MFP_ATTR_DB_TAGS);
        memset(C.ap.data(), 0, n * MFP_ATTR_DB_TAGS * sizeof(double));
    }
    const auto t0 = std::chrono::steady_clock::now();
    // page-locked buffers throughout: the device writes the results into them
    // (mfp_process_small_pinned); a buffer that could not be pinned takes the
    // copying path
    const bool pinned = C.arena.pinned && C.desc.pinned && C.rec.pinned && C.fp.pinned &&
                        (!want_an || (C.an.pinned && C.ap.pinned));
    auto *const process = pinned ? mfp_process_small_pinned : mfp_process_batch_host_ex;
    const long long used = process(ctx, C.arena.data(), C.arena.size(), C.desc.data(), n, C.rec.data(), C.fp.data(), cap,
                                   want_an ? C.an.data() : nullptr, want_an ? C.ap.data() : nullptr);
    const auto t1 = std::chrono::steady_clock::now();
    bt.dev_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    struct HostClock {
        BatchTimes &bt; std::chrono::steady_clock::time_point t;
        ~HostClock() {
            bt.host_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                std::chrono::steady_clock::now() - t).count();
        }
    } host_clock{bt, t1};
    if (used < 0) {
        log_error("%s\n", mfp_last_error());
        for (Req *r : batch) r->err = true;
        return;
    }
    for (size_t i = 0; i < n; i++) {
        Req &r = *batch[i];
        fill_context(ctx, *r.ac, C.arena.data() + C.desc[i].offset, C.desc[i].caplen, C.rec[i], C.fp.data(),
                     want_an ? &C.an[i] : nullptr, want_an ? &C.ap[i * MFP_ATTR_DB_TAGS] : nullptr);
        note_other(m, C.rec[i]);
        r.valid = want_an && (C.an[i].flags & MFP_AN_VALID);
    }
    if (!json_entry) return;
    C.ends.resize(n);
    if (C.out.size() < ((size_t)1 << 16) + 64 * total) C.out.resize(((size_t)1 << 16) + 64 * total);
    uint64_t skipped = 0;
    long long w;
    while (true) {
        w = want_an ? mfp_write_json_batch_analysis(ctx, C.arena.data(), C.desc.data(), n, C.rec.data(), C.fp.data(),
                                                    C.an.data(), C.ap.data(), C.ts.data(), C.out.data(), C.out.size(),
                                                    C.ends.data(), &skipped, 1)
                    : mfp_write_json_batch(C.arena.data(), C.desc.data(), n, C.rec.data(), C.fp.data(), C.ts.data(),
                                           C.out.data(), C.out.size(), C.ends.data(), &skipped, 1);
        if (w != -2) break;
        C.out.resize(C.out.size() * 2);
    }
    if (w < 0) {
        log_error("%s\n", mfp_last_error());
        for (Req *r : batch) r->err = true;
        return;
    }
    for (size_t i = 0; i < n; i++) {
        Req &r = *batch[i];
        const size_t b = i ? (size_t)C.ends[i - 1] : 0, e = (size_t)C.ends[i];
        if (e == b && (C.rec[i].flags & MFP_FLAG_EMIT) && skipped) {
            // the reference writes a record here; the writer could not rebuild it
            // (an encapsulation chain the host walk cannot follow): say so
            const uint8_t mg = C.rec[i].msg;
            log_error("write_json: record not rebuilt by the MI355X JSON writer (%s)\n",
                      mg == MFP_MSG_QUIC ? "QUIC Initial" : mg == MFP_MSG_STUN ? "STUN message"
                      : mg == MFP_MSG_OPENVPN ? "OpenVPN record" : "encapsulation chain");
        }
        // buffer_stream keeps one byte for its NUL (pkt_proc.cc:1249-1253)
        if (e > b && e - b < r.buf_size) { memcpy(r.buf, C.out.data() + b, e - b); r.out_len = e - b; }
    }
}

static void free_combiners(mercury *m) {
    const bool stats = getenv("MFP_SHIM_STATS") != nullptr;
    for (Combiner *&cb : m->comb) {
        if (cb && stats && cb->st_batches)
            fprintf(stderr, "{\"shim_stats\": {\"batches\": %llu, \"packets\": %llu, \"pkts_per_batch\": %.2f, "
                    "\"device_us_per_batch\": %.2f, \"host_us_per_batch\": %.2f}}\n",
                    (unsigned long long)cb->st_batches, (unsigned long long)cb->st_pkts,
                    (double)cb->st_pkts / (double)cb->st_batches, cb->st_dev_ns / 1e3 / (double)cb->st_batches,
                    cb->st_host_ns / 1e3 / (double)cb->st_batches);
        delete cb;
        cb = nullptr;
    }
}

static void submit(mercury *m, mfp_context ctx, int mode, Req &r) {
    Combiner *C;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        if (!m->comb[mode]) m->comb[mode] = new Combiner;
        C = m->comb[mode];
    }
    std::unique_lock<std::mutex> lk(C->m);
    C->q.push_back(&r);
    while (!r.done) {
        if (C->active < C->max_leaders && !C->q.empty()) {
            C->active++;
            std::vector<Req *> batch;
            batch.swap(C->q);
            Bufs *B = nullptr;
            if (!C->pool.empty()) { B = C->pool.back(); C->pool.pop_back(); }
            lk.unlock();
            BatchTimes bt;
            // the leader hands the batch back on every exit path: an exception
            // out of run_batch (an allocation of the staging vectors) fails the
            // batch's calls instead of leaving the leader counted and the
            // waiters asleep, and never crosses the extern "C" boundary
            // (libmerc.cc:145-149 turns exceptions into 0 / NULL the same way)
            struct Release {
                Combiner *C; std::unique_lock<std::mutex> &lk; std::vector<Req *> &batch; Bufs *&B; BatchTimes &bt;
                ~Release() {
                    lk.lock();
                    for (Req *x : batch) x->done = true;
                    if (B) C->pool.push_back(B);
                    C->active--;
                    C->st_batches++;
                    C->st_pkts += batch.size();
                    C->st_dev_ns += bt.dev_ns;
                    C->st_host_ns += bt.host_ns;
                    C->cv.notify_all();
                }
            } release{C, lk, batch, B, bt};
            try {
                if (!B) B = new Bufs;
                run_batch(m, ctx, *B, batch, mode == MFP_MODE_WRITE_JSON, bt);
            } catch (const std::exception &e) {
                log_error("per-packet batch failed: %s\n", e.what());
                for (Req *x : batch) x->err = true;
            } catch (...) {
                log_error("per-packet batch failed\n");
                for (Req *x : batch) x->err = true;
            }
        } else {
            C->cv.wait(lk);
        }
    }
}

// write_json libmerc.cc:131-175 -> stateful_pkt_proc::write_json pkt_proc.cc:1256-1383: the record text
// from a one-packet batch (device walk, --analysis classification, mfp_write_json_batch[_analysis]).
// Returns 0 when nothing is written or the record does not fit buf_size (buffer_stream truncation,
// pkt_proc.cc:1249-1253).
MFP_EXPORT size_t mercury_packet_processor_write_json_linktype(mercury_packet_processor p, void *buffer,
                                                               size_t buffer_size, uint8_t *pkt, size_t len,
                                                               struct timespec *ts, uint16_t linktype) {
    if (!p || !buffer || !pkt || !ts) return 0;
    mfp_context ctx = get_ctx(p->mc, MFP_MODE_WRITE_JSON);
    if (!ctx) return 0;
    fill_zero_ts(ts);
    if (!mfp_reassembly_enabled(ctx)) {
        Req r{pkt, len, linktype, (uint64_t)ts->tv_sec * 1000000000ull + (uint64_t)ts->tv_nsec, &p->ac, buffer,
              buffer_size};
        submit(p->mc, ctx, MFP_MODE_WRITE_JSON, r);
        return r.err ? 0 : r.out_len;
    }
    p->arena.assign(pkt, pkt + len);
    p->arena.resize(len + 16);
    mfp_pkt_desc d{0, (uint32_t)len, linktype, 0};
    mfp_record rec;
    mfp_analysis an;
    double ap[MFP_ATTR_DB_TAGS] = {0, 0, 0, 0, 0, 0};
    size_t cap = mfp_fp_arena_bound(1, len);
    p->fp.resize(cap);
    const bool want_an = mfp_analysis_enabled(ctx);
    uint64_t t = (uint64_t)ts->tv_sec * 1000000000ull + (uint64_t)ts->tv_nsec, end = 0, skipped = 0;
    long long n;
    if (mfp_reassembly_enabled(ctx)) {
        // process_tcp_data with the processor's reassembler (pkt_proc.cc:773-893)
        if (!p->reasm) p->reasm = mfp_reassembler_create();
        cap += mfp_fp_arena_bound(1, 8192 + 256);
        p->fp.resize(cap);
        uint16_t props = 0;
        mfp_pkt_desc d2 = d;
        long long used = want_an ? mfp_process_batch_reassembly_analysis(ctx, p->reasm, p->arena.data(), p->arena.size(),
                                                                         &d, 1, &t, &rec, p->fp.data(), cap, &props, &d2,
                                                                         &an, ap)
                                 : mfp_process_batch_reassembly(ctx, p->reasm, p->arena.data(), p->arena.size(), &d, 1,
                                                                &t, &rec, p->fp.data(), cap, &props, &d2);
        if (used < 0) { log_error("%s\n", mfp_last_error()); return 0; }
        // the record indexes arena ++ the reassembler's frames
        size_t flen = 0;
        const uint8_t *fr = mfp_reassembler_frames(p->reasm, &flen);
        if (d2.offset >= len + 16 && fr) p->arena.insert(p->arena.end(), fr, fr + flen);
        fill_context(ctx, p->ac, p->arena.data() + d2.offset, d2.caplen, rec, p->fp.data(), want_an ? &an : nullptr, ap);
        note_other(p->mc, rec);
        n = want_an ? mfp_write_json_batch_reassembly_analysis(ctx, p->arena.data(), &d2, 1, &rec, p->fp.data(), &props,
                                                               &an, ap, &t, (char *)buffer, buffer_size, &end, &skipped, 1)
                    : mfp_write_json_batch_reassembly(p->arena.data(), &d2, 1, &rec, p->fp.data(), &props, &t,
                                                      (char *)buffer, buffer_size, &end, &skipped, 1);
    } else {
        long long used = mfp_process_batch_host_ex(ctx, p->arena.data(), p->arena.size(), &d, 1, &rec, p->fp.data(),
                                                   cap, want_an ? &an : nullptr, want_an ? ap : nullptr);
        if (used < 0) { log_error("%s\n", mfp_last_error()); return 0; }
        fill_context(ctx, p->ac, pkt, (uint32_t)len, rec, p->fp.data(), want_an ? &an : nullptr, ap);
        note_other(p->mc, rec);
        n = want_an ? mfp_write_json_batch_analysis(ctx, p->arena.data(), &d, 1, &rec, p->fp.data(), &an, ap, &t,
                                                    (char *)buffer, buffer_size, &end, &skipped, 1)
                    : mfp_write_json_batch(p->arena.data(), &d, 1, &rec, p->fp.data(), &t, (char *)buffer,
                                           buffer_size, &end, &skipped, 1);
    }
    if (skipped) {
        // the reference writes a record here; the writer could not rebuild it
        // (an encapsulation chain the host walk cannot follow): say so instead
        // of returning a silent 0
        log_error("write_json: record not rebuilt by the MI355X JSON writer (%s)\n",
                  rec.msg == MFP_MSG_QUIC ? "QUIC Initial" : rec.msg == MFP_MSG_STUN ? "STUN message"
                  : rec.msg == MFP_MSG_OPENVPN ? "OpenVPN record" : "encapsulation chain");
        return 0;
    }
    if (n <= 0 || (size_t)n >= buffer_size) return 0;    // buffer_stream keeps one byte for its NUL
    return (size_t)n;
}
MFP_EXPORT size_t mercury_packet_processor_write_json(mercury_packet_processor p, void *buffer, size_t buffer_size,
                                                      uint8_t *pkt, size_t len, struct timespec *ts) {
    return mercury_packet_processor_write_json_linktype(p, buffer, buffer_size, pkt, len, ts, 1);   // LINKTYPE_ETHERNET
}

static const analysis_context *analyze(mercury_packet_processor p, uint8_t *pkt, size_t len, struct timespec *ts,
                                      uint16_t linktype) {
    if (!p || !pkt) return nullptr;
    mfp_context ctx = get_ctx(p->mc, MFP_MODE_ANALYSIS);
    if (!ctx) return nullptr;
    fill_zero_ts(ts);
    if (!mfp_reassembly_enabled(ctx)) {
        Req r{pkt, len, linktype, ts ? (uint64_t)ts->tv_sec * 1000000000ull + (uint64_t)ts->tv_nsec : 0, &p->ac,
              nullptr, 0};
        submit(p->mc, ctx, MFP_MODE_ANALYSIS, r);
        return r.valid ? &p->ac : nullptr;
    }
    p->arena.assign(pkt, pkt + len);
    p->arena.resize(len + 16);
    mfp_pkt_desc d{0, (uint32_t)len, linktype, 0};
    mfp_record rec;
    mfp_analysis an;
    double ap[MFP_ATTR_DB_TAGS] = {0, 0, 0, 0, 0, 0};
    size_t cap = mfp_fp_arena_bound(1, len);
    p->fp.resize(cap);
    bool want_an = mfp_analysis_enabled(ctx);
    const uint8_t *base = pkt;
    uint32_t base_len = (uint32_t)len;
    if (mfp_reassembly_enabled(ctx)) {
        // analyze_ip_packet with the processor's reassembler (pkt_proc.cc:1597-1662):
        // the flow table in stream order, flow_state_pkts_needed per packet
        if (!p->reasm) p->reasm = mfp_reassembler_create();
        const uint64_t t = ts ? (uint64_t)ts->tv_sec * 1000000000ull + (uint64_t)ts->tv_nsec : 0;
        cap += mfp_fp_arena_bound(1, 8192 + 256);
        p->fp.resize(cap);
        uint16_t props = 0;
        uint8_t more = 0;
        mfp_pkt_desc d2 = d;
        const long long used = mfp_process_batch_reassembly_context(
            ctx, p->reasm, p->arena.data(), p->arena.size(), &d, 1, &t, &rec, p->fp.data(), cap, &props, &d2,
            want_an ? &an : nullptr, want_an ? ap : nullptr, &more);
        if (used < 0) { log_error("%s\n", mfp_last_error()); return nullptr; }
        p->more_pkts = more != 0;
        size_t flen = 0;
        const uint8_t *fr = mfp_reassembler_frames(p->reasm, &flen);
        if (d2.offset >= len + 16 && fr) p->arena.insert(p->arena.end(), fr, fr + flen);
        base = p->arena.data() + d2.offset;
        base_len = d2.caplen;
    } else {
        const long long used = mfp_process_batch_host_ex(ctx, p->arena.data(), p->arena.size(), &d, 1, &rec,
                                                         p->fp.data(), cap, want_an ? &an : nullptr,
                                                         want_an ? ap : nullptr);
        if (used < 0) { log_error("%s\n", mfp_last_error()); return nullptr; }
    }
    analysis_context &ac = p->ac;
    fill_context(ctx, ac, base, base_len, rec, p->fp.data(), want_an ? &an : nullptr, ap);
    note_other(p->mc, rec);
    if (!want_an) return nullptr;   // no classifier: analysis result never valid
    return (an.flags & MFP_AN_VALID) ? &ac : nullptr;
}

MFP_EXPORT const struct analysis_context *mercury_packet_processor_ip_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts) {
    return analyze(processor, packet, length, ts, 101);
}
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts) {
    return analyze(processor, packet, length, ts, 1);
}
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context_linktype(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts, uint16_t linktype) {
    return analyze(processor, packet, length, ts, linktype);
}

MFP_EXPORT enum fingerprint_status analysis_context_get_fingerprint_status(const struct analysis_context *ac) {
    return ac ? (enum fingerprint_status)ac->status : fingerprint_status_no_info_available;
}
MFP_EXPORT enum fingerprint_type analysis_context_get_fingerprint_type(const struct analysis_context *ac) {
    return ac ? (enum fingerprint_type)ac->fp_type : fingerprint_type_unknown;
}
MFP_EXPORT const char *analysis_context_get_fingerprint_string(const struct analysis_context *ac) {
    return ac ? ac->fp : nullptr;
}
// analysis_context::get_server_name / get_user_agent result.h:391-403: NULL
// when the string is empty
MFP_EXPORT const char *analysis_context_get_server_name(const struct analysis_context *ac) {
    return ac && ac->sn[0] ? ac->sn : nullptr;
}
MFP_EXPORT const char *analysis_context_get_user_agent(const struct analysis_context *ac) {
    return ac && ac->ua[0] ? ac->ua : nullptr;
}
// analysis_result::get_process_info result.h:268-276
MFP_EXPORT bool analysis_context_get_process_info(const struct analysis_context *ac, const char **probable_process,
                                                  double *probability_score) {
    if (!ac || !ac->has_process || ac->process.empty()) return false;
    if (probable_process) *probable_process = ac->process.c_str();
    if (probability_score) *probability_score = ac->score;
    return true;
}
// analysis_result::get_malware_info result.h:278-286
MFP_EXPORT bool analysis_context_get_malware_info(const struct analysis_context *ac,
                                                  bool *probable_process_is_malware, double *probability_malware) {
    if (!ac || !ac->classify_malware) return false;
    if (probable_process_is_malware) *probable_process_is_malware = ac->malware;
    if (probability_malware) *probability_malware = ac->malware_prob;
    return true;
}

// analysis_result::get_os_info result.h:290-299 (the array holds os_information {name, prevalence})
MFP_EXPORT bool analysis_context_get_os_info(const struct analysis_context *ac, const struct os_information **os_info,
                                             size_t *os_info_len) {
    if (!ac || ac->os.empty()) return false;
    if (os_info) *os_info = ac->os.data();
    if (os_info_len) *os_info_len = ac->os.size();
    return true;
}

// analysis_context::get_alpns result.h:401-408
MFP_EXPORT bool analysis_context_get_alpns(const struct analysis_context *ac, const uint8_t **alpn_data,
                                           size_t *alpn_length) {
    if (!ac || ac->alpn[0] == 0) return false;
    if (alpn_data) *alpn_data = ac->alpn;
    if (alpn_length) *alpn_length = ac->alpn_len;
    return true;
}

// mercury_packet_processor_get_attributes libmerc.cc:398-411 / attribute_result::get_attributes result.h:102-116
MFP_EXPORT const struct attribute_context *mercury_packet_processor_get_attributes(mercury_packet_processor p) {
    if (!p || p->ac.attr == 0 || p->ac.n_tags == 0) return nullptr;
    analysis_context &ac = p->ac;
    ac.actx.tag_names = ac.tag_names;
    ac.actx.prob_scores = ac.prob;
    ac.actx.attributes_len = ac.n_tags;
    return &ac.actx;
}

// mercury_get_classifier libmerc.cc:85-90: an opaque handle, NULL without a classifier
MFP_EXPORT void *mercury_get_classifier(mercury_context mc) {
    if (!mc || !mc->analysis) return nullptr;
    mfp_context c = get_ctx(mc, MFP_MODE_ANALYSIS);
    return c && mfp_analysis_enabled(c) ? (void *)c : nullptr;
}

// libmerc.cc:242-253: analysis_context::flow_state_pkts_needed of the
// processor's last get_analysis_context call (reassembly configured)
MFP_EXPORT bool mercury_packet_processor_more_pkts_needed(mercury_packet_processor p) {
    return p ? p->more_pkts : false;
}

MFP_EXPORT uint32_t mercury_get_version_number(void) { return mfp_reference_version(); }
// semantic_version::print_version_string version.h:34-36 (size - 1, as the reference)
MFP_EXPORT void mercury_get_version_string(char *buf, size_t size) {
    if (buf && size) snprintf(buf, size - 1, "%u.%u.%u", mfp_reference_version() >> 16,
                              (mfp_reference_version() >> 8) & 0xff, mfp_reference_version() & 0xff);
}
// mercury_print_version_string libmerc.cc:59-62 (semantic_version::print version.h:30-32)
MFP_EXPORT void mercury_print_version_string(FILE *f) {
    if (f) fprintf(f, "%u.%u.%u\n", mfp_reference_version() >> 16, (mfp_reference_version() >> 8) & 0xff,
                   mfp_reference_version() & 0xff);
}
// mercury_print_git_commit libmerc.cc:64-66: the commit this library was built from
MFP_EXPORT void mercury_print_git_commit(FILE *f) {
    if (f) fprintf(f, "%s\n", MFP_GIT_COMMIT);
}
// mercury_write_stats_data libmerc.cc:377-396: false without a stats
// aggregator (do_stats is refused at init, so there never is one)
MFP_EXPORT bool mercury_write_stats_data(mercury_context mc, const char *stats_data_file_path) {
    if (mc && stats_data_file_path) log_error("mercury_write_stats_data: stats are not provided by libmercury_amd\n");
    return false;
}
// get_stats_aggregator_num_entries libmerc.cc:477-484
MFP_EXPORT size_t get_stats_aggregator_num_entries(mercury_context) { return 0; }
// mercury_packet_processor_get_analysis_context_fdc libmerc.cc:199-216: the
// FDC/CBOR encoding is outside this path; the call fails as the reference's
// does on an internal error (fdc_return::UNKNOWN_ERROR), with a log line
MFP_EXPORT int mercury_packet_processor_get_analysis_context_fdc(mercury_packet_processor processor,
                                                                 const struct flow_key_ext *, const uint8_t *, size_t,
                                                                 uint8_t *, size_t *,
                                                                 const struct analysis_context **context) {
    if (!processor) return -5;   // fdc_return::INVALID_INPUT
    if (context) *context = nullptr;
    log_error("mercury_packet_processor_get_analysis_context_fdc: FDC output is not provided by libmercury_amd\n");
    return -4;                   // fdc_return::UNKNOWN_ERROR
}
// the MFP_MSG_OTHER packets counted by note_other
MFP_EXPORT uint64_t mercury_amd_other_packets(mercury_context mc) {
    return mc ? mc->other.load(std::memory_order_relaxed) : 0;
}
MFP_EXPORT const char *mercury_get_license_string(void) {
    return "libmercury_amd: MI355X fingerprint/classify path for the libmerc API";
}
// mercury_get_resource_version libmerc.cc:78-83: the archive's VERSION, NULL without a classifier
MFP_EXPORT const char *mercury_get_resource_version(mercury_context mc) {
    void *c = mercury_get_classifier(mc);
    return c ? mfp_resource_version((mfp_context)c) : nullptr;
}

}  // extern "C"
