// mfp_libmerc.cpp -- the reference's per-packet libmerc C API
// (include/mercury_amd_libmerc.h) over the batch path of include/mfp.h.
// Every call is a one-packet batch on the GPU; the high-throughput
// interface is the batch API.  File:line cites are relative to
// /root/reference/src/libmerc/.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mercury_amd_libmerc.h"
#include "../../include/mfp.h"
#include "mfp_internal.h"

struct mercury {
    std::string cfg;              // packet_filter_cfg as mfp_init takes it
    std::string resource_version;
    bool analysis = false;
    std::mutex mu;
    mfp_context ctx[2] = {nullptr, nullptr};   // per reference entry point (write_json / analysis)
};

struct analysis_context {       // the fields libmerc's accessors read (result.h:383-420)
    char fp[8193];
    uint32_t fp_type = 0;
    uint32_t status = 0;
    char sn[257];               // destination_context::sn_str (MAX_SNI_LEN)
    char ua[512];               // destination_context::ua_str (MAX_USER_AGENT_LEN)
    std::string process;
    double score = 0, malware_prob = -1;
    bool malware = false, classify_malware = false, has_process = false;
};

struct mercury_packet_processor_s {
    mercury *mc;
    analysis_context ac;
    std::vector<uint8_t> arena;
    std::vector<char> fp;
};

static printf_err_ptr g_printf_err = nullptr;

static void log_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    if (g_printf_err) g_printf_err(log_err, fmt, ap);
    va_end(ap);
}

extern "C" {

MFP_EXPORT void register_printf_err_callback(printf_err_ptr callback) { g_printf_err = callback; }

// mercury_init libmerc.cc:92-128 / struct mercury pkt_proc.h:56-114
MFP_EXPORT mercury_context mercury_init(const struct libmerc_config *vars, int verbosity) {
    (void)verbosity;
    if (!vars) return nullptr;
    if (vars->enc_key || vars->key_type != enc_key_type_none) {
        log_error("encrypted resource archives are not supported by the MI355X path\n");
        return nullptr;
    }
    auto *m = new mercury;
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
    if (mfp_parse_filter(cfg.c_str(), &sel, &fmt) != 0) {
        log_error("%s\n", mfp_last_error());
        delete m;
        return nullptr;
    }
    return m;
}

MFP_EXPORT int mercury_finalize(mercury_context mc) {
    if (!mc) return -1;
    for (auto &c : mc->ctx) if (c) mfp_finalize(c);
    delete mc;
    return 0;
}

static mfp_context get_ctx(mercury *m, int mode) {
    std::lock_guard<std::mutex> lk(m->mu);
    if (!m->ctx[mode]) {
        m->ctx[mode] = mfp_init(m->cfg.c_str(), 0, mode);
        if (!m->ctx[mode]) log_error("%s\n", mfp_last_error());
    }
    return m->ctx[mode];
}

MFP_EXPORT mercury_packet_processor mercury_packet_processor_construct(mercury_context mc) {
    if (!mc) return nullptr;
    auto *p = new mercury_packet_processor_s;
    p->mc = mc;
    return p;
}

MFP_EXPORT void mercury_packet_processor_destruct(mercury_packet_processor mpp) { delete mpp; }

// write_json libmerc.cc:131-175 -> stateful_pkt_proc::write_json pkt_proc.cc:1256-1383: the record text
// from a one-packet batch (device walk + mfp_write_json_batch).  Returns 0 when nothing is written, the
// record does not fit buf_size (buffer_stream truncation, pkt_proc.cc:1249-1253), or --analysis is
// configured (the "analysis" object is not built by the JSON writer yet).
MFP_EXPORT size_t mercury_packet_processor_write_json_linktype(mercury_packet_processor p, void *buffer,
                                                               size_t buffer_size, uint8_t *pkt, size_t len,
                                                               struct timespec *ts, uint16_t linktype) {
    if (!p || !buffer || !pkt || !ts) return 0;
    if (p->mc->analysis) return 0;
    mfp_context ctx = get_ctx(p->mc, MFP_MODE_WRITE_JSON);
    if (!ctx) return 0;
    if (ts->tv_sec == 0) clock_gettime(CLOCK_REALTIME, ts);   // pkt_proc.cc:1086-1089
    p->arena.assign(pkt, pkt + len);
    p->arena.resize(len + 16);
    mfp_pkt_desc d{0, (uint32_t)len, linktype, 0};
    mfp_record rec;
    size_t cap = mfp_fp_arena_bound(1, len);
    p->fp.resize(cap);
    long long used = mfp_process_batch_host(ctx, p->arena.data(), p->arena.size(), &d, 1, &rec, p->fp.data(), cap);
    if (used < 0) { log_error("%s\n", mfp_last_error()); return 0; }
    uint64_t t = (uint64_t)ts->tv_sec * 1000000000ull + (uint64_t)ts->tv_nsec, end = 0, skipped = 0;
    long long n = mfp_write_json_batch(p->arena.data(), &d, 1, &rec, p->fp.data(), &t, (char *)buffer,
                                       buffer_size, &end, &skipped, 1);
    if (skipped) {
        // the reference writes a record here; the writer cannot rebuild it
        // (IP-in-IP with an outer IPv6 extension header): say so instead of
        // returning a silent 0
        log_error("write_json: record not rebuilt (IP-in-IP, outer IPv6 header with extension headers)\n");
        return 0;
    }
    if (n <= 0 || (size_t)n >= buffer_size) return 0;    // buffer_stream keeps one byte for its NUL
    return (size_t)n;
}
MFP_EXPORT size_t mercury_packet_processor_write_json(mercury_packet_processor p, void *buffer, size_t buffer_size,
                                                      uint8_t *pkt, size_t len, struct timespec *ts) {
    return mercury_packet_processor_write_json_linktype(p, buffer, buffer_size, pkt, len, ts, 1);   // LINKTYPE_ETHERNET
}

static void copy_cstr(char *dst, size_t cap, const uint8_t *src, size_t len) {   // datum::strncpy
    size_t n = len < cap - 1 ? len : cap - 1;
    size_t k = 0;
    for (; k < n && src[k]; k++) dst[k] = (char)src[k];
    dst[k] = 0;
}

static const analysis_context *analyze(mercury_packet_processor p, uint8_t *pkt, size_t len, uint16_t linktype) {
    if (!p || !pkt) return nullptr;
    mfp_context ctx = get_ctx(p->mc, MFP_MODE_ANALYSIS);
    if (!ctx) return nullptr;
    p->arena.assign(pkt, pkt + len);
    p->arena.resize(len + 16);
    mfp_pkt_desc d{0, (uint32_t)len, linktype, 0};
    mfp_record rec;
    mfp_analysis an;
    size_t cap = mfp_fp_arena_bound(1, len);
    p->fp.resize(cap);
    bool want_an = mfp_analysis_enabled(ctx);
    long long used = mfp_process_batch_host_ex(ctx, p->arena.data(), p->arena.size(), &d, 1, &rec, p->fp.data(), cap,
                                               want_an ? &an : nullptr);
    if (used < 0) { log_error("%s\n", mfp_last_error()); return nullptr; }
    analysis_context &ac = p->ac;
    ac.fp_type = rec.fp_type;
    copy_cstr(ac.fp, sizeof ac.fp, (const uint8_t *)p->fp.data() + rec.fp_offset, rec.fp_type ? rec.fp_len : 0);
    bool cert_slot = rec.msg == MFP_MSG_TLS_SH || rec.msg == MFP_MSG_TLS_CERT;   // sni slot = certificate_list
    copy_cstr(ac.sn, sizeof ac.sn, pkt + rec.sni_off, rec.sni_len == 0xffff || cert_slot ? 0 : rec.sni_len);
    copy_cstr(ac.ua, sizeof ac.ua, pkt + rec.ua_off, rec.ua_len == 0xffff ? 0 : rec.ua_len);
    if (!want_an) return nullptr;   // no classifier: analysis result never valid
    ac.status = an.status;
    ac.has_process = an.process != MFP_NO_PROCESS;
    ac.process = ac.has_process ? mfp_process_name(ctx, an.process) : "";
    ac.score = an.score;
    ac.malware = an.flags & MFP_AN_MALWARE;
    ac.classify_malware = an.flags & MFP_AN_CLASSIFY_MALWARE;
    ac.malware_prob = an.malware_prob;
    return (an.flags & MFP_AN_VALID) ? &ac : nullptr;
}

MFP_EXPORT const struct analysis_context *mercury_packet_processor_ip_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *) {
    return analyze(processor, packet, length, 101);
}
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *) {
    return analyze(processor, packet, length, 1);
}
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context_linktype(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *, uint16_t linktype) {
    return analyze(processor, packet, length, linktype);
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
MFP_EXPORT const char *analysis_context_get_server_name(const struct analysis_context *ac) {
    return ac ? ac->sn : nullptr;
}
MFP_EXPORT const char *analysis_context_get_user_agent(const struct analysis_context *ac) {
    return ac ? ac->ua : nullptr;
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

MFP_EXPORT bool mercury_packet_processor_more_pkts_needed(mercury_packet_processor) { return false; }

MFP_EXPORT uint32_t mercury_get_version_number(void) { return mfp_reference_version(); }
MFP_EXPORT void mercury_get_version_string(char *buf, size_t size) {
    if (buf && size) snprintf(buf, size, "%u.%u.%u", mfp_reference_version() >> 16, (mfp_reference_version() >> 8) & 0xff,
                              mfp_reference_version() & 0xff);
}
MFP_EXPORT const char *mercury_get_license_string(void) {
    return "libmercury_amd: MI355X fingerprint/classify path for the libmerc API";
}
MFP_EXPORT const char *mercury_get_resource_version(mercury_context mc) {
    return mc ? mc->resource_version.c_str() : nullptr;
}

}  // extern "C"
