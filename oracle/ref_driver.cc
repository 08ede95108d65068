// ref_driver.cc -- our own driver over the REFERENCE libmerc (compiled from
// /root/reference by oracle/Makefile.ref into oracle/_ref/merc_ref_drv).
// Test infrastructure only: it produces golden vectors and times the
// reference CPU path; nothing in mercury_amd/ links or calls it.
//
// Input: a classic pcap file, or our batch format (see tests/pcaplib.py:
// "MFPB" magic, n, then n x {u64 off,u32 caplen,u16 linktype,u16 flags},
// then the arena).
// Output (mode "fp"): one TSV line per packet:
//   idx  emit  fp_type  truncated  fp_string
// Output (mode "an"): analysis_context path, one TSV line per packet:
//   idx  valid  fp_type  status  process  score  malware  p_malware  fp_string
// Mode "anr": as "an", with mercury_packet_processor_more_pkts_needed after each
// packet in a column before the fingerprint:
//   idx  valid  fp_type  status  process  score  malware  p_malware  more  fp_string
// Mode "json": the write_json record text, one line per packet (empty line
// when the reference writes nothing).
// Mode "pcapw": the filtered pcap writer of `mercury -w` (pkt_proc_filter_pcap_writer[_llq],
// src/pkt_processing.h:92-121,230-259): each packet through the processor's
// Ethernet write_json (pkt_proc.cc:1258-1326, an LLQ_MAX_MSG_SIZE buffer, the
// packet's link type NOT passed, as there) and written in classic pcap format
// when a record was written or dump_pkt() is set (pkt_proc.cc:1842-1845), with
// the output file's header first (write_pcap_file_header pcap_file_io.c:88-104,
// pcap_queue_write :540-579).  The pcap bytes go to stdout.
// Modes "wjan" and "stat" run a TILED stream: MERC_TILE="u1:N" makes the
// stream packets [0, u1) once, then packets [u1, total) repeated until the
// stream holds N packets (bench.py's device batch is such a tiling of its unique
// packets).  Both use the write_json path with the classifier (the analysis
// result the record's "analysis" object prints, pkt_proc.cc:1195-1213).
//   "wjan": one TSV line per stream index listed in MERC_ROWS_FILE (sorted
//     little-endian u64):  idx  emit  fp_type  valid  status  process  score
//     malware  p_malware  fp_string
//   "stat": for the tiled part [u1, N), one bit per packet whose status is
//     randomized or unlabeled (an unknown-TLS sighting, analysis.h:1043-1083):
//     1 = unlabeled; packed MSB first (numpy.packbits) to stdout.
// Mode "meta": analysis_context path, one TSV line per packet:
//   idx  valid  server_name(hex)  user_agent(hex)   ("-" = NULL)
// Mode "attr": analysis_context path, the accessors the embedders read, one
// TSV line per packet:
//   idx  valid  status  attributes  os_info  alpn
// attributes: name=prob;... from mercury_packet_processor_get_attributes
// (prob %.17Lg, set tags only), os_info: name=prevalence;... from
// analysis_context_get_os_info, alpn: hex of analysis_context_get_alpns
// (first min(len, 128) bytes) and ":len".
// Environment: MERC_TS_FILE=<file of n little-endian u64 seconds> gives each
// packet its own timestamp (default 1700000000 for all); MERC_REPORT_OS=1 sets libmerc_config.report_os; MERC_ENC_KEY=<32
// hex digits> sets libmerc_config.enc_key (an encrypted resource archive).
// Mode "time": run write_json (or, with a trailing "an", the analysis_context
// entry) with T threads (one processor per thread over contiguous shards),
// print packets/s.
// Mode "lpm" (lpm <pyasn.db> <domain mappings> <queries>): the reference's
// subnet_data LC-tries queried directly (see lpm_mode).
//
// Uses the reference's public C API (libmerc.h:211-736) plus the processor's
// analysis context (pkt_proc.h:132), exactly as the reference's own unit-test
// fixture does (unit_tests/libmerc_fixture.cc:138).

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <thread>
#include <chrono>
#include <fcntl.h>
#include <unistd.h>
#include "libmerc.h"
#include "pkt_proc.h"
#include "addr.h"

struct pkt { const uint8_t *data; uint32_t len; uint16_t linktype; };

static std::vector<uint8_t> slurp(const char *fn) {
    std::vector<uint8_t> v;
    FILE *f = fopen(fn, "rb");
    if (!f) { perror(fn); exit(1); }
    fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    v.resize(n);
    if (n && fread(v.data(), 1, n, f) != (size_t)n) { perror("fread"); exit(1); }
    fclose(f);
    return v;
}

static std::vector<pkt> load(const std::vector<uint8_t> &buf) {
    std::vector<pkt> out;
    if (buf.size() >= 4 && memcmp(buf.data(), "MFPB", 4) == 0) {
        uint64_t n; memcpy(&n, buf.data() + 8, 8);
        const uint8_t *d = buf.data() + 16;
        const uint8_t *arena = d + n * 16;
        for (uint64_t i = 0; i < n; i++) {
            uint64_t off; uint32_t cl; uint16_t lt;
            memcpy(&off, d + 16 * i, 8); memcpy(&cl, d + 16 * i + 8, 4); memcpy(&lt, d + 16 * i + 12, 2);
            out.push_back({arena + off, cl, lt});
        }
        return out;
    }
    // classic pcap
    if (buf.size() < 24) { fprintf(stderr, "short pcap\n"); exit(1); }
    uint32_t magic; memcpy(&magic, buf.data(), 4);
    bool swap = (magic == 0xd4c3b2a1 || magic == 0x4d3cb2a1);
    auto rd32 = [&](const uint8_t *p) { uint32_t x; memcpy(&x, p, 4); return swap ? __builtin_bswap32(x) : x; };
    uint16_t lt = (uint16_t)rd32(buf.data() + 20);
    size_t o = 24;
    while (o + 16 <= buf.size()) {
        uint32_t incl = rd32(buf.data() + o + 8);
        o += 16;
        if (o + incl > buf.size()) break;
        out.push_back({buf.data() + o, incl, lt});
        o += incl;
    }
    return out;
}

static int quiet(enum log_level, const char *, va_list) { return 0; }

// mode "sni": server_identifier normalisation (watchlist.hpp:326-390) of
// each line of <input>, one output line each: <name>\t<normalized>
static int sni_mode(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); return 1; }
    char line[4096];
    while (fgets(line, sizeof line, f)) {
        size_t n = strlen(line);
        if (n && line[n - 1] == '\n') line[--n] = 0;
        server_identifier si{std::string(line, n)};
        printf("%s\t%s\n", line, si.get_normalized_domain_name(server_identifier::detail::on).c_str());
    }
    fclose(f);
    return 0;
}

// mode "lpm": the reference's subnet_data (addr.cc) built from a pyasn.db
// text file and a domain-mapping file (one "subnet<TAB>tag" line per entry,
// the pairs classifier::process_domain_mapping_line analysis.h:765-819 makes:
// the tag is the type for proxy/sinkhole), finalised as the classifier does
// (analysis.h:961-964); then for each query line "dst_ip<TAB>server_name":
//   dst_ip  server_name  get_asn_info(dst_ip)  is_domain_faking(server_name, dst_ip)
static std::vector<std::string> lines_of(const char *path) {
    std::vector<std::string> out;
    if (!path || strcmp(path, "-") == 0) return out;
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    char line[8192];
    while (fgets(line, sizeof line, f)) {
        size_t n = strlen(line);
        if (n && line[n - 1] == '\n') line[--n] = 0;
        out.emplace_back(line, n);
    }
    fclose(f);
    return out;
}

static int lpm_mode(const char *asn_path, const char *dom_path, const char *q_path) {
    fflush(stdout);
    int saved = dup(1), devnull = open("/dev/null", O_WRONLY);   // subnet_dedup prints
    if (devnull >= 0) dup2(devnull, 1);
    subnet_data sd;
    {
        std::vector<std::string> v4, v6;   // the split of analysis.h:896-905
        for (auto &l : lines_of(asn_path)) (l.find('.') != std::string::npos ? v4 : v6).push_back(l);
        sd.process_asn_subnets(v4);
        sd.process_asn_subnets_v6(v6);
        std::vector<std::pair<std::string, std::string>> d4, d6;
        for (auto &l : lines_of(dom_path)) {
            size_t t = l.find('\t');
            if (t == std::string::npos) continue;
            std::string sub = l.substr(0, t), tag = l.substr(t + 1);
            (sub.find('.') != std::string::npos ? d4 : d6).push_back({sub, tag});
        }
        sd.process_domain_mapping_subnets(d4);
        sd.process_domain_mapping_subnets_v6(d6);
        sd.process_final();
        sd.process_final_v6();
        sd.process_domain_mappings_final();
        sd.process_domain_mappings_final_v6();
    }
    fflush(stdout);
    if (saved >= 0) { dup2(saved, 1); close(saved); }
    if (devnull >= 0) close(devnull);
    for (auto &q : lines_of(q_path)) {
        size_t t = q.find('\t');
        std::string ip = t == std::string::npos ? q : q.substr(0, t);
        std::string name = t == std::string::npos ? "" : q.substr(t + 1);
        const uint32_t asn = sd.get_asn_info(ip.c_str());
        const int fake = name.empty() ? 0 : (int)sd.is_domain_faking(name.c_str(), ip.c_str());
        printf("%s\t%s\t%u\t%d\n", ip.c_str(), name.c_str(), asn, fake);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 3 && std::string(argv[1]) == "sni") return sni_mode(argv[2]);
    if (argc == 5 && std::string(argv[1]) == "lpm") return lpm_mode(argv[2], argv[3], argv[4]);
    if (argc < 4) {
        fprintf(stderr, "usage: %s fp|an|json|time <input> <config-string> [resources] [threads] [seconds] [json|an]\n", argv[0]);
        return 2;
    }
    std::string mode = argv[1];
    auto buf = slurp(argv[2]);
    auto pkts = load(buf);
    register_printf_err_callback(quiet);

    libmerc_config cfg{};
    std::string filt = argv[3];
    cfg.packet_filter_cfg = (char *)filt.c_str();
    std::string res;
    if (argc > 4 && strlen(argv[4]) > 0 && strcmp(argv[4], "-") != 0) {
        res = argv[4];
        cfg.resources = (char *)res.c_str();
        cfg.do_analysis = true;
    }
    static uint8_t key[16];
    const char *ek = getenv("MERC_ENC_KEY");
    if (ek && strlen(ek) == 32) {
        for (int k = 0; k < 16; k++) { unsigned v = 0; sscanf(ek + 2 * k, "%2x", &v); key[k] = (uint8_t)v; }
        cfg.enc_key = key;
        cfg.key_type = enc_key_type_aes_128;
    }
    const char *ros = getenv("MERC_REPORT_OS");
    cfg.report_os = ros && ros[0] == '1';
    // lctrie's subnet_dedup prints to stdout while the archive loads
    // (lctrie_ip.hpp:399-410): keep that out of the record stream
    fflush(stdout);
    int saved = dup(1), devnull = open("/dev/null", O_WRONLY);
    if (devnull >= 0) dup2(devnull, 1);
    mercury_context mc = mercury_init(&cfg, 0);
    fflush(stdout);
    if (saved >= 0) { dup2(saved, 1); close(saved); }
    if (devnull >= 0) close(devnull);
    if (!mc) { fprintf(stderr, "mercury_init failed\n"); return 1; }

    std::vector<uint64_t> tsv(pkts.size(), 1700000000ull);
    if (const char *tf = getenv("MERC_TS_FILE")) {
        auto tb = slurp(tf);
        for (size_t i = 0; i < pkts.size() && 8 * i + 8 <= tb.size(); i++) memcpy(&tsv[i], tb.data() + 8 * i, 8);
    }
    std::vector<char> out(1 << 16);
    // the stream order of the tiled modes
    size_t tile_u1 = 0, tile_n = pkts.size();
    if (const char *t = getenv("MERC_TILE")) {
        unsigned long long a = 0, b = 0;
        if (sscanf(t, "%llu:%llu", &a, &b) != 2 || a > pkts.size() || (b > a && a == pkts.size())) {
            fprintf(stderr, "bad MERC_TILE\n");
            return 2;
        }
        tile_u1 = a; tile_n = b;
    }
    auto stream_pkt = [&](size_t i) -> const pkt & {
        if (i < tile_u1) return pkts[i];
        return pkts[tile_u1 + (i - tile_u1) % (pkts.size() - tile_u1)];
    };
    if (mode == "wjan" || mode == "stat") {
        std::vector<uint64_t> rows;
        if (const char *rf = getenv("MERC_ROWS_FILE")) {
            auto rb = slurp(rf);
            rows.resize(rb.size() / 8);
            memcpy(rows.data(), rb.data(), rows.size() * 8);
        }
        size_t next_row = 0;
        std::vector<uint8_t> bits;
        uint8_t acc = 0;
        int nb = 0;
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < tile_n; i++) {
            const pkt &k = stream_pkt(i);
            struct timespec ts{(time_t)1700000000, 0};
            const size_t n = mercury_packet_processor_write_json_linktype(p, out.data(), out.size(), (uint8_t *)k.data,
                                                                         k.len, &ts, k.linktype);
            const bool valid = n > 0 && p->analysis.result.is_valid();
            const analysis_context *ac = valid ? &p->analysis : nullptr;
            const int status = ac ? (int)analysis_context_get_fingerprint_status(ac) : 0;
            if (mode == "stat") {
                if (i >= tile_u1 && (status == 2 || status == 3)) {
                    acc = (uint8_t)(acc << 1 | (status == 3));
                    if (++nb == 8) { bits.push_back(acc); acc = 0; nb = 0; }
                }
                continue;
            }
            if (next_row >= rows.size() || rows[next_row] != i) continue;
            next_row++;
            const int t = n > 0 ? p->analysis.fp.get_type() : 0;
            const char *proc = ""; double score = 0; bool mal = false; double pm = 0;
            if (ac) {
                analysis_context_get_process_info(ac, &proc, &score);
                analysis_context_get_malware_info(ac, &mal, &pm);
            }
            printf("%zu\t%d\t%d\t%d\t%d\t%s\t%.17g\t%d\t%.17g\t%s\n", i, n > 0, t, (int)valid, status,
                   proc ? proc : "", score, (int)mal, pm, t ? p->analysis.fp.string() : "");
        }
        if (mode == "stat") {
            fprintf(stderr, "sightings %zu\n", bits.size() * 8 + nb);
            if (nb) bits.push_back((uint8_t)(acc << (8 - nb)));
            fwrite(bits.data(), 1, bits.size(), stdout);
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "fp") {
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            size_t n = mercury_packet_processor_write_json_linktype(p, out.data(), out.size(),
                                                                   (uint8_t *)pkts[i].data, pkts[i].len, &ts, pkts[i].linktype);
            std::string json(out.data(), n);
            bool trunc = json.find("\"reassembly_properties\":{\"truncated\":true}") != std::string::npos;
            // the processor's fingerprint is only (re)computed for packets that
            // reach ip_write_json and emit a record (pkt_proc.cc:1157-1158)
            int t = n > 0 ? p->analysis.fp.get_type() : 0;
            printf("%zu\t%d\t%d\t%d\t%s\n", i, n > 0, t, (int)trunc, t ? p->analysis.fp.string() : "");
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "json") {
        // the reference's JSON record text, one line per packet ("" when none)
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            size_t n = mercury_packet_processor_write_json_linktype(p, out.data(), out.size(),
                                                                   (uint8_t *)pkts[i].data, pkts[i].len, &ts, pkts[i].linktype);
            fwrite(out.data(), 1, n, stdout);
            if (n == 0 || out[n - 1] != '\n') fputc('\n', stdout);
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "pcapw") {
        // the pcap structs as pcap_file_io.c:41-61 lays them out (little-endian
        // host, never byte-swapped when writing)
        auto put32 = [](uint8_t *d, uint32_t v) { memcpy(d, &v, 4); };
        auto put16 = [](uint8_t *d, uint16_t v) { memcpy(d, &v, 2); };
        uint8_t fh[24];
        put32(fh, 0xa1b2c3d4u); put16(fh + 4, 2); put16(fh + 6, 4); put32(fh + 8, 0); put32(fh + 12, 0);
        put32(fh + 16, 65535); put32(fh + 20, 1);                     // snaplen 65535, LINKTYPE_ETHERNET
        fwrite(fh, 1, sizeof fh, stdout);
        std::vector<uint8_t> big(1 << 20);                            // LLQ_MAX_MSG_SIZE (llq.h:17)
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            const size_t n = p->write_json(big.data(), big.size(), (uint8_t *)pkts[i].data, pkts[i].len, &ts);
            if (n == 0 && !p->dump_pkt()) continue;
            // (the _llq form `mercury -w` builds, pkt_processing.cc:35-38: an empty
            // packet still gets its 16-byte header, pcap_queue_write :555-569)
            uint8_t ph[16];
            put32(ph, (uint32_t)ts.tv_sec); put32(ph + 4, (uint32_t)(ts.tv_nsec / 1000));
            put32(ph + 8, pkts[i].len); put32(ph + 12, pkts[i].len);
            fwrite(ph, 1, sizeof ph, stdout);
            fwrite(pkts[i].data, 1, pkts[i].len, stdout);
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "an" || mode == "anr") {
        const bool more = mode == "anr";
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            const analysis_context *ac = mercury_packet_processor_get_analysis_context_linktype(
                p, (uint8_t *)pkts[i].data, pkts[i].len, &ts, pkts[i].linktype);
            const char *mp = more ? (mercury_packet_processor_more_pkts_needed(p) ? "1\t" : "0\t") : "";
            if (!ac) {
                int t = p->analysis.fp.get_type();
                printf("%zu\t0\t%d\t0\t\t0\t0\t0\t%s%s\n", i, t, mp, t ? p->analysis.fp.string() : "");
                continue;
            }
            const char *proc = ""; double score = 0; bool mal = false; double pm = 0;
            analysis_context_get_process_info(ac, &proc, &score);
            analysis_context_get_malware_info(ac, &mal, &pm);
            printf("%zu\t1\t%d\t%d\t%s\t%.17g\t%d\t%.17g\t%s%s\n", i,
                   (int)analysis_context_get_fingerprint_type(ac),
                   (int)analysis_context_get_fingerprint_status(ac),
                   proc ? proc : "", score, (int)mal, pm, mp,
                   analysis_context_get_fingerprint_string(ac));
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "meta") {
        // analysis_context path: the destination context's strings the
        // embedders read (libmerc.cc:276-288), hex; "-" when NULL
        //   idx  valid  server_name  user_agent
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        auto hex = [](const char *s) {
            if (!s) return std::string("-");
            std::string h;
            char t[3];
            for (const char *c = s; *c; c++) { snprintf(t, sizeof t, "%02x", (unsigned)(uint8_t)*c); h += t; }
            return h;
        };
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            const analysis_context *ac = mercury_packet_processor_get_analysis_context_linktype(
                p, (uint8_t *)pkts[i].data, pkts[i].len, &ts, pkts[i].linktype);
            if (!ac) { printf("%zu\t0\t-\t-\n", i); continue; }
            printf("%zu\t1\t%s\t%s\n", i, hex(analysis_context_get_server_name(ac)).c_str(),
                   hex(analysis_context_get_user_agent(ac)).c_str());
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "attr") {
        mercury_packet_processor p = mercury_packet_processor_construct(mc);
        for (size_t i = 0; i < pkts.size(); i++) {
            struct timespec ts{(time_t)tsv[i], 0};
            const analysis_context *ac = mercury_packet_processor_get_analysis_context_linktype(
                p, (uint8_t *)pkts[i].data, pkts[i].len, &ts, pkts[i].linktype);
            std::string attrs, os, alpn;
            const attribute_context *at = mercury_packet_processor_get_attributes(p);
            if (at) {
                for (size_t k = 0; k < at->attributes_len; k++) {
                    if (at->prob_scores[k] == 0) continue;
                    char t[96];
                    snprintf(t, sizeof t, "=%.17Lg;", at->prob_scores[k]);
                    attrs += std::string(at->tag_names[k]) + t;
                }
            }
            if (ac) {
                const os_information *oi = nullptr;
                size_t ol = 0;
                if (analysis_context_get_os_info(ac, &oi, &ol))
                    for (size_t k = 0; k < ol; k++) os += std::string(oi[k].os_name) + "=" + std::to_string(oi[k].os_prevalence) + ";";
                const uint8_t *ad = nullptr;
                size_t al = 0;
                if (analysis_context_get_alpns(ac, &ad, &al)) {
                    char h[3];
                    for (size_t k = 0; k < al && k < 128; k++) { snprintf(h, sizeof h, "%02x", ad[k]); alpn += h; }
                    alpn += ":" + std::to_string(al);
                }
            }
            printf("%zu\t%d\t%d\t%s\t%s\t%s\n", i, ac != nullptr, ac ? (int)analysis_context_get_fingerprint_status(ac) : 0,
                   attrs.c_str(), os.c_str(), alpn.c_str());
        }
        mercury_packet_processor_destruct(p);
    } else if (mode == "time") {
        int threads = argc > 5 ? atoi(argv[5]) : 1;
        double secs = argc > 6 ? atof(argv[6]) : 10.0;
        // entry point timed: "json" = write_json_linktype (the CLI's path),
        // "an" = get_analysis_context_linktype (the embedders' path)
        const bool an_entry = argc > 7 && std::string(argv[7]) == "an";
        std::vector<std::thread> th;
        std::vector<unsigned long long> counts(threads, 0);
        auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < threads; t++) {
            th.emplace_back([&, t]() {
                mercury_packet_processor p = mercury_packet_processor_construct(mc);
                std::vector<char> o(1 << 16);
                size_t lo = pkts.size() * t / threads, hi = pkts.size() * (t + 1) / threads;
                unsigned long long c = 0;
                auto start = std::chrono::steady_clock::now();
                do {
                    for (size_t i = lo; i < hi; i++) {
                        struct timespec ts{(time_t)tsv[i], 0};
                        if (an_entry)
                            mercury_packet_processor_get_analysis_context_linktype(p, (uint8_t *)pkts[i].data,
                                                                                   pkts[i].len, &ts, pkts[i].linktype);
                        else
                            mercury_packet_processor_write_json_linktype(p, o.data(), o.size(), (uint8_t *)pkts[i].data,
                                                                         pkts[i].len, &ts, pkts[i].linktype);
                    }
                    c += hi - lo;
                } while (std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count() < secs);
                counts[t] = c;
                mercury_packet_processor_destruct(p);
            });
        }
        for (auto &x : th) x.join();
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        unsigned long long tot = 0; for (auto c : counts) tot += c;
        printf("{\"threads\": %d, \"packets\": %llu, \"seconds\": %.6f, \"pps\": %.1f}\n", threads, tot, el, tot / el);
    }
    mercury_finalize(mc);
    return 0;
}
