/*
 * libmerc_link.c -- calls every function the reference's public header
 * declares (/root/reference/src/libmerc/libmerc.h; the list is
 * tests/golden/libmerc_h_symbols.txt), compiled against
 * include/mercury_amd_libmerc.h and linked against libmercury_amd.so with no
 * other library.  tests/test_abi.py builds and runs it on the CPU: the
 * calls that need the GPU (a packet through a processor) return 0 / NULL and
 * log through the printf_err callback; the rest print what they return.
 *
 *   gcc -std=gnu11 -Iinclude tests/c/libmerc_link.c -Lmercury_amd -lmercury_amd \
 *       -Wl,-rpath,$PWD/mercury_amd -o tests/c/libmerc_link
 */
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "mercury_amd_libmerc.h"

static int logged = 0;
static int log_cb(enum log_level level, const char *fmt, va_list ap) {
    (void)level; (void)fmt; (void)ap;
    return ++logged;
}

int main(int argc, char **argv) {
    const char *resources = argc > 1 ? argv[1] : NULL;
    register_printf_err_callback(log_cb);
    printf("version_number %u\n", mercury_get_version_number());
    char vs[32];
    mercury_get_version_string(vs, sizeof vs);
    printf("version_string %s\n", vs);
    printf("print_version ");
    mercury_print_version_string(stdout);
    printf("git_commit ");
    mercury_print_git_commit(stdout);
    printf("license %d\n", mercury_get_license_string() != NULL);

    struct libmerc_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.packet_filter_cfg = (char *)"select=tls,ssh,http;reassembly";
    cfg.do_stats = true;
    printf("init_with_stats %d\n", mercury_init(&cfg, 0) != NULL);   /* refused */
    cfg.do_stats = false;
    if (resources) { cfg.resources = (char *)resources; cfg.do_analysis = true; }
    mercury_context mc = mercury_init(&cfg, 0);
    printf("init %d\n", mc != NULL);
    if (!mc) return 1;
    printf("write_stats %d\n", (int)mercury_write_stats_data(mc, "/dev/null"));
    printf("stats_entries %zu\n", get_stats_aggregator_num_entries(mc));
    const char *rv = mercury_get_resource_version(mc);
    printf("resource_version %s\n", rv ? "set" : "none");
    printf("classifier %d\n", mercury_get_classifier(mc) != NULL);

    mercury_packet_processor p = mercury_packet_processor_construct(mc);
    printf("processor %d\n", p != NULL);
    uint8_t pkt[64] = {0};
    char buf[4096];
    struct timespec ts = {1700000000, 0};
    size_t n = mercury_packet_processor_write_json(p, buf, sizeof buf, pkt, sizeof pkt - 16, &ts);
    n += mercury_packet_processor_write_json_linktype(p, buf, sizeof buf, pkt, sizeof pkt - 16, &ts, 1);
    printf("write_json %zu\n", n);
    const struct analysis_context *ac[3];
    ac[0] = mercury_packet_processor_get_analysis_context(p, pkt, sizeof pkt - 16, &ts);
    ac[1] = mercury_packet_processor_get_analysis_context_linktype(p, pkt, sizeof pkt - 16, &ts, 1);
    ac[2] = mercury_packet_processor_ip_get_analysis_context(p, pkt, sizeof pkt - 16, &ts);
    printf("analysis_context %d %d %d\n", ac[0] != NULL, ac[1] != NULL, ac[2] != NULL);
    printf("more_pkts_needed %d\n", (int)mercury_packet_processor_more_pkts_needed(p));
    printf("attributes %d\n", mercury_packet_processor_get_attributes(p) != NULL);
    /* the accessors on a NULL context (libmerc.cc: every accessor checks ac) */
    const struct analysis_context *none = NULL;
    const char *proc = NULL; double score = 0; bool mal = false; double pm = 0;
    const struct os_information *os = NULL; size_t osn = 0;
    const uint8_t *alpn = NULL; size_t alpn_len = 0;
    printf("accessors %d %d %d %d %d %d %d %d %d\n",
           (int)analysis_context_get_fingerprint_status(none), (int)analysis_context_get_fingerprint_type(none),
           analysis_context_get_fingerprint_string(none) != NULL, analysis_context_get_server_name(none) != NULL,
           analysis_context_get_user_agent(none) != NULL,
           (int)analysis_context_get_process_info(none, &proc, &score),
           (int)analysis_context_get_malware_info(none, &mal, &pm),
           (int)analysis_context_get_os_info(none, &os, &osn),
           (int)analysis_context_get_alpns(none, &alpn, &alpn_len));
    struct flow_key_ext k;
    memset(&k, 0, sizeof k);
    size_t fdc_size = sizeof buf;
    const struct analysis_context *fac = NULL;
    printf("fdc %d\n", mercury_packet_processor_get_analysis_context_fdc(p, &k, pkt, 16, (uint8_t *)buf, &fdc_size, &fac));
    mercury_packet_processor_destruct(p);
    printf("finalize %d\n", mercury_finalize(mc));
    register_printf_err_callback(NULL);
    printf("logged %d\n", logged > 0);
    return 0;
}
