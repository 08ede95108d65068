/*
 * mercury_amd_libmerc.h -- the reference's per-packet C API (libmerc.h of
 * cisco/mercury 2.18.0), exported by libmercury_amd.so so that an existing
 * embedder links unchanged.  Every entry point below replaces the
 * declaration cited next to it (paths relative to /root/reference/src/libmerc/).
 *
 * Each per-packet call is a one-packet batch through the MI355X path (the
 * batch API of include/mfp.h is the high-throughput interface; the per-packet
 * shims exist for drop-in compatibility and parity tests).  Semantics kept:
 *   - a processor is not reentrant; one per thread (libmerc.h:227-231);
 *   - the returned analysis_context points into the processor and is
 *     overwritten by the next call on it (libmerc.cc:173-175);
 *   - errors return 0 / NULL, never abort (libmerc.cc:138-240).
 * Not provided on this path (the entry points exist, so the reference's own
 * binaries link, and refuse): stats (do_stats is refused at mercury_init;
 * mercury_write_stats_data returns false) and FDC/CBOR output.
 */
#ifndef MERCURY_AMD_LIBMERC_H
#define MERCURY_AMD_LIBMERC_H

#include <stdarg.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <time.h>

#include "mfp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* libmerc.h:46-56 */
enum log_level {
    log_emerg = 0, log_alert = 1, log_crit = 2, log_err = 3, log_warning = 4,
    log_notice = 5, log_info = 6, log_debug = 7, log_none = 8
};
typedef int (*printf_err_ptr)(enum log_level level, const char *format, va_list args);

/* libmerc.h:94-98 */
enum enc_key_type { enc_key_type_none = 0, enc_key_type_aes_128, enc_key_type_aes_256 };

/* libmerc.h:109-154 (C layout) */
struct libmerc_config {
    bool dns_json_output;
    bool certs_json_output;
    bool metadata_output;
    bool do_analysis;
    bool do_stats;
    bool report_os;
    bool output_tcp_initial_data;
    bool output_udp_initial_data;
    char *resources;
    const uint8_t *enc_key;
    enum enc_key_type key_type;
    char *packet_filter_cfg;
    float fp_proc_threshold;
    float proc_dst_threshold;
    size_t max_stats_entries;
};

/* libmerc.h:307-313 */
enum fingerprint_status {
    fingerprint_status_no_info_available = 0,
    fingerprint_status_labeled = 1,
    fingerprint_status_randomized = 2,
    fingerprint_status_unlabled = 3,
    fingerprint_status_unanalyzed = 4,
};

/* libmerc.h:351-373 */
enum fingerprint_type {
    fingerprint_type_unknown = 0, fingerprint_type_tls = 1, fingerprint_type_tls_server = 2,
    fingerprint_type_http = 3, fingerprint_type_http_server = 4, fingerprint_type_ssh = 5,
    fingerprint_type_ssh_kex = 6, fingerprint_type_tcp = 7, fingerprint_type_dhcp = 8,
    fingerprint_type_smtp_server = 9, fingerprint_type_dtls = 10, fingerprint_type_dtls_server = 11,
    fingerprint_type_quic = 12, fingerprint_type_tcp_server = 13, fingerprint_type_openvpn = 14,
    fingerprint_type_tofsee = 15, fingerprint_type_stun = 16, fingerprint_type_ssh_init = 17,
    fingerprint_type_ssh_server = 18, fingerprint_type_ssh_kex_server = 19, fingerprint_type_ssh_init_server = 20,
};

/* libmerc.h:164-180 */
struct attribute_context {
    const char *const *tag_names;      /* attribute names                         */
    const long double *prob_scores;    /* probability per name (0 when not set)   */
    size_t attributes_len;             /* length of both arrays                   */
};

/* libmerc.h:481-484 */
struct os_information {
    char *os_name;
    uint64_t os_prevalence;
};

typedef struct mercury *mercury_context;
typedef struct mercury_packet_processor_s *mercury_packet_processor;
struct analysis_context;

/* libmerc.h:88 */
MFP_EXPORT void register_printf_err_callback(printf_err_ptr callback);
/* libmerc.h:211 -- packet_filter_cfg, do_analysis, resources honoured */
MFP_EXPORT mercury_context mercury_init(const struct libmerc_config *vars, int verbosity);
/* libmerc.h:224 */
MFP_EXPORT int mercury_finalize(mercury_context mc);
/* libmerc.h:244 */
MFP_EXPORT mercury_packet_processor mercury_packet_processor_construct(mercury_context mc);
/* libmerc.h:253 */
MFP_EXPORT void mercury_packet_processor_destruct(mercury_packet_processor mpp);
/* libmerc.h:270, :293 -- the record text (mfp_write_json_batch[_analysis]), with the
 * "analysis" object under do_analysis; byte-identical to the reference except
 * 0 for IP-in-IP packets whose outer IPv6 header has extension headers */
MFP_EXPORT size_t mercury_packet_processor_write_json(mercury_packet_processor processor, void *buffer,
                                                      size_t buffer_size, uint8_t *packet, size_t length,
                                                      struct timespec *ts);
MFP_EXPORT size_t mercury_packet_processor_write_json_linktype(mercury_packet_processor processor, void *buffer,
                                                               size_t buffer_size, uint8_t *packet, size_t length,
                                                               struct timespec *ts, uint16_t linktype);
/* libmerc.h:332 (packet starts at the IP header) */
MFP_EXPORT const struct analysis_context *mercury_packet_processor_ip_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts);
/* libmerc.h:670 (Ethernet) */
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts);
/* libmerc.h:693 */
MFP_EXPORT const struct analysis_context *mercury_packet_processor_get_analysis_context_linktype(
    mercury_packet_processor processor, uint8_t *packet, size_t length, struct timespec *ts, uint16_t linktype);
/* libmerc.h:348 */
MFP_EXPORT enum fingerprint_status analysis_context_get_fingerprint_status(const struct analysis_context *ac);
/* libmerc.h:395 */
MFP_EXPORT enum fingerprint_type analysis_context_get_fingerprint_type(const struct analysis_context *ac);
/* libmerc.h:410 */
MFP_EXPORT const char *analysis_context_get_fingerprint_string(const struct analysis_context *ac);
/* libmerc.h:425 */
MFP_EXPORT const char *analysis_context_get_server_name(const struct analysis_context *ac);
/* libmerc.h:711 */
MFP_EXPORT const char *analysis_context_get_user_agent(const struct analysis_context *ac);
/* libmerc.h:446 */
MFP_EXPORT bool analysis_context_get_process_info(const struct analysis_context *ac, const char **probable_process,
                                                  double *probability_score);
/* libmerc.h:471 */
MFP_EXPORT bool analysis_context_get_malware_info(const struct analysis_context *ac,
                                                  bool *probable_process_is_malware, double *probability_malware);
/* libmerc.h:505 -- os_info of the selected process (report_os) */
MFP_EXPORT bool analysis_context_get_os_info(const struct analysis_context *ac, const struct os_information **os_info,
                                             size_t *os_info_len);
/* libmerc.h:733 -- the ClientHello's ALPN protocol_name_list */
MFP_EXPORT bool analysis_context_get_alpns(const struct analysis_context *ac, const uint8_t **alpn_data,
                                           size_t *alpn_length);
/* libmerc.h:790 -- the attributes of the processor's last result */
MFP_EXPORT const struct attribute_context *mercury_packet_processor_get_attributes(mercury_packet_processor processor);
/* libmerc.h:647 -- opaque classifier handle (the analysis context), NULL without one */
MFP_EXPORT void *mercury_get_classifier(mercury_context mc);
/* libmerc.h:754 -- flow_state_pkts_needed of the last get_analysis_context call
 * ("reassembly" configured: a flow waits for more segments) */
MFP_EXPORT bool mercury_packet_processor_more_pkts_needed(mercury_packet_processor processor);
/* libmerc.h:603, :617, :556, :638 */
MFP_EXPORT uint32_t mercury_get_version_number(void);
MFP_EXPORT void mercury_get_version_string(char *buf, size_t size);
MFP_EXPORT const char *mercury_get_license_string(void);
MFP_EXPORT const char *mercury_get_resource_version(mercury_context mc);
/* libmerc.h:570 -- "2.18.0\n" */
MFP_EXPORT void mercury_print_version_string(FILE *f);
/* libmerc.h:584 -- the commit this library was built from */
MFP_EXPORT void mercury_print_git_commit(FILE *f);
/* libmerc.h:536 -- no stats aggregator on this path: false */
MFP_EXPORT bool mercury_write_stats_data(mercury_context mc, const char *stats_data_file_path);
/* libmerc.h:771 -- 0 */
MFP_EXPORT size_t get_stats_aggregator_num_entries(mercury_context mc);

/* libmerc.h:799-829 */
struct ipv6_addr_ext { uint32_t a, b, c, d; };
struct flow_key_ext {
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t protocol;
    uint8_t ip_vers;
    union {
        struct { uint32_t src; uint32_t dst; } ipv4;
        struct { struct ipv6_addr_ext src; struct ipv6_addr_ext dst; } ipv6;
    } addr;
};
/* libmerc.h:833-840 */
enum fdc_return {
    FDC_NO_DATA = 0, FDC_WRITE_INSUFFICIENT_SPACE = -1, FDC_WRITE_FAILURE = -2, MORE_PACKETS_NEEDED = -3,
    UNKNOWN_ERROR = -4, INVALID_INPUT = -5,
};
/* libmerc.h:877 -- FDC/CBOR output is not provided: UNKNOWN_ERROR (INVALID_INPUT
 * for a NULL processor), *ac = NULL, and a log line */
MFP_EXPORT int mercury_packet_processor_get_analysis_context_fdc(mercury_packet_processor processor,
                                                                 const struct flow_key_ext *key, const uint8_t *data,
                                                                 size_t len, uint8_t *buffer, size_t *buffer_size,
                                                                 const struct analysis_context **ac);

/* libmercury_amd extension (not in libmerc.h): the packets, since mercury_init,
 * that a selection naming protocols outside this path (e.g. "all") let such a
 * protocol claim (MFP_MSG_OTHER): the reference writes a record for them, this
 * library writes none (logged once per context) */
MFP_EXPORT uint64_t mercury_amd_other_packets(mercury_context mc);

#ifdef __cplusplus
}
#endif
#endif
