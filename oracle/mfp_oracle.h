/*
 * mfp_oracle.h -- CPU restatement (plain C) of cisco/mercury's packet
 * fingerprint path, used ONLY as a test checker and as the CPU baseline leg
 * of bench.py.  It is test infrastructure: the product (mercury_amd/) never
 * links, loads or calls it.
 *
 * Parity: pinned against the reference itself (oracle/_ref, built from
 * /root/reference by oracle/Makefile.ref) and against the reference's golden
 * file test/data/top_100_fingerprints.fp -- see tests/test_oracle.py.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to /root/reference/src/libmerc/).
 */
#ifndef MFP_ORACLE_H
#define MFP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* selection bits (proto_identify.h:620-895 traffic_selector ctor, the subset
 * this path implements) */
enum {
    MFPO_SEL_TLS_CH     = 1u << 0,   /* "tls" / "tls.client_hello"       */
    MFPO_SEL_TLS_SH     = 1u << 1,   /* "tls" / "tls.server_hello"       */
    MFPO_SEL_TLS_CERT   = 1u << 2,   /* "tls" / "tls.server_certificate" */
    MFPO_SEL_SSH_CLIENT = 1u << 3,   /* "ssh" / "ssh.client"             */
    MFPO_SEL_SSH_SERVER = 1u << 4,   /* "ssh" / "ssh.server"             */
    MFPO_SEL_HTTP_REQ   = 1u << 5,   /* "http" / "http.request"          */
    MFPO_SEL_HTTP_RESP  = 1u << 6,   /* "http" / "http.response"         */
    MFPO_SEL_TCP_SYN    = 1u << 7,   /* "tcp"                            */
    MFPO_SEL_TCP_SYNACK = 1u << 8,   /* "tcp.syn_ack"                    */
    MFPO_SEL_DTLS       = 1u << 9,   /* "dtls"                           */
};

/* fingerprint_type values (libmerc.h fingerprint_type) */
enum {
    MFPO_FP_UNKNOWN = 0, MFPO_FP_TLS = 1, MFPO_FP_TLS_SERVER = 2,
    MFPO_FP_HTTP = 3, MFPO_FP_HTTP_SERVER = 4, MFPO_FP_SSH = 5,
    MFPO_FP_SSH_KEX = 6, MFPO_FP_TCP = 7, MFPO_FP_DTLS = 10,
    MFPO_FP_DTLS_SERVER = 11, MFPO_FP_TCP_SERVER = 13, MFPO_FP_SSH_INIT = 17,
    MFPO_FP_SSH_SERVER = 18, MFPO_FP_SSH_KEX_SERVER = 19,
    MFPO_FP_SSH_INIT_SERVER = 20,
};

/* which reference entry point's semantics to follow */
enum {
    MFPO_MODE_WRITE_JSON = 0,   /* stateful_pkt_proc::write_json  pkt_proc.cc:1063 */
    MFPO_MODE_ANALYSIS   = 1,   /* stateful_pkt_proc::analyze_ip_packet pkt_proc.cc:1597 */
};

/* message kinds (our own protocol tag, one per protocol-variant alternative) */
enum {
    MFPO_MSG_NONE = 0, MFPO_MSG_TLS_CH, MFPO_MSG_TLS_SH, MFPO_MSG_TLS_CERT,
    MFPO_MSG_SSH_INIT, MFPO_MSG_SSH_KEX, MFPO_MSG_HTTP_REQ, MFPO_MSG_HTTP_RESP,
    MFPO_MSG_TCP_SYN, MFPO_MSG_TCP_SYNACK, MFPO_MSG_DTLS_CH, MFPO_MSG_DTLS_SH,
    MFPO_MSG_DTLS_HVR,
};

typedef struct {
    uint32_t select;      /* MFPO_SEL_* */
    uint32_t tls_format;  /* 0, 1 or 2 (global_config.h fp_format) */
    uint32_t mode;        /* MFPO_MODE_* */
} mfpo_config;

#define MFPO_MAX_FP 8192  /* fingerprint::MAX_FP_STR_LEN fingerprint.h:15 */

typedef struct {
    uint32_t fp_type;       /* MFPO_FP_*; 0 = no fingerprint */
    uint32_t fp_len;
    uint32_t msg;           /* MFPO_MSG_* */
    uint32_t emit;          /* is_not_empty(x): reference would emit a record */
    uint32_t truncated;     /* more bytes needed (reassembly_properties.truncated) */
    /* classifier inputs (destination_context, result.h:346) */
    int32_t  sni_off, sni_len;   /* offsets into the packet, -1 = none */
    int32_t  ua_off, ua_len;
    uint8_t  ip_vers;            /* flow key (flow_key.h:71) */
    uint8_t  ip_proto;
    uint16_t src_port, dst_port; /* host order */
    uint8_t  src_addr[16], dst_addr[16];
    char     fp[MFPO_MAX_FP + 1];
} mfpo_result;

/* process one packet; returns fp_type */
int mfpo_process(const uint8_t *pkt, size_t len, uint16_t linktype,
                 const mfpo_config *cfg, mfpo_result *res);

/* batch over an arena with 16-byte descriptors (see include/mfp.h);
 * writes per-packet fp_type/fp_len/flags and the concatenated fp strings
 * (arena order = packet order) into caller buffers; returns total fp bytes
 * or -1 if fp_cap is too small. */
typedef struct {
    uint64_t offset;
    uint32_t caplen;
    uint16_t linktype;
    uint16_t flags;
} mfpo_desc;

long long mfpo_process_batch(const uint8_t *arena, const mfpo_desc *desc, size_t n,
                             const mfpo_config *cfg,
                             uint8_t *fp_type, uint32_t *fp_len, uint8_t *flags,
                             uint64_t *fp_off, char *fp_arena, size_t fp_cap);

/* multi-threaded timing harness (one worker per thread over contiguous
 * shards, like mercury's one-processor-per-thread model); returns seconds */
double mfpo_time_batch(const uint8_t *arena, const mfpo_desc *desc, size_t n,
                       const mfpo_config *cfg, int threads, int reps,
                       unsigned long long *fp_bytes_out);

#ifdef __cplusplus
}
#endif
#endif
