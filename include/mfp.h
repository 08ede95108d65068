/*
 * mfp.h -- C-ABI of libmercury_amd.so, the MI355X-native packet
 * fingerprint/classify path.  Plain pointers and sizes only.
 *
 * Two layers:
 *  1. the BATCH API below (mfp_*): packet batches in HBM or host memory,
 *     one launch per batch; this is what the libmerc per-packet shims
 *     (include/mercury_amd_libmerc.h) and our host pipeline call;
 *  2. libmerc-compatible per-packet symbols, declared in
 *     include/mercury_amd_libmerc.h, replacing src/libmerc/libmerc.h.
 *
 * The batch entry point replaces the reference's per-packet plugin call
 * pkt_proc::apply(packet_info*, uint8_t*) (src/pkt_proc.hpp:26-33) as driven
 * by pcap_file_dispatch_pkt_processor (src/pcap_file_io.c:470-512) and
 * process_all_packets_in_block (src/af_packet_v3.c:174-210): instead of one
 * C-ABI crossing per packet, the caller fills an arena + descriptor array
 * and crosses once per batch.
 */
#ifndef MFP_H
#define MFP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFP_EXPORT __attribute__((visibility("default")))

/* One packet of a batch (16 bytes).  `offset` is the byte offset of the
 * captured frame in the arena; `linktype` is the pcap LINKTYPE (1 Ethernet,
 * 9 PPP, 101 raw IP, 113 Linux SLL, 276 Linux SLL2, 0 BSD loopback), as in
 * mercury_packet_processor_write_json_linktype (libmerc.h:293). */
typedef struct {
    uint64_t offset;
    uint32_t caplen;
    uint16_t linktype;
    uint16_t flags;      /* 0, or MFP_DESC_* */
} mfp_pkt_desc;
enum {
    /* a QUIC Initial whose ClientHello was reassembled across datagrams (the
     * reassembler's frames, mfp_reassembler_frames): the packet's caplen bytes,
     * zero padding to a multiple of 8, a little-endian u32 length L, 4 zero
     * bytes, then the L bytes of reassembled CRYPTO data the ClientHello is
     * parsed from (quic_init::reparse_crypto_buf quic.h:1593-1598) */
    MFP_DESC_QUIC_CRYPTO = 1,
};

/* Per-packet result (32 bytes). */
typedef struct {
    uint64_t fp_offset;  /* fingerprint string offset in the fp arena    */
    uint32_t fp_len;     /* string length (no NUL), 0 when fp_type == 0  */
    uint8_t  fp_type;    /* enum fingerprint_type (libmerc.h:351-373)     */
    uint8_t  msg;        /* protocol tag, MFP_MSG_*                       */
    uint8_t  flags;      /* MFP_FLAG_*                                    */
    uint8_t  xflags;     /* MFP_XF_* (the classifier status is mfp_analysis.status) */
    /* classifier inputs (destination_context, result.h:346): offsets are
     * relative to the packet start, len 0xffff = absent */
    uint16_t sni_off, sni_len;
    uint16_t ua_off, ua_len;
    uint16_t src_port, dst_port;   /* host byte order */
    uint32_t net;        /* innermost IP header: offset (bits 0-15), version (16-19);
                            IP-in-IP (MFP_FLAG_ENCAP): levels (20-22), outer
                            level i is IPv6 (bit 23+i, outermost = 0), an outer
                            header with IPv6 extension headers (27) */
} mfp_record;

/* Per-packet classifier result (analysis_result, result.h:174-300), written
 * by the --analysis pass for packets whose message the classifier sees
 * (TLS ClientHello, HTTP request, SSH client KEXINIT: MFP_AN_VALID). */
typedef struct {
    double   score;          /* analysis_result::max_score                      */
    double   malware_prob;   /* analysis_result::malware_prob (-1 if none)      */
    uint32_t process;        /* process-name id (mfp_process_name), or ~0u     */
    uint16_t attr;           /* attribute_result tags (mfp_attribute_name bits):
                                the selected process's tags (bits >=
                                MFP_ATTR_DB_FIRST) plus encrypted_dns,
                                encrypted_channel, domain_faking, faketls     */
    uint8_t  status;         /* enum fingerprint_status (libmerc.h:307-313)     */
    uint8_t  flags;          /* MFP_AN_*                                        */
    uint32_t proc_slot;      /* the selected process of its fingerprint entry
                                (os_info: mfp_process_os_info), or ~0u          */
    uint32_t reserved;       /* 0 */
} mfp_analysis;

enum {
    MFP_AN_VALID     = 1,    /* the message was classified: the reference writes
                                an "analysis" object (pkt_proc.cc:1211-1213)  */
    MFP_AN_MALWARE   = 2,    /* max_mal                                      */
    MFP_AN_CLASSIFY_MALWARE = 4,   /* malware fields meaningful (malware db) */
    MFP_AN_PENDING   = 8,    /* internal: unknown TLS, status resolved later */
};
#define MFP_NO_PROCESS 0xffffffffu

/* Attribute probabilities (attribute_result::prob_score, result.h:38).  Tags
 * 0-9 are the reserved names (residential_proxy ... faketls, pkt_proc.h:72,
 * analysis.h:830); the archive's own tags take 10-15 (attribute_names,
 * result.h:133-172).  A reserved tag's probability follows from the record:
 * encrypted_channel = malware_prob, encrypted_dns / domain_faking / faketls =
 * 1.0 (analysis.h:555-577).  The archive tags' probabilities (the softmax
 * mass of the processes carrying the tag, analysis.h:268-277,335-341) come in
 * an optional per-packet array of MFP_ATTR_DB_TAGS doubles: attr_prob[i *
 * MFP_ATTR_DB_TAGS + (bit - MFP_ATTR_DB_FIRST)], written for the set bits. */
#define MFP_ATTR_DB_FIRST 10
#define MFP_ATTR_DB_TAGS  6
#define MFP_ATTR_MAX_TAGS 16

enum {
    MFP_FLAG_EMIT      = 1,  /* the reference's write_json emits a record   */
    MFP_FLAG_TRUNCATED = 2,  /* reassembly_properties.truncated             */
    MFP_FLAG_HASHED    = 4,  /* device arena: the string's 64-bit hash follows it
                                at fp_offset + round_up(fp_len, 8) (the
                                classifier's lookup key; cleared when the
                                strings are packed for the host) */
    MFP_FLAG_CERT_CLIENT = 8,  /* TLS certificate message: entity client (tls.h:728-744) */
    MFP_FLAG_CERT_SERVER = 16, /* ... entity server; neither = undetermined   */
    MFP_FLAG_ENCAP       = 32, /* reached through IP-in-IP encapsulation (pkt_proc.cc:959) */
    MFP_FLAG_NO_CIPHERS  = 64, /* (D)TLS ClientHello with an empty cipher-suite list: the
                                  reference writes no "tls"/"dtls" object for it (tls.h:1882-1885) */
    MFP_FLAG_SIDECAR     = 128,/* QUIC: a sidecar follows the string's hash, at fp_offset +
                                  round_up(fp_len, 8) + 8 (also when fp_len is 0): a header
                                  {u16 alpn_off, u16 alpn_len, u16 side_len (bytes of the
                                  sidecar), u16 json_off (0: none)}, then the server name, the
                                  QUIC user agent and the ALPN list, which exist only in the
                                  decrypted payload (sni/ua spans index the sidecar); contexts in
                                  MFP_MODE_WRITE_JSON add at json_off what the JSON writer prints
                                  (the plaintext, the handshake bytes, the cc frame's place, the
                                  salt); with reassembly inputs requested an Initial whose CRYPTO
                                  data may need reassembly has the block too (its plaintext).
                                  Packed host arenas keep it. */
};
enum {
    MFP_XF_TLS_UA = 1,   /* (D)TLS ClientHello: ua_off/ua_len hold the user agent of a
                            quic_transport_parameters_draft extension (transport parameter
                            0x3129, tls_extensions::set_meta_data tls.h:1346-1355), not the
                            ALPN list; host outputs re-read the ALPN list from the packet */
};
/* For MFP_MSG_TLS_SH / MFP_MSG_TLS_CERT records sni_off/sni_len hold the
 * certificate_list datum (tls.h:275-296), the bytes the JSON writer's
 * "certs" array is built from; len 0xffff = no list.  For MFP_MSG_TLS_CH and
 * MFP_MSG_DTLS_CH records ua_off/ua_len hold the ALPN protocol_name_list
 * (destination_context::alpn_array, analysis_context_get_alpns), unless
 * MFP_XF_TLS_UA; sni_off/sni_len hold the LAST server_name extension (the
 * destination context's, tls.h:1316-1345; the JSON text prints the first,
 * tls.h:1052-1080, which the writer re-reads from the packet). */

enum {
    MFP_MSG_NONE = 0, MFP_MSG_TLS_CH, MFP_MSG_TLS_SH, MFP_MSG_TLS_CERT,
    MFP_MSG_SSH_INIT, MFP_MSG_SSH_KEX, MFP_MSG_HTTP_REQ, MFP_MSG_HTTP_RESP,
    MFP_MSG_TCP_SYN, MFP_MSG_TCP_SYNACK, MFP_MSG_DTLS_CH, MFP_MSG_DTLS_SH,
    MFP_MSG_DTLS_HVR, MFP_MSG_QUIC,
    MFP_MSG_STUN,     /* stun::message (stun.h:783); sni_off/sni_len: the STUN message, ua: SOFTWARE */
    MFP_MSG_OPENVPN,  /* openvpn_tcp (openvpn.h:353); sni_off/sni_len: the TCP payload         */
    MFP_MSG_OTHER,    /* identified as a protocol the selection names but this path does not
                         parse ("all", or e.g. "dns": traffic_selector proto_identify.h:620-895):
                         no record; counted (mercury_packet_processor_* log it once)             */
};

/* Reassembly inputs, one per packet (the device walk's view of tcp_packet,
 * tcpip.h:137-173, after set_tcp_protocol pkt_proc.cc:488-572; for DTLS
 * ClientHello fragments, MFP_SEG_DTLS, of the handshake header) */
typedef struct {
    uint32_t seq;        /* TCP sequence number (host order)                          */
    uint32_t more;       /* additional_bytes_needed of the message parsed here        */
    uint32_t pay_off;    /* TCP data: offset in the packet                            */
    uint16_t pay_len;    /* TCP data length (tcp_packet::data_length)                 */
    uint8_t  kind;       /* MFP_SEG_* bits; 0 = not a data segment                    */
    uint8_t  reserved;
} mfp_tcp_seg;
enum {
    MFP_SEG_DATA = 1,           /* a TCP data segment process_tcp_data sees (pkt_proc.cc:773) */
    MFP_SEG_SUPPLEMENTARY = 2,  /* tcp_packet::supplementary_reassembly (SSH KEXINIT)          */
    MFP_SEG_SSH = 4,            /* reassembly_type::ssh (indefinite, pkt_proc.cc:552)          */
    MFP_SEG_TCP = 8,            /* a TCP packet with a whole header (tcp_packet::is_valid)     */
    MFP_SEG_SYN_RST = 16,       /* SYN, SYN/ACK or RST: analyze_ip_packet skips it in reassembly
                                   mode (pkt_proc.cc:1632-1634)                                */
    MFP_SEG_IP = 32,            /* the link layer led to an IP packet: analyze_ip_packet ran    */
    MFP_SEG_DTLS = 64,          /* a DTLS ClientHello handshake fragment (dtls_client_hello,
                                   dtls.h:155-175): seq = fragment_offset, more =
                                   additional_bytes_needed, pay_off / pay_len = the fragment's
                                   bytes; its message_seq is the 2 bytes at pay_off - 8       */
    MFP_SEG_QUIC = 128,         /* a QUIC Initial (quic_init): more = additional_bytes_needed,
                                   pay_off / pay_len = the UDP payload; when its CRYPTO data
                                   may take part in reassembly the record's sidecar carries the
                                   plaintext (JSON block flag bit 2)                          */
};

/* semantics of the reference entry point to follow */
enum {
    MFP_MODE_WRITE_JSON = 0,  /* stateful_pkt_proc::write_json (pkt_proc.cc:1063)      */
    MFP_MODE_ANALYSIS   = 1,  /* stateful_pkt_proc::analyze_ip_packet (pkt_proc.cc:1597) */
};

typedef struct mfp_context_s *mfp_context;

/* Create a context on HIP device `device`.  `packet_filter_cfg` uses the
 * reference's syntax (global_config.h:143-153): a bare protocol list, or
 * "key=value;..." with select=/format=.  Supported selections: tls,
 * tls.client_hello, tls.server_hello, tls.server_certificate, ssh,
 * ssh.client, ssh.server, http, http.request, http.response, tcp,
 * tcp.syn_ack, dtls, quic (QUIC Initial packets: decrypted and fingerprinted
 * on the device), stun, openvpn_tcp, gre, vxlan, geneve (decapsulation,
 * pkt_proc.cc:959-1049); "format=" takes tls/N and quic/N; "reassembly"
 * enables mfp_process_batch_reassembly; "report_os" as the reference's.
 * ""/"all" and names of protocols outside the path are accepted: their
 * messages get MFP_MSG_OTHER and no record.  Options that change the
 * reference's records (metadata, certs-json, raw-features of tls/stun/all,
 * crypto-assess, network-behavioral-detections, exposed-creds, http-headers,
 * http-body-max > 0, nonselected-tcp-data / -udp-data, quic-trial-decryption,
 * minimize-ram, fp_proc_threshold / proc_dst_threshold > 0, stats) are
 * refused.  Returns NULL on error (refused option, no HIP device, extension
 * not loadable). */
MFP_EXPORT mfp_context mfp_init(const char *packet_filter_cfg, int device, int mode);
/* mfp_init with the resource archive's decryption key (libmerc_config.enc_key,
 * libmerc.h:124-125): 16 bytes, AES-128-CBC with the IV as the file's first
 * block (encrypted_file enc_file_reader.h:86-231); NULL or all zero = plain. */
MFP_EXPORT mfp_context mfp_init_ex(const char *packet_filter_cfg, int device, int mode, const uint8_t *enc_key);
MFP_EXPORT void mfp_finalize(mfp_context ctx);

/* Device-resident batch: all pointers are device (HBM) pointers.  The fp
 * arena receives the fingerprint strings (each string contiguous at
 * rec[i].fp_offset, in no particular order; the arena may contain unused
 * gaps).  d_fp_used is a device u64[4], zeroed by the call:
 * [0] arena bytes reserved (copy [0, d_fp_used[0]) to read every string),
 * [1] overflow flag (arena too small: records without strings), [2] string
 * bytes written (sum of fp_len), [3] packets handled by the fallback lane.
 * Packets are read with aligned 16-byte loads: the 16-byte block holding a
 * packet's last byte must be readable.  d_fp_arena must be 256-byte aligned
 * (as hipMalloc returns): strings start on 16- or 64-byte boundaries and are
 * written in whole 16-byte blocks.  `stream` is a hipStream_t (NULL =
 * default stream).  Asynchronous; returns 0 or a negative error.  For no
 * overflow fp_cap must be >= mfp_fp_arena_bound(n, total caplen). */
MFP_EXPORT int mfp_process_batch_device(mfp_context ctx, const uint8_t *d_arena, const mfp_pkt_desc *d_desc,
                                        size_t n, mfp_record *d_rec, char *d_fp_arena, size_t fp_cap,
                                        uint64_t *d_fp_used, void *stream);

/* Host batch: copies arena/descriptors to the device, runs, copies back.
 * The strings come back packed in packet order (fp_arena holds the strings
 * back to back, each QUIC record's sidecar right behind its string).
 * Synchronous.  Returns bytes of fp arena used, or a negative error. */
MFP_EXPORT long long mfp_process_batch_host(mfp_context ctx, const uint8_t *arena, size_t arena_len,
                                            const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                            char *fp_arena, size_t fp_cap);

/* Pre-allocate the context's device workspace for batches of up to n
 * packets (otherwise grown on demand by the first larger batch). */
MFP_EXPORT int mfp_reserve(mfp_context ctx, size_t n);

/* Upper bound on fp-arena bytes for packets totalling `total_caplen` bytes. */
MFP_EXPORT size_t mfp_fp_arena_bound(size_t n, size_t total_caplen);

/* Parse a packet_filter_cfg string exactly as mfp_init does (host only, no
 * device needed): *select receives the MFP selection bits, *tls_format the TLS
 * format (0/1/2) in bits 0-7 and the QUIC format (0/1) in bits 8-15.
 * Mirrors global_config's parser (global_config.h:55-121, 143-153, 246-276;
 * config_generator.cc:115-162), including what it only logs: an unknown
 * protocol name ends the list, an unknown format keeps the default.  Returns
 * 0; 1 when the reference would have logged such a problem (the text is in
 * mfp_last_error()); -1 on error. */
MFP_EXPORT int mfp_parse_filter(const char *packet_filter_cfg, uint32_t *select, uint32_t *tls_format);
/* as mfp_parse_filter, and *other = the protocols the selection names outside
 * this path whose identification comes first (bit set of mfp_device.hpp's
 * BLK_*; "all" sets all of them): their messages write no record
 * (MFP_MSG_OTHER). */
MFP_EXPORT int mfp_parse_filter_ex(const char *packet_filter_cfg, uint32_t *select, uint32_t *tls_format,
                                   uint32_t *other);

/* ---- --analysis: the process classifier (classifier, analysis.h) ----
 * Enabled by mfp_init when packet_filter_cfg holds "resources=<archive.tgz>"
 * and "analysis" (key=value form), mirroring libmerc_config.resources and
 * do_analysis; the TLS fingerprint format is then the archive's
 * (pkt_proc.h:93-99). */
MFP_EXPORT int mfp_analysis_enabled(mfp_context ctx);

/* Classify a device-resident batch already fingerprinted by
 * mfp_process_batch_device on the same stream (records and fp arena as it
 * left them).  d_out: n mfp_analysis records (the records are read only);
 * d_attr_prob: NULL, or n * MFP_ATTR_DB_TAGS doubles for the archive tags'
 * probabilities.  Batches must be submitted in stream order: the unknown-TLS
 * status (randomized / unlabeled) depends on earlier sightings. */
MFP_EXPORT int mfp_analyze_batch_device(mfp_context ctx, const uint8_t *d_arena, const mfp_pkt_desc *d_desc, size_t n,
                                        mfp_record *d_rec, const char *d_fp_arena, mfp_analysis *d_out,
                                        double *d_attr_prob, void *stream);
/* Pipelined form of mfp_analyze_batch_device for a stream of device batches:
 * launches this batch's kernels on `stream`, then decides the PREVIOUS
 * batch's unknown-TLS sightings (stream order, the context's LRU) and applies
 * them while the device runs this one.  A batch's analysis records are final
 * after the next call or mfp_analysis_flush; keep its buffers until then.
 * Decisions equal the synchronous call's. */
MFP_EXPORT int mfp_analyze_batch_device_pipelined(mfp_context ctx, const uint8_t *d_arena, const mfp_pkt_desc *d_desc,
                                                  size_t n, mfp_record *d_rec, const char *d_fp_arena,
                                                  mfp_analysis *d_out, double *d_attr_prob, void *stream);
/* decide the batch mfp_analyze_batch_device_pipelined left pending; waits */
MFP_EXPORT int mfp_analysis_flush(mfp_context ctx);
/* The deferred form (mfp_analysis_defer on; the shards of one stream): launches
 * this batch's kernels and leaves the PREVIOUS batch, if undecided, as the one
 * mfp_analysis_distinct / _sequence / _resolve / _resolve_sequence act on, so
 * the shards' ordered merge of batch k-1 runs while the device runs batch k.
 * Every batch must be decided before the call after next (-1 otherwise);
 * mfp_analysis_defer_newest then selects the last batch for its decision. */
MFP_EXPORT int mfp_analyze_batch_device_deferred_pipelined(mfp_context ctx, const uint8_t *d_arena,
                                                           const mfp_pkt_desc *d_desc, size_t n, mfp_record *d_rec,
                                                           const char *d_fp_arena, mfp_analysis *d_out,
                                                           double *d_attr_prob, void *stream);
MFP_EXPORT int mfp_analysis_defer_newest(mfp_context ctx);

/* mfp_process_batch_host plus classification into analysis[n] (NULL: none)
 * and attr_prob[n * MFP_ATTR_DB_TAGS] (NULL: not wanted). */
MFP_EXPORT long long mfp_process_batch_host_ex(mfp_context ctx, const uint8_t *arena, size_t arena_len,
                                               const mfp_pkt_desc *desc, size_t n, mfp_record *rec,
                                               char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                               double *attr_prob);

/* Host batch, pipelined (the end-to-end path: capture buffer in, records
 * out).  The batch is cut into chunks of `chunk` packets (0: 1M); two chunks
 * are in flight on two HIP streams, so the H2D copy of one overlaps the
 * kernels of the other and the D2H copies of both.  `analysis` may be NULL
 * (fingerprints only).  Results are those of mfp_process_batch_host_ex on
 * the whole batch: rec[i].fp_offset indexes fp_arena, whose strings are laid
 * out chunk after chunk.  attr_prob as for mfp_process_batch_host_ex (NULL:
 * not copied back).  Host buffers should be page-locked
 * (hipHostMalloc / hipHostRegister) for full PCIe rate.  Synchronous;
 * returns the fp-arena bytes used or a negative error. */
MFP_EXPORT long long mfp_process_pipelined(mfp_context ctx, const uint8_t *arena, size_t arena_len,
                                           const mfp_pkt_desc *desc, size_t n, mfp_record *rec, char *fp_arena,
                                           size_t fp_cap, mfp_analysis *analysis, double *attr_prob, size_t chunk);

/* ---- the unknown-TLS prevalence set (fingerprint_prevalence, analysis.h:362-421) ----
 * A TLS fingerprint the archive does not label, and not in its known
 * prevalence list, is "randomized" when it is not in an LRU of the 100000 most
 * recently seen such fingerprints (analysis.h:433) and "unlabeled" when it is;
 * the LRU is updated on every sighting, in stream order
 * (perform_analysis_common analysis.h:1043-1083).  The device finds each
 * batch's sightings; the decisions are made on the host, in stream order, by
 * an mfp_prevalence object (identity: the string's 64-bit hash).  By default
 * every analysis call decides its own batch (the call waits for its kernels);
 * shards of one stream (several contexts) defer the decision and resolve their
 * batches in shard order against one shared object. */
/* ---- TCP reassembly ("reassembly" in the config) ----
 * The reference's write_json path with reassembly (process_tcp_data
 * pkt_proc.cc:773-893, tcp_reassembler reassembly.hpp:140-900): a message
 * whose first segment needs more bytes is buffered per flow; the flow's later
 * segments are added by sequence number; the completing (or truncating)
 * segment's record carries the fingerprint of the reassembled message, and
 * the segments before it write no record. */
typedef struct mfp_reassembler_s *mfp_reassembler;   /* the processor's tcp_reassembler */
MFP_EXPORT mfp_reassembler mfp_reassembler_create(void);
MFP_EXPORT void mfp_reassembler_destroy(mfp_reassembler r);
MFP_EXPORT uint64_t mfp_reassembler_flows(mfp_reassembler r);   /* flows in reassembly */
MFP_EXPORT int mfp_reassembly_enabled(mfp_context ctx);
/* The device walk plus, per packet, the reassembly inputs (mfp_tcp_seg). */
MFP_EXPORT long long mfp_process_batch_host_seg(mfp_context ctx, const uint8_t *arena, size_t arena_len,
                                                const mfp_pkt_desc *desc, size_t n, mfp_record *rec, char *fp_arena,
                                                size_t fp_cap, mfp_tcp_seg *seg);
/* One host batch in stream order through the reassembler (state persists in
 * r across calls).  ts_ns: per-packet capture times (the 15 s flow timeout;
 * NULL = all 0).  props[i]: bit 0 = the record is a reassembled message
 * ("reassembled":true), bits 1-7 = reassembly_flag_val (missing_segment,
 * timeout, out_of_order, out_of_buffer, max_segments_exceed,
 * segment_overlaps, truncated), bits 8-11 = reassembly_overlap_flags.
 * Reassembled messages are rebuilt as frames (IP + TCP headers of the
 * completing packet, then the buffer; LINKTYPE_RAW), kept in r until its
 * next call (mfp_reassembler_frames); out_desc (optional) = desc with those
 * packets' entries pointing at their frames at offset arena_len + offset, so
 * arena ++ frames with out_desc is the input the records index (the JSON
 * writer's input).  Returns the fingerprint bytes used, or < 0. */
MFP_EXPORT long long mfp_process_batch_reassembly(mfp_context ctx, mfp_reassembler r, const uint8_t *arena,
                                                  size_t arena_len, const mfp_pkt_desc *desc, size_t n,
                                                  const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                                                  size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc);
MFP_EXPORT const uint8_t *mfp_reassembler_frames(mfp_reassembler r, size_t *len);
/* Per packet of the last batch (*n of them): 1 when the reference's
 * tcp_reassembler::dump_pkt is set after that packet (stateful_pkt_proc::dump_pkt
 * pkt_proc.cc:1842-1845) -- its data went into the flow table (TCP segments
 * pkt_proc.cc:852-866, QUIC / DTLS reassembly.hpp:931-1009,1074-1079); a packet
 * that does not reach the IP layer keeps the value of the packet before it, as
 * the reference does.  The filtered pcap writer writes these packets too
 * (pkt_processing.h:104,250).  Valid until the reassembler's next call. */
MFP_EXPORT const uint8_t *mfp_reassembler_dumped(mfp_reassembler r, size_t *n);
/* With --analysis (a context with resources=...;analysis;reassembly): the same,
 * then the records the reference writes -- packets with a record, the
 * reassembled messages -- fingerprinted and classified once more in stream
 * order; analysis/attr_prob as in mfp_process_batch_host_ex; out_desc required. */
MFP_EXPORT long long mfp_process_batch_reassembly_analysis(mfp_context ctx, mfp_reassembler r, const uint8_t *arena,
                                                           size_t arena_len, const mfp_pkt_desc *desc, size_t n,
                                                           const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                                                           size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc,
                                                           mfp_analysis *analysis, double *attr_prob);
/* The analysis_context path with reassembly (analyze_ip_packet
 * pkt_proc.cc:1597-1662, a context created with MFP_MODE_ANALYSIS and
 * "reassembly"): TCP SYN, SYN/ACK and RST packets are skipped; every other TCP
 * data segment goes through the flow table as in mfp_process_batch_reassembly;
 * the packets with a result and the reassembled messages are then fingerprinted
 * and (analysis != NULL) classified in stream order; a reassembled message
 * whose flow was truncated (timeout, max segments, ...) is "unlabeled"
 * (pkt_proc.cc:1716-1719).  more_pkts[i] (optional) =
 * analysis_context::flow_state_pkts_needed after packet i: cleared by every
 * packet that reaches the IP layer (analysis_context::reinit result.h:434-440),
 * set while its TCP flow is in reassembly, kept by packets that are not IP
 * (the state carries across calls in r). */
MFP_EXPORT long long mfp_process_batch_reassembly_context(mfp_context ctx, mfp_reassembler r, const uint8_t *arena,
                                                          size_t arena_len, const mfp_pkt_desc *desc, size_t n,
                                                          const uint64_t *ts_ns, mfp_record *rec, char *fp_arena,
                                                          size_t fp_cap, uint16_t *props, mfp_pkt_desc *out_desc,
                                                          mfp_analysis *analysis, double *attr_prob, uint8_t *more_pkts);
/* mfp_write_json_batch for the output of mfp_process_batch_reassembly (arena ++
 * frames, out_desc, records, props): completing records carry the
 * reassembler's "reassembly_properties" (reassembly.hpp:860-880,1231-1247). */
MFP_EXPORT long long mfp_write_json_batch_reassembly(const uint8_t *arena, const mfp_pkt_desc *desc, size_t n,
                                                     const mfp_record *rec, const char *fp_arena, const uint16_t *props,
                                                     const uint64_t *ts_ns, char *out, size_t out_cap,
                                                     uint64_t *line_end, uint64_t *skipped, int threads);
MFP_EXPORT long long mfp_write_json_batch_reassembly_analysis(mfp_context ctx, const uint8_t *arena,
                                                              const mfp_pkt_desc *desc, size_t n, const mfp_record *rec,
                                                              const char *fp_arena, const uint16_t *props,
                                                              const mfp_analysis *analysis, const double *attr_prob,
                                                              const uint64_t *ts_ns, char *out, size_t out_cap,
                                                              uint64_t *line_end, uint64_t *skipped, int threads);

typedef struct mfp_prevalence_s *mfp_prevalence;

/* one distinct fingerprint of a batch's sightings */
typedef struct {
    uint64_t hash;        /* the fingerprint string's hash                         */
    uint64_t first, last; /* stream positions of its first and last sighting (the
                             batch's packet indices; add a shard's base to order
                             the shards of one stream)                             */
    uint32_t count;       /* sightings                                             */
    uint32_t first_seen;  /* decision: 1 = in the LRU at the first sighting
                             (unlabeled), 0 = randomized; later sightings are all
                             unlabeled                                             */
} mfp_sighting;

MFP_EXPORT mfp_prevalence mfp_prevalence_create(uint32_t capacity);   /* the reference: 100000 */
MFP_EXPORT void mfp_prevalence_destroy(mfp_prevalence p);
MFP_EXPORT uint64_t mfp_prevalence_size(mfp_prevalence p);
/* the capacity it was created with */
MFP_EXPORT uint32_t mfp_prevalence_capacity(mfp_prevalence p);
MFP_EXPORT int mfp_prevalence_contains(mfp_prevalence p, uint64_t hash);
/* the set from least to most recently used (hashes); returns its size */
MFP_EXPORT long long mfp_prevalence_keys(mfp_prevalence p, uint64_t *out, size_t cap);
/* 1 when the distinct form is exact for these entries (no eviction possible) */
MFP_EXPORT int mfp_prevalence_distinct_exact(mfp_prevalence p, const mfp_sighting *d, size_t u);
/* decide first_seen of every entry (entries of several shards together, in
 * any order: `first`/`last` order them) and apply them; -2 when the entries
 * could evict (nothing applied: resolve the sighting sequence instead) */
MFP_EXPORT int mfp_prevalence_resolve_distinct(mfp_prevalence p, mfp_sighting *d, size_t u);
/* every sighting in stream order: seen[j] = 1 when hash[j] was in the LRU */
MFP_EXPORT int mfp_prevalence_resolve_sequence(mfp_prevalence p, const uint64_t *hash, size_t m, uint8_t *seen);
/* Shards decided where they lie (each rank its own sightings; the set at a
 * shard's start follows from the shards before it by their summaries):
 *   summary: the distinct hashes of hash[0..m) by last sighting, most recent
 *     first, at most the capacity (out holds capacity entries); returns the count;
 *   resolve_shard: decide hash[0..m) from the set that `prior` (the earlier
 *     shards' summaries, the nearest shard's first) leaves on top of p's set;
 *     p is not changed;
 *   advance: p becomes the set after a step of shards (`recent` = every
 *     shard's summary, the last shard's first).
 * Over shards in stream order these equal mfp_prevalence_resolve_sequence
 * over the concatenation. */
MFP_EXPORT long long mfp_prevalence_summary(mfp_prevalence p, const uint64_t *hash, size_t m, uint64_t *out);
MFP_EXPORT int mfp_prevalence_resolve_shard(mfp_prevalence p, const uint64_t *hash, size_t m, const uint64_t *prior,
                                            size_t nprior, uint8_t *seen);
MFP_EXPORT int mfp_prevalence_advance(mfp_prevalence p, const uint64_t *recent, size_t n);

/* the context's own LRU (created with the classifier) */
MFP_EXPORT mfp_prevalence mfp_analysis_prevalence(mfp_context ctx);
/* decide this context's sightings against p (shared by the shards of one
 * stream; the caller keeps ownership), or against its own again (p = NULL) */
MFP_EXPORT int mfp_analysis_set_prevalence(mfp_context ctx, mfp_prevalence p);
/* on != 0: analysis calls leave the unknown-TLS statuses of their batch
 * provisional (randomized, MFP_AN_PENDING) until mfp_analysis_resolve[_sequence] */
MFP_EXPORT int mfp_analysis_defer(mfp_context ctx, int on);
/* the last deferred batch's distinct unknown-TLS fingerprints (first/last =
 * batch indices); returns their count, or -3 when the batch has more distinct
 * fingerprints than its table holds (use the sequence) */
MFP_EXPORT long long mfp_analysis_distinct(mfp_context ctx, mfp_sighting *out, size_t cap);
/* its sightings' hashes in stream order; returns their count */
MFP_EXPORT long long mfp_analysis_sequence(mfp_context ctx, uint64_t *hash, size_t cap);
/* apply the decisions (entries in mfp_analysis_distinct's order / one byte
 * per sighting in stream order) to the last deferred batch's records */
MFP_EXPORT int mfp_analysis_resolve(mfp_context ctx, const mfp_sighting *d, size_t u);
MFP_EXPORT int mfp_analysis_resolve_sequence(mfp_context ctx, const uint8_t *seen, size_t m);
/* the last analysed batch's analysis records as they are now on the device
 * (for host batches analysed deferred, after the decision); returns the
 * batch's packet count */
MFP_EXPORT long long mfp_analysis_last(mfp_context ctx, mfp_analysis *out, size_t cap);

/* names behind mfp_analysis.process and the bits of mfp_analysis.attr */
MFP_EXPORT const char *mfp_process_name(mfp_context ctx, uint32_t id);
MFP_EXPORT const char *mfp_attribute_name(mfp_context ctx, uint32_t bit);
/* the archive's VERSION text (classifier::get_resource_version analysis.h:1174) */
MFP_EXPORT const char *mfp_resource_version(mfp_context ctx);
/* number of attribute names (attribute_names::value().size(), <= 16) */
MFP_EXPORT int mfp_attribute_count(mfp_context ctx);

/* libmerc_config.report_os (libmerc.h:118): os_info of the selected process
 * in analysis results (fingerprint_data ctor analysis.h:195-205).  Off by
 * default, as in the reference. */
MFP_EXPORT int mfp_analysis_report_os(mfp_context ctx, int on);
/* os_info entry k of a process slot (mfp_analysis.proc_slot): *name and
 * *prevalence (os_information, libmerc.h:481-484; archive order).  Returns the
 * entry count (0 when report_os is off or the process has none), -1 on a bad
 * slot. */
MFP_EXPORT int mfp_process_os_info(mfp_context ctx, uint32_t proc_slot, uint32_t k, const char **name,
                                   uint64_t *prevalence);

/* last analysis batch: [0] packets classified, [1] unknown-TLS sightings,
 * [2] fingerprints with more processes than the kernel handles (512),
 * [3] fingerprints in the context's prevalence LRU.  "Last batch" means the
 * last batch of the batch API (slots 0-4); the per-packet libmerc shim's
 * concurrent small batches run on slots of their own and are not counted
 * here or in mfp_analysis_counters. */
MFP_EXPORT int mfp_analysis_stats(mfp_context ctx, uint64_t out[4]);

/* the last analysis batch's counters, up to n of: [0] packets classified,
 * [1] unknown-TLS sightings, [2] packets whose fingerprint has more than 4096 processes (scored by k_analyze_huge),
 * [3] packets scored wave-per-packet (k_analyze_wave), [4] / [5] prior and
 * update-list entries read by the lane-per-packet scorer, [6] / [7] the same
 * for the wave scorer (SURVEY 8(d)'s 8*P + 12*U table bytes), [8] work items
 * k_analyze hands to k_an_features, [9] packets scored lane-per-packet
 * (k_an_score), [10] feature-table slots read by k_an_features, [11] unknown-
 * TLS sightings merged into the batch's sighting table by k_seen_scan */
#define MFP_AN_NCOUNTERS 12
MFP_EXPORT int mfp_analysis_counters(mfp_context ctx, uint64_t *out, size_t n);

/* bytes of the classifier's device tables in HBM */
MFP_EXPORT uint64_t mfp_analysis_device_bytes(mfp_context ctx);

/* host only (tests): load an archive; out = {fingerprints, entries,
 * processes, feature updates, known-prevalence, asn prefixes, disabled,
 * distinct process names} */
MFP_EXPORT int mfp_resource_stats(const char *path, uint64_t out[8]);
MFP_EXPORT int mfp_resource_stats_ex(const char *path, const uint8_t *enc_key, uint64_t out[8]);   /* keyed archive */

/* host only (tests): server_identifier::get_normalized_domain_name (the
 * normalisation the device applies to server names); returns the length */
MFP_EXPORT int mfp_normalize_server_name(const char *name, size_t len, char *out, size_t cap);

/* host only (tests): the archive's subnet tries (pyasn.db, domain mappings)
 * built exactly as the device gets them -- the reference's LC-tries
 * (lctrie/lctrie.hpp) -- and queried with the device's lct_find: per
 * "dst_ip<TAB>server_name" line of `queries`, asn[i] = get_asn_info(dst_ip)
 * and fake[i] = is_domain_faking(server_name, dst_ip) (addr.cc:172-208,
 * 707-792; no name: 0).  Returns the lines answered (<= cap), -1 on error. */
MFP_EXPORT long long mfp_lpm_query(const char *resources, const char *queries, uint32_t *asn, int8_t *fake,
                                   size_t cap);

/* ---- per-kernel timing (bench.py's roofline; the rocprofv3 cross-check) ----
 * on != 0: from now on every kernel launch of this context is bracketed by
 * HIP events recorded on its launch stream (totals reset); on == 0: off. */
MFP_EXPORT int mfp_profile_enable(mfp_context ctx, int on);

/* Kernel i (first-launch order) since mfp_profile_enable: its name
 * ("k_classify", "k_fingerprint/<bin>", "k_wave_fp/<bin>", "k_analyze", ...),
 * launch count and summed duration in ms.  Waits for the recorded events.
 * Returns 0, 1 when i is past the last kernel, or a negative error. */
MFP_EXPORT int mfp_profile_read(mfp_context ctx, uint32_t i, char *name, size_t cap, uint64_t *launches,
                                double *total_ms);

/* ---- host ingest into batch arenas (host only, no device needed) ---- */
typedef struct mfp_pcap_s *mfp_pcap;

/* Replaces pcap_file_open (src/pcap_file_io.c:106-254) for reading: classic
 * pcap only (magic a1b2c3d4 / d4c3b2a1); pcap-ng, other magics and link types
 * outside {0, 1, 9, 101, 113, 276} fail with mfp_last_error() set (the
 * reference exits).  A byte-swapped file's link type is the reference's
 * htons() of the 32-bit header field (pcap_file_io.c:236). */
MFP_EXPORT mfp_pcap mfp_pcap_open(const char *path);
MFP_EXPORT int mfp_pcap_linktype(mfp_pcap p);

/* Replaces the pcap_file_read_packet loop (pcap_file_io.c:393-468, 470-512):
 * up to max_pkts packets back to back into arena, followed by 16 zero bytes,
 * one descriptor each (offset, caplen, the file's link type); ts_ns
 * (optional) gets tv_sec * 1e9 + tv_usec * 1000.  A record longer than 65536
 * bytes yields its first 65536 (the reference's BUFLEN).  A record that does
 * not fit the remaining arena starts the next batch.  Returns the packet count
 * (0 at end of file) or -1 on a read error (after the packets before it have
 * been returned); *arena_used = packet bytes written. */
MFP_EXPORT long long mfp_pcap_read_batch(mfp_pcap p, uint8_t *arena, size_t arena_cap, mfp_pkt_desc *desc,
                                         size_t max_pkts, uint64_t *ts_ns, size_t *arena_used);
MFP_EXPORT void mfp_pcap_close(mfp_pcap p);

/* Replaces process_all_packets_in_block (src/af_packet_v3.c:174-210):
 * descriptors for the packets of one TPACKET_V3 ring block, offsets relative
 * to arena_base (zero copy: the mapped ring is the arena), caplen =
 * tp_snaplen, link type Ethernet; ts_ns (optional) = tp_sec * 1e9 + tp_nsec.
 * Returns the packet count, or -1 when a header or packet lies outside
 * block_len or the block holds more than max_pkts packets. */
MFP_EXPORT long long mfp_tpacket3_block(const uint8_t *arena_base, const uint8_t *block, size_t block_len,
                                        mfp_pkt_desc *desc, size_t max_pkts, uint64_t *ts_ns);

/* ---- JSON records (host only, no device needed) ----
 * Replaces the record text of stateful_pkt_proc::write_json
 * (pkt_proc.cc:1157-1253, metadata_output off, no --analysis object;
 * "encapsulations" arrays, QUIC "tls"/"quic" objects included): one
 * line per record with MFP_FLAG_EMIT, byte-identical to the reference, built
 * from records + packet arena + fp arena as mfp_process_batch_host /
 * mfp_process_pipelined return them.  ts_ns (optional): per-packet time; 0 or
 * NULL = now (pkt_proc.cc:1086-1089).  line_end[i] = end offset of packet
 * i's line in out (its line is [line_end[i-1], line_end[i]), empty when the
 * reference writes nothing).  *skipped (optional) = emitted records this
 * writer cannot rebuild (a QUIC record without its sidecar, i.e. fingerprinted
 * in MFP_MODE_ANALYSIS, or an encapsulation chain the host walk cannot
 * follow); they get an empty line.  `threads` host threads.
 * Returns the bytes written, -1 on bad arguments, -2 when out_cap is too
 * small (nothing written; mfp_last_error() names the size needed). */
MFP_EXPORT long long mfp_write_json_batch(const uint8_t *arena, const mfp_pkt_desc *desc, size_t n,
                                          const mfp_record *rec, const char *fp_arena, const uint64_t *ts_ns,
                                          char *out, size_t out_cap, uint64_t *line_end, uint64_t *skipped,
                                          int threads);

/* mfp_write_json_batch with --analysis: records whose analysis has
 * MFP_AN_VALID get the "analysis" object (analysis_result::write_json
 * result.h:207-252, placed as pkt_proc.cc:1211-1213 places it), with names,
 * os_info and attribute names from ctx (the context that classified the
 * batch; mfp_analysis_enabled).  analysis: the batch's n results; attr_prob:
 * as mfp_process_batch_host_ex returned it (NULL only when no record carries
 * an archive tag). */
MFP_EXPORT long long mfp_write_json_batch_analysis(mfp_context ctx, const uint8_t *arena, const mfp_pkt_desc *desc,
                                                   size_t n, const mfp_record *rec, const char *fp_arena,
                                                   const mfp_analysis *analysis, const double *attr_prob,
                                                   const uint64_t *ts_ns, char *out, size_t out_cap,
                                                   uint64_t *line_end, uint64_t *skipped, int threads);

/* last error string for this thread */
MFP_EXPORT const char *mfp_last_error(void);

/* version: 0x00MMmmpp of the reference semantics implemented (2.18.0) */
MFP_EXPORT uint32_t mfp_reference_version(void);

#ifdef __cplusplus
}
#endif
#endif
