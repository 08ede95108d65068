/*
 * mfp_pkt_proc.h -- batch packet processors: the C-ABI behind the
 * reference's pkt_proc plugin interface (src/pkt_proc.hpp:26-33), so the
 * `mercury` binary's capture and file readers can hand packets to the
 * MI355X path one at a time, as they do today, while the device sees whole
 * batches.  Plain pointers and sizes only; the C++ pkt_proc subclasses over
 * it are in include/mercury_amd_pkt_proc.hpp.
 *
 * Two kinds, the two the reference's factory builds
 * (pkt_proc_new_from_config, src/pkt_processing.cc:14-52):
 *
 *  MFP_PKT_PROC_JSON         replaces pkt_proc_json_writer_llq
 *                            (src/pkt_processing.h:129-173): one JSON record
 *                            line per packet the reference's
 *                            write_json_linktype writes a record for
 *                            (libmerc.h:293, pkt_proc.cc:1328-1383), in packet
 *                            order, with the packet's capture time as
 *                            event_start; "analysis" objects with
 *                            resources=...;analysis, reassembly_properties with
 *                            "reassembly".
 *  MFP_PKT_PROC_FILTER_PCAP  replaces pkt_proc_filter_pcap_writer[_llq]
 *                            (src/pkt_processing.h:92-121,230-259), `mercury
 *                            -w`: every packet for which the processor's
 *                            Ethernet write_json (pkt_proc.cc:1258-1326; the
 *                            packet's link type is NOT used, as there) writes
 *                            a record, or whose data went into the
 *                            reassembler (dump_pkt, pkt_proc.cc:1842-1845), as
 *                            a classic pcap record (pcap_queue_write
 *                            src/pcap_file_io.c:540-579: ts_sec, ts_usec =
 *                            tv_nsec / 1000, incl_len = orig_len = the length).
 *                            The file header (mfp_pcap_file_header) is the
 *                            output file's, written once by its opener, as
 *                            src/output.c:192 does.
 *
 * apply() copies the packet into a page-locked batch arena.  A full batch
 * (batch_pkts packets or the arena's bytes), flush(), or a batch whose first
 * packet has waited flush_us microseconds (checked in apply) is handed to the
 * processor's device thread, which runs it through the context
 * (mfp_process_pipelined, or mfp_process_batch_reassembly[_analysis] with
 * "reassembly") while apply() fills the next batch; a writer thread then
 * renders the output and calls the sink, batch after batch, in packet order.
 * Three batches are in flight at most (filling, on the device, being
 * written); apply() waits only when all three are taken.
 *
 * The sink is called from the writer thread, never concurrently with itself,
 * with consecutive pieces of the output stream (each a whole number of records);
 * it returns 0, or non-zero to fail the processor (every later call returns
 * -5).  Batches of one processor are processed in stream order (the
 * unknown-TLS prevalence LRU, the reassembler's flow table).
 */
#ifndef MFP_PKT_PROC_H
#define MFP_PKT_PROC_H

#include "mfp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mfp_pkt_proc_s *mfp_pkt_proc;

/* output sink: consecutive bytes of the output stream */
typedef int (*mfp_sink_fn)(void *user, const void *data, size_t len);

enum {
    MFP_PKT_PROC_JSON = 0,
    MFP_PKT_PROC_FILTER_PCAP = 1,
};

typedef struct {
    size_t   batch_pkts;     /* packets per batch (0: 131072)                         */
    size_t   arena_bytes;    /* page-locked bytes per batch arena (0: 1 KiB per packet,
                                at least 64 MiB; at most 2 GiB); a packet that does not
                                fit starts the next batch.  Three batches' arenas and
                                result buffers (the fingerprint arena by
                                mfp_fp_arena_bound) are page-locked at create       */
    uint32_t flush_us;       /* hand a batch over once its first packet waited this
                                long (checked in apply; 0: only when full / flush)   */
    int      json_threads;   /* host threads rendering JSON text (0: 16)              */
    size_t   chunk;          /* mfp_process_pipelined chunk (0: its default)          */
} mfp_pkt_proc_opts;

/* A processor over ctx (created with MFP_MODE_WRITE_JSON; the caller keeps
 * it and finalizes it after the processor).  opts may be NULL.  Several
 * processors may share one context, as the reference's per-thread processors
 * share one mercury_context (the classifier and its prevalence LRU).  Returns
 * NULL on error (mfp_last_error()). */
MFP_EXPORT mfp_pkt_proc mfp_pkt_proc_create(mfp_context ctx, int kind, const mfp_pkt_proc_opts *opts,
                                            mfp_sink_fn sink, void *user);

/* pkt_proc::apply(packet_info *pi, uint8_t *eth): the packet's capture time,
 * caplen bytes at `packet`, its original length and its link type
 * (packet_info, src/pkt_proc.hpp:13-19).  The reference processes pi->len
 * bytes; both of its readers set len = caplen (pcap_file_io.c:464-468,
 * af_packet_v3.c:196-197) except for a pcap record over 65 536 bytes, where
 * it reads past its buffer; here min(len, caplen) bytes are processed and
 * written.  tv_sec == 0 stands for "now" (pkt_proc.cc:1086-1089).  Returns
 * 0, or < 0 after an error (the processor's first error is kept). */
MFP_EXPORT int mfp_pkt_proc_apply(mfp_pkt_proc p, int64_t tv_sec, int64_t tv_nsec, uint32_t caplen, uint32_t len,
                                  uint16_t linktype, const uint8_t *packet);

/* apply() for n packets at once (a TPACKET_V3 block walked by
 * mfp_tpacket3_block, or a block of a pcap file read by mfp_pcap_read_batch:
 * process_all_packets_in_block af_packet_v3.c:174-210 without its per-packet
 * call); ts_ns[i] = tv_sec * 1e9 + tv_nsec (NULL: "now").  Returns 0 or < 0. */
MFP_EXPORT int mfp_pkt_proc_apply_batch(mfp_pkt_proc p, const uint8_t *arena, const mfp_pkt_desc *desc, size_t n,
                                        const uint64_t *ts_ns);

/* pkt_proc::flush(): hand the packets buffered so far to the device thread
 * (the capture loop calls it before it waits, af_packet_v3.c:744-754);
 * does not wait for their output. */
MFP_EXPORT int mfp_pkt_proc_flush(mfp_pkt_proc p);

/* flush and wait until every applied packet's output has gone to the sink. */
MFP_EXPORT int mfp_pkt_proc_drain(mfp_pkt_proc p);

/* pkt_proc::finalize(): drain, then clear the reassembler's flows
 * (stateful_pkt_proc::finalize pkt_proc.h:205-210). */
MFP_EXPORT int mfp_pkt_proc_finalize(mfp_pkt_proc p);

/* stop the threads and free the processor (after finalize, or to abandon it) */
MFP_EXPORT void mfp_pkt_proc_destroy(mfp_pkt_proc p);

/* counters: [0] packets applied, [1] batches processed, [2] records (JSON
 * lines / pcap packets) written, [3] bytes handed to the sink, [4] ns spent
 * on the device thread's batches, [5] ns spent rendering and writing,
 * [6] records the JSON writer could not rebuild (0 on every golden) */
#define MFP_PKT_PROC_NSTATS 7
MFP_EXPORT int mfp_pkt_proc_stats(mfp_pkt_proc p, uint64_t *out, size_t n);

/* the 24-byte classic pcap file header the reference's writer puts first
 * (write_pcap_file_header src/pcap_file_io.c:88-104: magic a1b2c3d4, v2.4,
 * snaplen 65535, LINKTYPE_ETHERNET); returns 24 */
MFP_EXPORT size_t mfp_pcap_file_header(uint8_t out[24]);

#ifdef __cplusplus
}
#endif
#endif
