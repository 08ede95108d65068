// mercury_amd_pkt_proc.hpp -- pkt_proc subclasses over the batch packet
// processors of include/mfp_pkt_proc.h: the two processors the reference's
// factory builds (pkt_proc_new_from_config, src/pkt_processing.cc:14-52),
// with the device path behind them.
//
//   pkt_proc_gpu_json_writer          in place of pkt_proc_json_writer_llq
//                                     (src/pkt_processing.h:129-173)
//   pkt_proc_gpu_filter_pcap_writer   in place of pkt_proc_filter_pcap_writer[_llq]
//                                     (src/pkt_processing.h:92-121,230-259)
//
// Inside the mercury tree (-I src) this header derives from the reference's
// own struct pkt_proc (src/pkt_proc.hpp:26-33); outside it (this
// repository's driver, mercury_amd/csrc/mfp_drv.cpp) it declares the same two
// structs itself, with the same members, so code written against one compiles
// against the other.
#ifndef MERCURY_AMD_PKT_PROC_HPP
#define MERCURY_AMD_PKT_PROC_HPP

#include <stdio.h>
#include <time.h>

#include <stdexcept>
#include <string>

#include "mfp_pkt_proc.h"

#if __has_include("pkt_proc.hpp")
#if __has_include("libmerc/libmerc.h")
#include "libmerc/libmerc.h"   // mercury_context, which pkt_proc.hpp's factory declaration names
#endif
#include "pkt_proc.hpp"
#else
// the plugin interface of src/pkt_proc.hpp:10-33 (packet_info, pkt_proc)
struct packet_info {
    struct timespec ts;
    uint32_t caplen;
    uint32_t len;
    uint16_t linktype = 1;   // LINKTYPE_ETHERNET
};
struct pkt_proc {
    virtual void apply(struct packet_info *pi, uint8_t *eth) = 0;
    virtual void flush() = 0;
    virtual void finalize() = 0;
    virtual ~pkt_proc() {}
    size_t bytes_written = 0;
    size_t packets_written = 0;
};
#endif

namespace mercury_amd {

// a FILE* as the processors' sink (the output file the reference's output
// thread writes, src/output.c)
inline int file_sink(void *f, const void *data, size_t len) {
    return fwrite(data, 1, len, (FILE *)f) == len ? 0 : -1;
}

// the classic pcap file header of a `mercury -w` output file
// (write_pcap_file_header src/pcap_file_io.c:88-104)
inline bool write_pcap_header(FILE *f) {
    uint8_t h[24];
    mfp_pcap_file_header(h);
    return fwrite(h, 1, sizeof h, f) == sizeof h;
}

// the common part: a batch processor of one kind; errors throw, as the
// reference's processors throw from their constructors
// (pkt_processing.h:162-165) -- a silently dropped batch would be worse
class gpu_batch_proc : public pkt_proc {
public:
    gpu_batch_proc(mfp_context ctx, int kind, mfp_sink_fn sink, void *user, const mfp_pkt_proc_opts *opts)
        : p_{mfp_pkt_proc_create(ctx, kind, opts, sink, user)} {
        if (!p_) throw std::runtime_error(std::string("mercury_amd: ") + mfp_last_error());
    }
    ~gpu_batch_proc() override { mfp_pkt_proc_destroy(p_); }
    gpu_batch_proc(const gpu_batch_proc &) = delete;
    gpu_batch_proc &operator=(const gpu_batch_proc &) = delete;

    void apply(struct packet_info *pi, uint8_t *eth) override {
        check(mfp_pkt_proc_apply(p_, (int64_t)pi->ts.tv_sec, (int64_t)pi->ts.tv_nsec, pi->caplen, pi->len,
                                 pi->linktype, eth));
    }
    void flush() override { check(mfp_pkt_proc_flush(p_)); }
    // a whole block of packets (mfp_pkt_proc_apply_batch)
    void apply_batch(const uint8_t *arena, const mfp_pkt_desc *desc, size_t n, const uint64_t *ts_ns) {
        check(mfp_pkt_proc_apply_batch(p_, arena, desc, n, ts_ns));
    }
    void finalize() override { check(mfp_pkt_proc_finalize(p_)); }

    // [MFP_PKT_PROC_NSTATS] counters (include/mfp_pkt_proc.h)
    void stats(uint64_t *out) const { mfp_pkt_proc_stats(p_, out, MFP_PKT_PROC_NSTATS); }

private:
    static void check(int r) {
        if (r) throw std::runtime_error(std::string("mercury_amd: ") + mfp_last_error());
    }
    mfp_pkt_proc p_;
};

// JSON records, in place of pkt_proc_json_writer_llq
class pkt_proc_gpu_json_writer : public gpu_batch_proc {
public:
    pkt_proc_gpu_json_writer(mfp_context ctx, mfp_sink_fn sink, void *user, const mfp_pkt_proc_opts *opts = nullptr)
        : gpu_batch_proc(ctx, MFP_PKT_PROC_JSON, sink, user, opts) {}
    pkt_proc_gpu_json_writer(mfp_context ctx, FILE *out, const mfp_pkt_proc_opts *opts = nullptr)
        : gpu_batch_proc(ctx, MFP_PKT_PROC_JSON, file_sink, out, opts) {}
};

// selected packets in pcap format, in place of pkt_proc_filter_pcap_writer[_llq]
// (the file header is the output file's: write_pcap_header when it is opened)
class pkt_proc_gpu_filter_pcap_writer : public gpu_batch_proc {
public:
    pkt_proc_gpu_filter_pcap_writer(mfp_context ctx, mfp_sink_fn sink, void *user,
                                    const mfp_pkt_proc_opts *opts = nullptr)
        : gpu_batch_proc(ctx, MFP_PKT_PROC_FILTER_PCAP, sink, user, opts) {}
    pkt_proc_gpu_filter_pcap_writer(mfp_context ctx, FILE *out, const mfp_pkt_proc_opts *opts = nullptr)
        : gpu_batch_proc(ctx, MFP_PKT_PROC_FILTER_PCAP, file_sink, out, opts) {}
};

}  // namespace mercury_amd

#endif
