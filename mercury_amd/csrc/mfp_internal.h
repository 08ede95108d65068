// mfp_internal.h -- declarations shared by the host translation units of
// libmercury_amd.so (not part of the public C-ABI).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include <atomic>
#include <string>

#include "../../include/mfp.h"

void mfp_set_error(const char *fmt, ...);
bool mfp_parse_config(const char *cfg, uint32_t &sel, uint32_t &tls_format, std::string *resources, bool *analysis,
                      bool *reassembly, uint32_t *block = nullptr, std::string *warn = nullptr,
                      int *report_os = nullptr);
int mfp_set_config(mfp_context c, uint32_t select, uint32_t tls_format, uint32_t mode);
uint32_t mfp_context_mode(mfp_context c);   // MFP_MODE_*

// kernel strategies of the fingerprint pass (mfp_kernels.hip)
// BINNED: classify, then a kernel per protocol bin; LANE: one HBM lane walker
// over the whole batch; SMALL (small batches, the per-packet API): one
// LDS-staged walker over the whole batch (no classify pass, the packets'
// dependent reads are LDS round trips), then the fallback lane
enum { MFP_STRATEGY_BINNED = 0, MFP_STRATEGY_LANE = 2, MFP_STRATEGY_SMALL = 3 };

// per-kernel HIP-event timing (mfp_profile_enable): the launchers bracket
// every launch with begin/end when `p` is non-null
struct mfp_prof;
void mfp_prof_begin(mfp_prof *p, const char *kernel, hipStream_t s);
void mfp_prof_end(mfp_prof *p, hipStream_t s);

// the total length of the context's attribute names (computed once; mfp_json.cpp's bounds)
size_t mfp_attribute_names_len(mfp_context c);

// (D)TLS ClientHello records with MFP_XF_TLS_UA: the ALPN list re-read from
// the packet (mfp_json.cpp)
bool mfp_hello_alpn(const uint8_t *pkt, uint32_t caplen, const mfp_record &r, const uint8_t **alpn, uint32_t *len);
// mfp_process_batch_host_ex for the per-packet shim's small batches, whose
// buffers are all page-locked (mfp_host.cpp)
long long mfp_process_small_pinned(mfp_context c, const uint8_t *arena, size_t arena_len, const mfp_pkt_desc *desc,
                                   size_t n, mfp_record *rec, char *fp_arena, size_t fp_cap, mfp_analysis *analysis,
                                   double *attr_prob);

// the JSON writer (mfp_json.cpp) handing its text to a sink in packet order:
// the batch packet processors (mfp_pktproc.cpp); props / analysis optional
typedef int (*mfp_json_sink)(void *user, const void *data, size_t len);
long long mfp_write_json_to_sink(mfp_context ctx, const uint16_t *props, const uint8_t *arena, const mfp_pkt_desc *desc,
                                 size_t n, const mfp_record *rec, const char *fp_arena, const mfp_analysis *analysis,
                                 const double *attr_prob, const uint64_t *ts_ns, uint64_t *line_end, uint64_t *skipped,
                                 int threads, mfp_json_sink sink, void *user);

// A launch-shape value computed once per device (occupancy x CUs): cached per
// hipGetDevice index, so contexts on different devices of one process each get
// their own device's value (0 in a slot means not computed yet)
template <class F>
inline uint64_t mfp_per_device(std::atomic<uint64_t> (&cache)[64], F compute) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return (uint64_t)compute();
    }
    uint64_t v = cache[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        v = (uint64_t)compute() + 1;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v - 1;
}
