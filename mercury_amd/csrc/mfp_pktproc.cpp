// mfp_pktproc.cpp -- the batch packet processors behind the reference's
// pkt_proc plugin interface (src/pkt_proc.hpp:26-33); include/mfp_pkt_proc.h
// states the contract.
//
// The reference's processors do all their work inside apply(), one packet at a
// time, and put each record on a lock-free queue for the output thread
// (pkt_proc_json_writer_llq, pkt_proc_filter_pcap_writer_llq,
// src/pkt_processing.h:129-173,230-259).  Here apply() only copies the packet
// into a page-locked arena; whole batches then go through three stages on
// three threads, each batch in stream order:
//
//   caller (apply)  -> fills batch k+2
//   device thread   -> batch k+1: mfp_process_pipelined (copies in, bin kernels,
//                      classifier, copies out), or the reassembler's batch call
//   writer thread   -> batch k:   JSON text (mfp_write_json_to_sink, 16 host
//                      threads) or pcap records, to the sink
//
// so the device, the host's JSON rendering and the capture loop overlap.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mfp_pkt_proc.h"
#include "mfp_internal.h"

namespace {

// page-locked buffer of T, grown (never shrunk) on demand
template <class T>
struct Pinned {
    T *p = nullptr;
    size_t cap = 0;
    bool reserve(size_t n) {
        if (n <= cap) return true;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t nc = std::max(n, cap + cap / 2);
        if (hipHostMalloc((void **)&p, nc * sizeof(T), hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return false;
        }
        cap = nc;
        return true;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

constexpr size_t kPad = 64;   // zero bytes behind the last packet (the walkers read aligned 16-byte blocks)

struct Batch {
    Pinned<uint8_t> arena;              // packets back to back, then kPad zero bytes
    size_t used = 0;                    // packet bytes
    Pinned<mfp_pkt_desc> desc;
    std::vector<uint64_t> ts_ns;        // JSON event_start (0 = now)
    std::vector<uint32_t> ts_sec, ts_usec;   // the pcap record's timestamp (pcap_queue_write)
    size_t n = 0;
    std::chrono::steady_clock::time_point first;   // when its first packet was applied
    // device results
    Pinned<mfp_record> rec;
    Pinned<char> fp;
    Pinned<mfp_analysis> an;
    Pinned<double> ap;
    std::vector<uint16_t> props;        // reassembly properties
    std::vector<mfp_pkt_desc> out_desc; // reassembly: desc with the rebuilt frames
    std::vector<uint8_t> merged;        // reassembly: arena ++ frames (the JSON writer's input)
    std::vector<uint8_t> dump;          // reassembly: dump_pkt per packet
    std::vector<uint64_t> line_end;
    std::vector<uint8_t> out;           // pcap records
    bool reassembled = false, analysed = false;

    void release() {
        arena.release(); desc.release(); rec.release(); fp.release(); an.release(); ap.release();
    }
};

}  // namespace

struct mfp_pkt_proc_s {
    mfp_context ctx = nullptr;
    int kind = MFP_PKT_PROC_JSON;
    mfp_pkt_proc_opts o{};
    mfp_sink_fn sink = nullptr;
    void *user = nullptr;
    bool reassembly = false, analysis = false;
    mfp_reassembler R = nullptr;

    static constexpr int NB = 3;
    Batch b[NB];
    int fill = 0;                        // the batch apply() fills
    std::mutex mu;
    std::condition_variable cv;
    std::deque<int> q_dev, q_out, q_free;
    uint64_t submitted = 0, written = 0; // batches handed over / finished by the writer
    bool stop = false;
    std::atomic<int> err{0};             // first error (negative), sticky
    std::string errmsg;
    std::thread t_dev, t_out;
    // counters (MFP_PKT_PROC_NSTATS)
    std::atomic<uint64_t> st_pkts{0}, st_batches{0}, st_records{0}, st_bytes{0}, st_dev_ns{0}, st_out_ns{0},
        st_skipped{0};

    void fail(int code, const std::string &m) {   // under mu
        if (!err) { err = code; errmsg = m; }
        cv.notify_all();
    }
};

static int report(mfp_pkt_proc p) {   // the sticky error, made this thread's last error (under mu)
    mfp_set_error("%s", p->errmsg.c_str());
    return p->err.load();
}

static uint64_t ns_since(std::chrono::steady_clock::time_point t0) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// the device stage of one batch; returns 0 or a negative error (message set)
static int device_stage(mfp_pkt_proc p, Batch &B) {
    const size_t n = B.n;
    memset(B.arena.p + B.used, 0, kPad);
    if (!B.rec.reserve(n + 1)) { mfp_set_error("page-locked allocation failed (records)"); return -2; }
    // fingerprint arena: the packed strings of the batch, and with reassembly
    // the rebuilt messages' (at most one frame of <= 8 KiB + headers per packet)
    size_t fp_cap = mfp_fp_arena_bound(n, B.used);
    if (p->reassembly) fp_cap += mfp_fp_arena_bound(n, n * (size_t)8400);
    if (!B.fp.reserve(fp_cap)) { mfp_set_error("page-locked allocation failed (fingerprints)"); return -2; }
    // the filtered pcap writer needs only which packets write a record: the
    // classifier's objects never decide that (pkt_proc.cc:1195-1253)
    const bool an = p->analysis && p->kind == MFP_PKT_PROC_JSON;
    if (an && (!B.an.reserve(n + 1) || !B.ap.reserve((n + 1) * MFP_ATTR_DB_TAGS))) {
        mfp_set_error("page-locked allocation failed (analysis)");
        return -2;
    }
    B.analysed = an;
    B.reassembled = p->reassembly;
    long long used;
    if (p->reassembly) {
        B.props.resize(n + 1);
        B.out_desc.resize(n + 1);
        if (an)
            used = mfp_process_batch_reassembly_analysis(p->ctx, p->R, B.arena.p, B.used + kPad, B.desc.p, n,
                                                         B.ts_ns.data(), B.rec.p, B.fp.p, fp_cap, B.props.data(),
                                                         B.out_desc.data(), B.an.p, B.ap.p);
        else
            used = mfp_process_batch_reassembly(p->ctx, p->R, B.arena.p, B.used + kPad, B.desc.p, n, B.ts_ns.data(),
                                                B.rec.p, B.fp.p, fp_cap, B.props.data(), B.out_desc.data());
        if (used < 0) return (int)used;
        // the reassembler's frames and flags live until its next call, which the
        // next batch makes while this one is being written: keep copies
        size_t fl = 0, nd = 0;
        const uint8_t *fr = mfp_reassembler_frames(p->R, &fl);
        const uint8_t *dm = mfp_reassembler_dumped(p->R, &nd);
        if (p->kind == MFP_PKT_PROC_JSON) {
            B.merged.resize(B.used + kPad + fl + kPad);
            memcpy(B.merged.data(), B.arena.p, B.used + kPad);
            if (fl) memcpy(B.merged.data() + B.used + kPad, fr, fl);
            memset(B.merged.data() + B.used + kPad + fl, 0, kPad);
        }
        B.dump.assign(n, 0);
        if (dm && nd == n) memcpy(B.dump.data(), dm, n);
    } else {
        used = mfp_process_pipelined(p->ctx, B.arena.p, B.used + kPad, B.desc.p, n, B.rec.p, B.fp.p, fp_cap,
                                     an ? B.an.p : nullptr, an ? B.ap.p : nullptr, p->o.chunk);
        if (used < 0) return (int)used;
    }
    return 0;
}

static int sink_call(void *u, const void *d, size_t len) {
    mfp_pkt_proc p = (mfp_pkt_proc)u;
    const int r = p->sink(p->user, d, len);
    if (r == 0) p->st_bytes += len;   // (the writer thread only)
    return r;
}

// the writer stage: the batch's output, in packet order, to the sink
static int output_stage(mfp_pkt_proc p, Batch &B) {
    const size_t n = B.n;
    if (p->kind == MFP_PKT_PROC_JSON) {
        B.line_end.resize(n + 1);
        uint64_t skipped = 0;
        const uint8_t *arena = B.reassembled ? B.merged.data() : B.arena.p;
        const mfp_pkt_desc *desc = B.reassembled ? B.out_desc.data() : B.desc.p;
        const long long r = mfp_write_json_to_sink(p->ctx, B.reassembled ? B.props.data() : nullptr, arena, desc, n, B.rec.p,
                                                   B.fp.p, B.analysed ? B.an.p : nullptr, B.analysed ? B.ap.p : nullptr,
                                                   B.ts_ns.data(), B.line_end.data(), &skipped,
                                                   p->o.json_threads, sink_call, p);
        if (r < 0) return (int)r;
        uint64_t lines = 0, prev = 0;
        for (size_t i = 0; i < n; i++) { lines += B.line_end[i] != prev; prev = B.line_end[i]; }
        p->st_records += lines;
        p->st_skipped += skipped;
        return 0;
    }
    // filtered pcap: the packets that wrote a record or fed the reassembler
    // (pkt_processing.h:250-256), each as pcap_queue_write lays it out
    size_t bytes = 0, m = 0;
    for (size_t i = 0; i < n; i++)
        if ((B.rec.p[i].flags & MFP_FLAG_EMIT) || (B.reassembled && B.dump[i])) { bytes += 16 + B.desc.p[i].caplen; m++; }
    if (!m) return 0;
    B.out.resize(bytes);
    uint8_t *o = B.out.data();
    for (size_t i = 0; i < n; i++) {
        if (!((B.rec.p[i].flags & MFP_FLAG_EMIT) || (B.reassembled && B.dump[i]))) continue;
        const uint32_t len = B.desc.p[i].caplen;
        const uint32_t h[4] = {B.ts_sec[i], B.ts_usec[i], len, len};   // ts_sec, ts_usec, incl_len, orig_len
        memcpy(o, h, 16);
        memcpy(o + 16, B.arena.p + B.desc.p[i].offset, len);
        o += 16 + len;
    }
    p->st_records += m;
    if (sink_call(p, B.out.data(), bytes) != 0) { mfp_set_error("pcap output: the sink failed"); return -5; }
    return 0;
}

static void device_loop(mfp_pkt_proc p) {
    std::unique_lock<std::mutex> lk(p->mu);
    for (;;) {
        p->cv.wait(lk, [&] { return p->stop || !p->q_dev.empty(); });
        if (p->q_dev.empty()) return;   // stop
        const int k = p->q_dev.front();
        p->q_dev.pop_front();
        const bool ok = !p->err;
        lk.unlock();
        int r = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (ok && p->b[k].n) r = device_stage(p, p->b[k]);
        const uint64_t dt = ns_since(t0);
        const std::string m = r ? std::string(mfp_last_error()) : std::string();
        lk.lock();
        p->st_dev_ns += dt;
        if (r) p->fail(r, m);
        p->q_out.push_back(k);
        p->cv.notify_all();
    }
}

static void output_loop(mfp_pkt_proc p) {
    std::unique_lock<std::mutex> lk(p->mu);
    for (;;) {
        p->cv.wait(lk, [&] { return p->stop || !p->q_out.empty(); });
        if (p->q_out.empty()) return;
        const int k = p->q_out.front();
        p->q_out.pop_front();
        const bool ok = !p->err;
        lk.unlock();
        int r = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (ok && p->b[k].n) r = output_stage(p, p->b[k]);
        const uint64_t dt = ns_since(t0);
        const std::string m = r ? std::string(mfp_last_error()) : std::string();
        lk.lock();
        p->st_out_ns += dt;
        if (p->b[k].n) p->st_batches++;
        if (r) p->fail(r, m);
        p->b[k].n = 0;
        p->b[k].used = 0;
        p->written++;
        p->q_free.push_back(k);
        p->cv.notify_all();
    }
}

// hand the filling batch to the device thread and take a free one (waits
// while all three are in flight); under mu
static int submit_locked(mfp_pkt_proc p, std::unique_lock<std::mutex> &lk) {
    if (p->b[p->fill].n == 0) return 0;
    p->q_dev.push_back(p->fill);
    p->submitted++;
    p->cv.notify_all();
    p->cv.wait(lk, [&] { return !p->q_free.empty() || p->err; });
    if (p->q_free.empty()) { p->fill = -1; return p->err.load(); }
    p->fill = p->q_free.front();
    p->q_free.pop_front();
    return 0;
}

extern "C" MFP_EXPORT size_t mfp_pcap_file_header(uint8_t out[24]) {
    // struct pcap_file_hdr (pcap_file_io.c:41-49) as write_pcap_file_header fills it
    const uint32_t magic = 0xa1b2c3d4u, zone = 0, sigfigs = 0, snaplen = 65535, network = 1;
    const uint16_t major = 2, minor = 4;
    memcpy(out, &magic, 4); memcpy(out + 4, &major, 2); memcpy(out + 6, &minor, 2);
    memcpy(out + 8, &zone, 4); memcpy(out + 12, &sigfigs, 4); memcpy(out + 16, &snaplen, 4); memcpy(out + 20, &network, 4);
    return 24;
}

extern "C" MFP_EXPORT mfp_pkt_proc mfp_pkt_proc_create(mfp_context ctx, int kind, const mfp_pkt_proc_opts *opts,
                                                       mfp_sink_fn sink, void *user) {
    if (!ctx || !sink) { mfp_set_error("mfp_pkt_proc_create: null context or sink"); return nullptr; }
    if (kind != MFP_PKT_PROC_JSON && kind != MFP_PKT_PROC_FILTER_PCAP) {
        mfp_set_error("mfp_pkt_proc_create: unknown kind %d", kind);
        return nullptr;
    }
    if (mfp_context_mode(ctx) != MFP_MODE_WRITE_JSON) {
        mfp_set_error("mfp_pkt_proc_create: the context must be created with MFP_MODE_WRITE_JSON (write_json semantics)");
        return nullptr;
    }
    auto *p = new mfp_pkt_proc_s;
    p->ctx = ctx;
    p->kind = kind;
    if (opts) p->o = *opts;
    if (!p->o.batch_pkts) p->o.batch_pkts = 131072;
    if (!p->o.arena_bytes) p->o.arena_bytes = std::max<size_t>((size_t)64 << 20, p->o.batch_pkts * 1024);
    p->o.arena_bytes = std::min<size_t>(p->o.arena_bytes, (size_t)2 << 30);
    p->o.arena_bytes = std::max<size_t>(p->o.arena_bytes, 65536 + 16);   // any one packet fits
    if (p->o.json_threads <= 0) p->o.json_threads = 16;
    p->sink = sink;
    p->user = user;
    p->reassembly = mfp_reassembly_enabled(ctx) != 0;
    p->analysis = mfp_analysis_enabled(ctx) != 0;
    if (p->reassembly) p->R = mfp_reassembler_create();
    // every page-locked buffer up front (pinning gigabytes takes a while: not in
    // the capture loop's path); the fingerprint arena by its bound for a full batch
    size_t fp_cap = mfp_fp_arena_bound(p->o.batch_pkts, p->o.arena_bytes);
    if (p->reassembly) fp_cap += mfp_fp_arena_bound(p->o.batch_pkts, p->o.batch_pkts * (size_t)8400);
    const bool an = p->analysis && kind == MFP_PKT_PROC_JSON;
    for (int k = 0; k < mfp_pkt_proc_s::NB; k++) {
        Batch &B = p->b[k];
        if (!B.arena.reserve(p->o.arena_bytes + kPad) || !B.desc.reserve(p->o.batch_pkts + 1) ||
            !B.rec.reserve(p->o.batch_pkts + 1) || !B.fp.reserve(fp_cap) ||
            (an && (!B.an.reserve(p->o.batch_pkts + 1) || !B.ap.reserve((p->o.batch_pkts + 1) * MFP_ATTR_DB_TAGS)))) {
            for (auto &x : p->b) x.release();
            if (p->R) mfp_reassembler_destroy(p->R);
            delete p;
            mfp_set_error("mfp_pkt_proc_create: page-locked allocation of the batch arenas failed");
            return nullptr;
        }
        B.ts_ns.reserve(p->o.batch_pkts);
        B.ts_sec.reserve(p->o.batch_pkts);
        B.ts_usec.reserve(p->o.batch_pkts);
        if (k) p->q_free.push_back(k);
    }
    p->fill = 0;
    p->t_dev = std::thread(device_loop, p);
    p->t_out = std::thread(output_loop, p);
    return p;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_apply(mfp_pkt_proc p, int64_t tv_sec, int64_t tv_nsec, uint32_t caplen,
                                             uint32_t len, uint16_t linktype, const uint8_t *packet) {
    if (!p) { mfp_set_error("null processor"); return -1; }
    if (p->err) { std::lock_guard<std::mutex> lk(p->mu); return report(p); }
    const uint32_t L = std::min(len, caplen);
    if (L && !packet) { mfp_set_error("null packet"); return -1; }
    if (L > p->o.arena_bytes) {   // (no batch could hold it; the readers cap records at 65 536 bytes)
        mfp_set_error("a %u-byte packet is larger than the %zu-byte batch arena", L, p->o.arena_bytes);
        return -1;
    }
    Batch *B = &p->b[p->fill];
    if (B->n == p->o.batch_pkts || B->used + L > p->o.arena_bytes ||
        (p->o.flush_us && B->n && (B->n & 63) == 0 &&
         std::chrono::steady_clock::now() - B->first > std::chrono::microseconds(p->o.flush_us))) {
        std::unique_lock<std::mutex> lk(p->mu);
        if (submit_locked(p, lk)) return report(p);
        B = &p->b[p->fill];
    }
    if (B->n == 0) {
        if (p->o.flush_us) B->first = std::chrono::steady_clock::now();
        B->ts_ns.clear(); B->ts_sec.clear(); B->ts_usec.clear();
    }
    // the filtered pcap writer runs the processor's Ethernet write_json
    // whatever the packet's link type (pkt_processing.h:250)
    const uint16_t lt = p->kind == MFP_PKT_PROC_FILTER_PCAP ? (uint16_t)1 : linktype;
    B->desc.p[B->n] = mfp_pkt_desc{B->used, L, lt, 0};
    if (L) memcpy(B->arena.p + B->used, packet, L);
    B->used += L;
    B->ts_ns.push_back(tv_sec == 0 ? 0ull : (uint64_t)tv_sec * 1000000000ull + (uint64_t)tv_nsec);
    B->ts_sec.push_back((uint32_t)tv_sec);
    B->ts_usec.push_back((uint32_t)(tv_nsec / 1000));
    B->n++;
    p->st_pkts++;
    return 0;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_apply_batch(mfp_pkt_proc p, const uint8_t *arena, const mfp_pkt_desc *desc,
                                                   size_t n, const uint64_t *ts_ns) {
    if (!p || (n && (!arena || !desc))) { mfp_set_error("null argument"); return -1; }
    for (size_t i = 0; i < n; i++) {
        const uint64_t t = ts_ns ? ts_ns[i] : 0;
        const int r = mfp_pkt_proc_apply(p, (int64_t)(t / 1000000000ull), (int64_t)(t % 1000000000ull), desc[i].caplen,
                                         desc[i].caplen, desc[i].linktype, arena + desc[i].offset);
        if (r) return r;
    }
    return 0;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_flush(mfp_pkt_proc p) {
    if (!p) { mfp_set_error("null processor"); return -1; }
    std::unique_lock<std::mutex> lk(p->mu);
    if (p->err) return report(p);
    if (submit_locked(p, lk)) return report(p);
    return 0;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_drain(mfp_pkt_proc p) {
    if (!p) { mfp_set_error("null processor"); return -1; }
    std::unique_lock<std::mutex> lk(p->mu);
    if (!p->err && submit_locked(p, lk)) return report(p);
    p->cv.wait(lk, [&] { return p->written == p->submitted; });
    if (p->err) return report(p);
    return 0;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_finalize(mfp_pkt_proc p) {
    const int r = mfp_pkt_proc_drain(p);
    if (r) return r;
    if (p->R) {   // tcp_reassembler::clear_all: a fresh flow table
        mfp_reassembler_destroy(p->R);
        p->R = mfp_reassembler_create();
    }
    return 0;
}

extern "C" MFP_EXPORT void mfp_pkt_proc_destroy(mfp_pkt_proc p) {
    if (!p) return;
    {
        std::unique_lock<std::mutex> lk(p->mu);
        // batches already handed over finish (their buffers may be in use by
        // a HIP copy); nothing new is taken
        p->cv.wait(lk, [&] { return p->written == p->submitted; });
        p->stop = true;
        p->cv.notify_all();
    }
    p->t_dev.join();
    p->t_out.join();
    for (auto &B : p->b) B.release();
    if (p->R) mfp_reassembler_destroy(p->R);
    delete p;
}

extern "C" MFP_EXPORT int mfp_pkt_proc_stats(mfp_pkt_proc p, uint64_t *out, size_t n) {
    if (!p || (n && !out)) { mfp_set_error("null argument"); return -1; }
    std::lock_guard<std::mutex> lk(p->mu);
    const uint64_t v[MFP_PKT_PROC_NSTATS] = {p->st_pkts.load(), p->st_batches.load(), p->st_records.load(),
                                             p->st_bytes.load(), p->st_dev_ns.load(), p->st_out_ns.load(),
                                             p->st_skipped.load()};
    for (size_t i = 0; i < n && i < MFP_PKT_PROC_NSTATS; i++) out[i] = v[i];
    return 0;
}
