// mfp_kernels.hip -- k_classify (the protocol bins) and the fingerprint
// launcher: k_classify, then one launch per bin through the per-family
// launchers (mfp_k_*.hip; kernels in mfp_kernels.hpp), the fallback lane, k_quic.
#include <hip/hip_runtime.h>

#include "mfp_kernels.hpp"

namespace mfp {

// protocol bins of the classify pass: each bin is then fingerprinted by its
// own k_fingerprint launch over a compact index list, so the lanes of a wave
// walk the same protocol (same parser, similar loop trip counts)
constexpr int NBINS = 9;
constexpr int QUIC_BIN = 8;   // run by k_quic after every other bin (mfp_quic.hip)
DEV int msg_bin(uint32_t msg) {
    switch (msg) {
    case MFP_MSG_TLS_CH: return 0;
    case MFP_MSG_HTTP_REQ: return 1;
    case MFP_MSG_TCP_SYN: case MFP_MSG_TCP_SYNACK: return 2;
    case MFP_MSG_HTTP_RESP: return 3;
    case MFP_MSG_TLS_SH: case MFP_MSG_TLS_CERT: return 5;
    case MFP_MSG_SSH_INIT: case MFP_MSG_SSH_KEX: return 6;
    case MFP_MSG_DTLS_CH: case MFP_MSG_DTLS_SH: case MFP_MSG_DTLS_HVR: return 7;
    case MFP_MSG_QUIC: case MFP_MSG_OPENVPN: return QUIC_BIN;
    default: return 4;   // no message of a selected protocol
    }
}

// k_classify: lane-per-packet link/IP/transport walk + protocol
// identification only (proto_identify.h:936-968); appends each packet index
// to its bin with one wave-aggregated atomic per non-empty bin
// The walk runs on the first CLS_WIN bytes of each packet, staged in LDS with
// nine independent 16-byte loads per lane (one memory round trip instead of a
// dependent byte load per header field).  The bin only decides which kernel
// walks the whole packet, and every bin's kernel handles any packet, so a
// packet that needs more than the window to be identified is merely binned
// less well, never fingerprinted differently.
//
// Persistent blocks, two phases, so that the bin counters see one atomic per
// bin per BLOCK (same-address atomics serialise in one L2 channel): phase 1
// classifies the block's tiles (bin id per packet to `cls`, counts in LDS),
// then each non-empty bin reserves the block's span, and phase 2 re-reads the
// bin ids and scatters the packet indices in tile order.
constexpr int CLS_WIN = 128;
__global__ __launch_bounds__(TILE) void k_classify(KParams P, uint32_t *bins, uint64_t bin_stride,
                                                     unsigned long long *bin_count, uint8_t *cls) {
    __shared__ uint4 win[TILE][CLS_WIN / 16 + 1];
    __shared__ uint32_t blk_cnt[NBINS], run[NBINS];
    __shared__ unsigned long long blk_base[NBINS];
    __shared__ uint32_t wcnt[TILE / 64][NBINS];
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    if (tid < NBINS) { blk_cnt[tid] = 0; run[tid] = 0; }
    __syncthreads();
    for (uint64_t tile = blockIdx.x; tile * TILE < P.n; tile += gridDim.x) {
        const uint64_t i = tile * TILE + tid;
        int bin = -1;
        if (i < P.n) {
            const mfp_pkt_desc dsc = P.desc[i];
            const uint8_t *pkt = P.arena + dsc.offset;
            const uint32_t sh = (uint32_t)((uintptr_t)pkt & 15);
            const uint32_t take = dsc.caplen < (uint32_t)CLS_WIN ? dsc.caplen : (uint32_t)CLS_WIN;
            const uint32_t nch = (sh + take + 15) / 16;      // aligned blocks holding bytes [0, take)
            const uint4 *src = (const uint4 *)((uintptr_t)pkt - sh);
            uint4 v[CLS_WIN / 16 + 1];
#pragma unroll
            for (int k = 0; k <= CLS_WIN / 16; k++) v[k] = (uint32_t)k < nch ? src[k] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k <= CLS_WIN / 16; k++) win[tid][k] = v[k];
            Out o;
            Em<false> e;
            TlsPlan plan;                 // never filled: classification stops before any parser
            e.plan = &plan;
            Cfg c = P.cfg;
            c.classify = 1;
            c.seg = 0;
            packet_walk(e, c, o, (const uint8_t *)&win[tid][0] + sh, take, dsc.linktype);
            bin = msg_bin(o.msg);
            // selected protocols outside this path may claim a QUIC, OpenVPN
            // or DTLS packet first (Cfg::block): k_quic and the DTLS walker do
            // not decide that, the "other" bin's walker does
            if (P.cfg.block && (bin == QUIC_BIN || (bin == 7 && (P.cfg.block & BLK_UDP)))) bin = 4;
            cls[i] = (uint8_t)bin;
        }
#pragma unroll
        for (int b = 0; b < NBINS; b++) {
            const uint64_t m = __ballot(bin == b);
            if (m && lane == 0) atomicAdd(&blk_cnt[b], (uint32_t)__builtin_popcountll(m));
        }
    }
    __syncthreads();
    if (tid < NBINS) blk_base[tid] = blk_cnt[tid] ? atomicAdd(&bin_count[tid], (unsigned long long)blk_cnt[tid]) : 0ull;
    __syncthreads();
    for (uint64_t tile = blockIdx.x; tile * TILE < P.n; tile += gridDim.x) {
        const uint64_t i = tile * TILE + tid;
        const int bin = i < P.n ? (int)cls[i] : -1;
        uint64_t mine = 0;
#pragma unroll
        for (int b = 0; b < NBINS; b++) {
            const uint64_t m = __ballot(bin == b);
            if (bin == b) mine = m;
            if (lane == 0) wcnt[wid][b] = (uint32_t)__builtin_popcountll(m);
        }
        __syncthreads();
        if (bin >= 0) {
            uint32_t off = run[bin];
            for (uint32_t w = 0; w < wid; w++) off += wcnt[w][bin];
            off += (uint32_t)__builtin_popcountll(mine & ((1ull << lane) - 1));
            bins[(uint64_t)bin * bin_stride + blk_base[bin] + off] = (uint32_t)i;
        }
        __syncthreads();
        if (tid < NBINS) {
            uint32_t t = 0;
            for (int w = 0; w < TILE / 64; w++) t += wcnt[w][tid];
            run[tid] += t;
        }
        __syncthreads();
    }
}

}  // namespace mfp

extern "C" int mfp_launch_quic(const void *kparams, uint8_t *scratch, uint32_t quic_format, uint32_t grid,
                               hipStream_t stream, mfp_prof *prof);

// launchers used by the host library (mfp_host.cpp)
extern "C" int mfp_launch_fingerprint(uint32_t select, uint32_t block, uint32_t tls_format, uint32_t mode,
                                      const uint8_t *arena,
                                      const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, mfp_tcp_seg *seg,
                                      uint8_t *fp_arena,
                                      uint64_t fp_cap, unsigned long long *fp_used, uint32_t *work,
                                      unsigned long long *bin_count, int strategy, uint32_t bin_seg_mask,
                                      uint32_t bin_lds_mask, uint32_t quic_format, uint8_t *quic_scratch,
                                      uint32_t quic_grid, hipStream_t stream, mfp_prof *prof,
                                      unsigned long long *fin, unsigned long long *host_out) {
#define MFP_LAUNCH(name, ...)                                \
    do {                                                     \
        if (prof) mfp_prof_begin(prof, name, stream);        \
        hipLaunchKernelGGL(__VA_ARGS__);                     \
        if (prof) mfp_prof_end(prof, stream);                \
    } while (0)
    if (n == 0) return 0;
    mfp::KParams P;
    P.cfg.select = select; P.cfg.tls_format = tls_format; P.cfg.mode = mode; P.cfg.classify = 0; P.cfg.spread = 0;
    P.cfg.seg = seg ? 1u : 0u;
    P.cfg.block = block;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.fp_cap = fp_cap;
    P.fp_used = fp_used;
    P.seg = seg;
    P.idx = nullptr; P.count = nullptr;
    P.fin = nullptr; P.host_out = nullptr;
    // QUIC and OpenVPN packets (bin 8 of the classify pass, plus any a walker hands over)
    P.quic_idx = work + (uint64_t)mfp::QUIC_BIN * n;
    P.quic_count = bin_count + mfp::QUIC_BIN;
    const bool quic = (select & (mfp::SEL_QUIC | mfp::SEL_OPENVPN)) != 0;
    if (quic && !quic_scratch) return -1;
    auto launch_quic = [&]() -> int {
        if (!quic) return 0;
        mfp::KParams Q = P;
        Q.idx = P.quic_idx;
        Q.count = P.quic_count;
        return mfp_launch_quic(&Q, quic_scratch, quic_format, quic_grid, stream, prof);
    };
    const uint64_t tiles = (n + mfp::TILE - 1) / mfp::TILE;
    if (strategy == MFP_STRATEGY_LANE) {
        if (mfp_launch_bin_all(&P, nullptr, 0, "k_fingerprint", 0, (uint32_t)tiles, stream, prof) != 0) return -1;
        return launch_quic();
    }
    if (strategy == MFP_STRATEGY_SMALL) {
        // the whole batch through the all-family LDS walker (then k_quic
        // over the QUIC / OpenVPN packets it queued)
        uint32_t *fallback = work + (uint64_t)mfp::NBINS * n;
        // (one packet per wave: a batch's walk takes as long as its slowest
        // packet, not the sum of the protocols its lanes diverge over)
        P.cfg.spread = 1;
        // (host_out: the walker's records and strings go straight to the
        // caller's page-locked buffers, and the batch ends with this launch)
        if (host_out && !quic) { P.fin = fin; P.host_out = host_out; }
        const uint64_t lb = n < 2048 ? n : 2048;
        if (mfp_launch_bin_all(&P, fallback, 1, "k_fp_lds/small", (uint32_t)lb, 0, stream, prof) != 0) return -1;
        P.cfg.spread = 0;
        P.fin = nullptr; P.host_out = nullptr;
        // (spread: the walker handled its large packets and queued its QUIC
        // and OpenVPN packets itself -- no fallback lane)
        return launch_quic();
    }
    // classify, then one launch per protocol bin over its index list: the
    // LDS-staged walker (bin_lds_mask), the HBM lane walker, or for the HTTP
    // bins (bin_seg_mask) the segment-expansion variant of either
    uint32_t *fallback = work + (uint64_t)mfp::NBINS * n;
    const uint64_t cblocks = tiles < 2048 ? tiles : 2048;
    MFP_LAUNCH("k_classify", mfp::k_classify, dim3((uint32_t)cblocks), dim3(mfp::TILE), 0, stream, P, work, n, bin_count,
               (uint8_t *)(work + (uint64_t)(mfp::NBINS + 1) * n + 1));
    if (hipGetLastError() != hipSuccess) return -1;
    const uint64_t fblocks = tiles < 2048 ? tiles : 2048;
    const uint64_t lblocks = ((n + 63) / 64) < 2048 ? (n + 63) / 64 : 2048;
    static const char *const lane_name[mfp::NBINS] = {"k_fingerprint/tls_ch", "k_fingerprint/http_req",
        "k_fingerprint/tcp_syn", "k_fingerprint/http_resp", "k_fingerprint/other", "k_fingerprint/tls_sh",
        "k_fingerprint/ssh", "k_fingerprint/dtls", "k_quic"};
    static const char *const seg_name[mfp::NBINS] = {"k_fp_seg/tls_ch", "k_fp_seg/http_req",
        "k_fp_seg/tcp_syn", "k_fp_seg/http_resp", "k_fp_seg/other", "k_fp_seg/tls_sh",
        "k_fp_seg/ssh", "k_fp_seg/dtls", "k_quic"};
    static const char *const lds_name[mfp::NBINS] = {"k_fp_lds/tls_ch", "k_fp_lds/http_req",
        "k_fp_lds/tcp_syn", "k_fp_lds/http_resp", "k_fp_lds/other", "k_fp_lds/tls_sh",
        "k_fp_lds/ssh", "k_fp_lds/dtls", "k_quic"};
    // each bin's kernel carries its protocol's parser family only (bin 4,
    // "other", all of them); misbinned packets are punted to the fallback lane
    using namespace mfp;
    for (int b = 0; b < NBINS; b++) {
        if (b == QUIC_BIN) continue;
        P.idx = work + (uint64_t)b * n;
        P.count = bin_count + b;
        const bool seg = bin_seg_mask & (1u << b);
        const bool lds = bin_lds_mask & (1u << b);
        // (the TLS bins' lane walker is the one-pass k_fp_tls1: its own name in the profiles)
        const char *nm = lds ? lds_name[b] : seg ? seg_name[b]
                       : (MFP_TLS_ONEPASS && (b == 0 || b == 5)) ? (b == 0 ? "k_fp_tls1/tls_ch" : "k_fp_tls1/tls_sh")
                                                                  : lane_name[b];
        const uint32_t lb = (uint32_t)lblocks, fb = (uint32_t)fblocks;
        int rc;
        if (seg && b == 6) rc = mfp_launch_bin_ssh_seg(&P, fallback, lds, nm, lb, fb, stream, prof);
        else if (seg) rc = mfp_launch_bin_seg(&P, fallback, lds, nm, lb, fb, stream, prof);
        else switch (b) {
        case 0: case 5: rc = mfp_launch_bin_tls(&P, fallback, lds, nm, lb, fb, stream, prof); break;    // TLS ClientHello, ServerHello/Certificate
        case 1: case 3: rc = mfp_launch_bin_http(&P, fallback, lds, nm, lb, fb, stream, prof); break;   // HTTP request, response
        case 2: rc = mfp_launch_bin_tcp(&P, fallback, lds, nm, lb, fb, stream, prof); break;            // SYN, SYN-ACK
        case 6: rc = mfp_launch_bin_ssh(&P, fallback, lds, nm, lb, fb, stream, prof); break;
        case 7: rc = mfp_launch_bin_dtls(&P, fallback, lds, nm, lb, fb, stream, prof); break;
        default: rc = mfp_launch_bin_all(&P, fallback, lds, nm, lb, fb, stream, prof); break;          // no message of a selected protocol (or misbinned)
        }
        if (rc != 0) return -1;
    }
    {
        // the fallback lane: every parser family, straight from HBM, over the
        // packets the bin kernels handed back (fp_used[3] of them)
        P.idx = fallback;
        P.count = fp_used + 3;
        const uint64_t fb = tiles < 1024 ? tiles : 1024;
        if (mfp_launch_bin_all(&P, nullptr, 0, "k_fingerprint/fallback", 0, (uint32_t)fb, stream, prof) != 0) return -1;
    }
    return launch_quic();
}
#undef MFP_LAUNCH
