// mfp_kernels.hip -- gfx950 kernels of the fingerprint path.
//
// k_fingerprint: one 256-lane workgroup per tile of 256 packets.
//   1. each lane walks its packet (descriptor read is coalesced) and computes
//      protocol tag + exact fingerprint length (pass 1, no writes);
//   2. workgroup exclusive scan of the lengths (wave64 shuffles + LDS);
//   3. one device-scope atomicAdd per tile reserves the tile's slice of the
//      fingerprint arena (tiles land in arbitrary order, each packet's string
//      is contiguous and addressed by its record);
//   4. lanes with a fingerprint re-walk the (now L2-resident) packet and write
//      the string with 8-byte write-combined stores (pass 2);
//   5. the 32-byte record is written (coalesced).
#include <hip/hip_runtime.h>

#include "mfp_device.hpp"
#include "mfp_wave.hpp"

namespace mfp {

constexpr int TILE = 256;

struct KParams {
    Cfg cfg;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    uint8_t *fp_arena;
    uint64_t fp_cap;
    unsigned long long *fp_used;     // [0] bytes reserved, [1] overflow flag, [2] bytes written, [3] fallback count
    const uint32_t *idx;             // packet indices (count = *count); nullptr = all n packets
    const unsigned long long *count;
};

// k_fingerprint -- lane-per-packet walker, grid-stride over tiles of TILE
// packets.  Used as the fallback lane of k_wave_fp (packets larger than the
// wave kernel's LDS staging buffer, or whose fingerprint overflows its segment
// table); with idx == nullptr it processes the whole batch.
#ifndef MFP_LANE_MINW
#define MFP_LANE_MINW 4      // 4 waves per SIMD: measured best for the TLS CH and mixed bins
#endif
__global__ __launch_bounds__(TILE, MFP_LANE_MINW) void k_fingerprint(KParams P) {
    // per-lane extension scratch for TLS formats 1/2 (dynamic: 0 bytes for
    // format 0, so the default path keeps full occupancy)
    extern __shared__ uint32_t dyn_lds[];
    uint32_t *lds_key = dyn_lds;
    uint16_t *lds_off = (uint16_t *)(dyn_lds + MAX_LDS_EXT * TILE);
    __shared__ uint32_t wave_tot[TILE / 64], wave_len[TILE / 64];
    __shared__ uint64_t out_line[TILE][8];   // pass-2 output staging, one 64-byte line per lane
    __shared__ unsigned long long tile_base;

    const int tid = threadIdx.x;
    const uint64_t count = P.idx ? (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : P.n;
    for (uint64_t tile = blockIdx.x; tile * TILE < count; tile += gridDim.x) {
    const uint64_t t = tile * TILE + tid;
    const bool live = t < count;
    const uint64_t i = live ? (P.idx ? (uint64_t)P.idx[t] : t) : 0;

    mfp_pkt_desc dsc;
    if (live) dsc = P.desc[i];
    else { dsc.offset = 0; dsc.caplen = 0; dsc.linktype = 0xffff; dsc.flags = 0; }
    const uint8_t *data = P.arena + dsc.offset;

    // pass 1: walk + length
    Out o;
    uint32_t len = 0;
    {
        Em<false> e;
        packet_walk(e, P.cfg, o, data, dsc.caplen, dsc.linktype, lds_key + tid, lds_off + tid, TILE);
        if (o.fp_type) {
            if (e.valid()) len = e.n;
            else o.fp_type = 0;       // fingerprint::final drops truncated fingerprints
        }
    }

    // workgroup exclusive scan of the 64-byte slots (strings start 64-byte aligned)
    const int lane = tid & 63, wid = tid >> 6;
    const uint32_t slot = (len + 63) & ~63u;
    uint32_t incl = slot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wave_tot[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < TILE / 64; w++) {
        uint32_t tt = wave_tot[w];
        if (w < wid) wbase += tt;
        total += tt;
    }
    const uint32_t excl = wbase + incl - slot;
    // bytes written (fp_used[2]): the exact lengths
    uint32_t lsum = len;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) lsum += __shfl_xor(lsum, d, 64);
    if (lane == 0) wave_len[wid] = lsum;
    __syncthreads();
    if (tid == 0) {
        unsigned long long b = total ? atomicAdd(&P.fp_used[0], (unsigned long long)total) : 0ull;
        if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
        else if (total) {
            uint32_t lt = 0;
            for (int w = 0; w < TILE / 64; w++) lt += wave_len[w];
            atomicAdd(&P.fp_used[2], (unsigned long long)lt);
        }
        tile_base = b;
    }
    __syncthreads();
    const unsigned long long base = tile_base;
    const bool fits = base != ~0ull;

    // pass 2: emit
    if (len && fits) {
        Em<true> e;
        e.begin(P.fp_arena + base + excl, out_line[tid]);
        Out o2;
        packet_walk(e, P.cfg, o2, data, dsc.caplen, dsc.linktype, lds_key + tid, lds_off + tid, TILE);
        e.finish();
    }

    if (live) {
        mfp_record r;
        r.fp_offset = fits ? base + excl : 0;
        r.fp_len = fits ? len : 0;
        r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
        r.msg = (uint8_t)o.msg;
        r.flags = (uint8_t)o.flags;    // the lane kernel leaves hashing to the classifier
        r.status = 0;
        r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
        r.sni_len = (uint16_t)o.sni_len;
        r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
        r.ua_len = (uint16_t)o.ua_len;
        r.src_port = (uint16_t)o.src_port;
        r.dst_port = (uint16_t)o.dst_port;
        r.net = o.net;
        P.rec[i] = r;
    }
    __syncthreads();   // tile_base / wave_tot reuse
    }
}

// k_fp_seg -- the HTTP bins: lane-per-packet walk (the lane walker's SWAR
// scans and packed header-name lookup) that records the fingerprint as a
// segment list in LDS (SegEm), one reservation per tile, then each wave
// expands its packets' strings one after another with all 64 lanes: every
// store instruction writes 512 consecutive bytes, where the lane kernel's
// emission pass issues a divergent load/LDS/store stream per lane.  One walk
// instead of two.  Packets whose fingerprint is not an HTTP one, or whose list
// overflows SEG_MAX, go to the fallback lane kernel.
#ifndef MFP_SEG_MINW
#define MFP_SEG_MINW 4
#endif
constexpr int SEG_STRIDE = SEG_MAX + 1;   // odd word stride: lane-private lists are bank-conflict free
constexpr uint32_t SEG_STAGE = 2048;      // packets up to this (minus alignment) are staged in LDS for expansion
__global__ __launch_bounds__(TILE, MFP_SEG_MINW) void k_fp_seg(KParams P, uint32_t *fallback) {
    __shared__ uint32_t segs[TILE * SEG_STRIDE];
    __shared__ uint32_t wave_tot[TILE / 64], wave_len[TILE / 64];
    __shared__ unsigned long long tile_base;
    __shared__ uint8_t pool[32];
    __shared__ uint4 stage[TILE / 64][SEG_STAGE / 16];   // per wave: the packet being expanded
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    if (tid < 32) {
        const char *lp = MFP_SEG_POOL;
        pool[tid] = (uint8_t)(tid < (int)sizeof(MFP_SEG_POOL) ? lp[tid] : 0);
    }
    __syncthreads();
    const uint64_t count = (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t tile = blockIdx.x; tile * TILE < count; tile += gridDim.x) {
        const uint64_t t = tile * TILE + tid;
        const bool live = t < count;
        const uint64_t i = live ? (uint64_t)P.idx[t] : 0;
        mfp_pkt_desc dsc;
        if (live) dsc = P.desc[i];
        else { dsc.offset = 0; dsc.caplen = 0; dsc.linktype = 0xffff; dsc.flags = 0; }
        const uint8_t *data = P.arena + dsc.offset;

        Out o;
        SegEm e(data, segs + tid * SEG_STRIDE);
        packet_walk(e, P.cfg, o, data, dsc.caplen, dsc.linktype, nullptr, nullptr, 0);
        e.finish();
        const bool fb = live && e.ovf;
        uint32_t len = 0;
        if (!fb && o.fp_type) {
            if (e.valid()) len = e.n;
            else o.fp_type = 0;
        }

        // reservation: 16-byte aligned slots holding string + hash
        const uint32_t slot = len ? (len + 8 + 15) & ~15u : 0u;
        uint32_t incl = slot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        if (lane == 63) wave_tot[wid] = incl;
        uint32_t lsum = len;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) lsum += __shfl_xor(lsum, d, 64);
        if (lane == 0) wave_len[wid] = lsum;
        __syncthreads();
        uint32_t wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < TILE / 64; w++) {
            const uint32_t tt = wave_tot[w];
            if ((uint32_t)w < wid) wbase += tt;
            total += tt;
        }
        const uint32_t excl = wbase + incl - slot;
        if (tid == 0) {
            unsigned long long b = total ? atomicAdd(&P.fp_used[0], (unsigned long long)total) : 0ull;
            if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
            else if (total) {
                uint32_t lt = 0;
                for (int w = 0; w < TILE / 64; w++) lt += wave_len[w];
                atomicAdd(&P.fp_used[2], (unsigned long long)lt);
            }
            tile_base = b;
        }
        __syncthreads();
        const unsigned long long base = tile_base;
        const bool fits = base != ~0ull;

        // packets for the fallback lane kernel
        const uint64_t fbm = __ballot(fb);
        if (fbm) {
            uint32_t b = 0;
            if (lane == 0) b = (uint32_t)atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(fbm));
            b = (uint32_t)__shfl((int)b, 0, 64);
            if (fb) fallback[b + __builtin_popcountll(fbm & ((1ull << lane) - 1))] = (uint32_t)i;
        }

        // wave-cooperative expansion, one packet at a time
        uint64_t todo = fits ? __ballot(len != 0) : 0ull;
#ifdef MFP_PROBE_SEG_NOEXPAND
        todo = 0;
#endif
        const uint64_t dptr = (uint64_t)(uintptr_t)data;
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
            const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)excl, j);
            const uint32_t ns = (uint32_t)__builtin_amdgcn_readlane((int)e.nseg, j);
            const uint64_t src = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dptr, j) |
                                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(dptr >> 32), j) << 32);
            uint8_t *out = P.fp_arena + base + ex;
            // stage the packet in LDS (one coalesced 16-byte load per lane):
            // the expansion's byte reads then cost an LDS round trip, not a
            // dependent L2 round trip per character group
            const uint32_t cl = (uint32_t)__builtin_amdgcn_readlane((int)dsc.caplen, j);
            const uint8_t *pk = (const uint8_t *)(uintptr_t)src;
            const uint32_t a16 = (uint32_t)(src & 15);
            if (a16 + cl <= SEG_STAGE) {
                const uint32_t nvec = (a16 + cl + 15) >> 4;
                const uint4 *s16 = (const uint4 *)(uintptr_t)(src - a16);
                __builtin_amdgcn_wave_barrier();
                for (uint32_t v = lane; v < nvec; v += 64) stage[wid][v] = s16[v];
                __builtin_amdgcn_wave_barrier();
                pk = (const uint8_t *)&stage[wid][0] + a16;
            }
            uint64_t h = seg_expand(segs + (wid * 64 + j) * SEG_STRIDE, ns, pk, T, out, pool, lane);
            h = wave_xor64(h);
            if (lane == 0) *(uint64_t *)(out + ((T + 7) & ~7u)) = mfpc::hash_final(h, T);
        }

        if (live && !fb) {
            mfp_record r;
            r.fp_offset = fits ? base + excl : 0;
            r.fp_len = fits ? len : 0;
            r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
            r.msg = (uint8_t)o.msg;
            r.flags = (uint8_t)(o.flags | (fits && len ? MFP_FLAG_HASHED : 0));
            r.status = 0;
            r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
            r.sni_len = (uint16_t)o.sni_len;
            r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
            r.ua_len = (uint16_t)o.ua_len;
            r.src_port = (uint16_t)o.src_port;
            r.dst_port = (uint16_t)o.dst_port;
            r.net = o.net;
            P.rec[i] = r;
        }
        __syncthreads();   // tile_base / wave_tot / segs reuse
    }
}


// protocol bins of the classify pass: each bin is then fingerprinted by its
// own k_fingerprint launch over a compact index list, so the lanes of a wave
// walk the same protocol (same parser, similar loop trip counts)
constexpr int NBINS = 8;
DEV int msg_bin(uint32_t msg) {
    switch (msg) {
    case MFP_MSG_TLS_CH: return 0;
    case MFP_MSG_HTTP_REQ: return 1;
    case MFP_MSG_TCP_SYN: case MFP_MSG_TCP_SYNACK: return 2;
    case MFP_MSG_HTTP_RESP: return 3;
    case MFP_MSG_TLS_SH: case MFP_MSG_TLS_CERT: return 5;
    case MFP_MSG_SSH_INIT: case MFP_MSG_SSH_KEX: return 6;
    case MFP_MSG_DTLS_CH: case MFP_MSG_DTLS_SH: case MFP_MSG_DTLS_HVR: return 7;
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
            Cfg c = P.cfg;
            c.classify = 1;
            packet_walk(e, c, o, (const uint8_t *)&win[tid][0] + sh, take, dsc.linktype, nullptr, nullptr, 0);
            bin = msg_bin(o.msg);
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

#include "mfp_internal.h"
#define MFP_WAVE_GRID 2048   // 8 workgroups of 4 waves per CU x 256 CUs
#ifndef MFP_WAVE_MINW
#define MFP_WAVE_MINW 8      // min waves per SIMD (caps VGPRs at 64; measured best for the HTTP bins)
#endif

namespace mfpw {

constexpr uint64_t CHUNK = 32 * 1024;    // fp-arena bytes reserved per wave at a time

struct WParams {
    Cfg cfg;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    uint8_t *fp_arena;
    uint64_t fp_cap;
    unsigned long long *fp_used;     // see KParams
    uint32_t *fallback;              // packet indices for the lane-per-packet kernel
    const uint32_t *idx;             // packet indices (count = *count); nullptr = all n packets
    const unsigned long long *count;
};

WDEV uint64_t rfl64(uint64_t v) {
    return (uint64_t)rfl((uint32_t)v) | ((uint64_t)rfl((uint32_t)(v >> 32)) << 32);
}
WDEV uint32_t rdl(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }

// k_wave_fp: every wave takes groups of 64 consecutive packets (one
// descriptor per lane, coalesced) in a grid-stride loop, then handles the
// group's packets one at a time with the whole wave (mfp_wave.hpp).  Each
// wave reserves fingerprint-arena space CHUNK bytes at a time (one atomic per
// CHUNK); every string starts 16-byte aligned.  Records are gathered in the
// lanes (lane j holds packet j's record) and stored coalesced.
template <uint32_t SPEC>
__global__ __launch_bounds__(64 * WAVES, MFP_WAVE_MINW) void k_wave_fp(WParams P) {
    __shared__ WaveLds lds[WAVES];
    // wave index made provably uniform: the compiler would otherwise treat the
    // group loop as divergent and move all the scalar parse state to VGPRs
    const int wid = (int)rfl(threadIdx.x >> 6);
    WaveLds &L = lds[wid];
    const uint32_t lane = lane_id();
    const uint64_t n_eff = P.idx ? (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : P.n;
    const uint64_t ngroups = (n_eff + 63) / 64;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    uint64_t cur = 0, end = 0;
    bool dead = false;
    unsigned long long exact = 0;

    for (uint64_t g = (uint64_t)blockIdx.x * WAVES + wid; g < ngroups; g += nw) {
        const uint64_t t = g * 64 + lane;
        const bool live = t < n_eff;
        const uint64_t i = live ? (P.idx ? (uint64_t)P.idx[t] : t) : 0;
        uint32_t d_lo = 0, d_hi = 0, d_len = 0, d_lt = 0xffff;
        if (live) {
            const uint4 dv = *(const uint4 *)(P.desc + i);
            d_lo = dv.x; d_hi = dv.y; d_len = dv.z; d_lt = dv.w & 0xffff;
        }
        const int npk = (int)min((uint64_t)64, n_eff - g * 64);
        // this lane's record
        uint64_t r_off = 0;
        uint32_t r_len = 0, r_w2 = 0, r_sni = 0xffff0000u, r_ua = 0xffff0000u, r_ports = 0, r_net = 0;
        bool fb = false;

        for (int j = 0; j < npk; j++) {
            const uint64_t off = (uint64_t)rdl(d_lo, j) | ((uint64_t)rdl(d_hi, j) << 32);
            const uint32_t caplen = rdl(d_len, j), lt = rdl(d_lt, j);
            if (caplen > (uint32_t)MAX_PKT) { fb |= (int)lane == j; continue; }
            const uint32_t a = (uint32_t)(off & 15);
            const uint32_t nvec = (a + caplen + 15) >> 4;
            const uint8_t *src = P.arena + (off - a);
            __builtin_amdgcn_wave_barrier();
            for (uint32_t v = lane; v < nvec; v += 64) *(uint4 *)(L.buf + 16 * v) = *(const uint4 *)(src + 16 * v);
            __builtin_amdgcn_wave_barrier();

            W<SPEC> w(L, P.cfg);
            w.packet_walk((int)a, caplen, lt);
            w.flush();
            if (w.ovf || w.punt) { fb |= (int)lane == j; continue; }
            uint32_t type = w.o.fp_type, T = 0;
            uint64_t fpo = 0;
            if (type) {
                if (!w.valid()) {
                    type = 0;                       // fingerprint::final drops truncated fingerprints
                } else {
                    T = w.n;
                    const uint64_t slot = (T + 8 + 15) & ~15u;     // string + hash
                    if (!dead && cur + slot > end) {
                        uint64_t b = 0;
                        if (lane == 0) b = atomicAdd(&P.fp_used[0], (unsigned long long)CHUNK);
                        b = rfl64(b);
                        if (b + CHUNK > P.fp_cap) {
                            dead = true;
                            if (lane == 0) atomicExch(&P.fp_used[1], 1ull);
                        } else {
                            cur = b; end = b + CHUNK;
                        }
                    }
                    if (dead) {
                        type = 0; T = 0;
                    } else {
                        fpo = cur; cur += slot;
                        w.expand(P.fp_arena + fpo);
                        exact += T;
                    }
                }
            }
            if ((int)lane == j) {
                r_off = fpo; r_len = T;
                r_w2 = type | (w.o.msg << 8) | ((w.o.flags | (T ? MFP_FLAG_HASHED : 0u)) << 16);
                r_sni = (w.o.sni_len == 0xffff ? 0 : (w.o.sni_off & 0xffff)) | (w.o.sni_len << 16);
                r_ua = (w.o.ua_len == 0xffff ? 0 : (w.o.ua_off & 0xffff)) | (w.o.ua_len << 16);
                r_ports = (w.o.src_port & 0xffff) | (w.o.dst_port << 16);
                r_net = w.o.net;
            }
        }
        const uint64_t fbm = ballot(fb);
        if (fbm) {
            uint64_t b = 0;
            if (lane == 0) b = atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(fbm));
            b = rfl64(b);
            if (fb) P.fallback[b + __builtin_popcountll(fbm & ((1ull << lane) - 1))] = (uint32_t)i;
        }
        if (live && !fb) {
            uint4 *rp = (uint4 *)(P.rec + i);
            rp[0] = make_uint4((uint32_t)r_off, (uint32_t)(r_off >> 32), r_len, r_w2);
            rp[1] = make_uint4(r_sni, r_ua, r_ports, r_net);
        }
    }
    if (lane == 0 && exact) atomicAdd(&P.fp_used[2], exact);
}

}  // namespace mfpw

// launchers used by the host library (mfp_host.cpp)
extern "C" int mfp_launch_fingerprint(uint32_t select, uint32_t tls_format, uint32_t mode, const uint8_t *arena,
                                      const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, uint8_t *fp_arena,
                                      uint64_t fp_cap, unsigned long long *fp_used, uint32_t *work,
                                      unsigned long long *bin_count, int strategy, uint32_t bin_wave_mask,
                                      uint32_t bin_seg_mask, hipStream_t stream, mfp_prof *prof) {
#define MFP_LAUNCH(name, ...)                                \
    do {                                                     \
        if (prof) mfp_prof_begin(prof, name, stream);        \
        hipLaunchKernelGGL(__VA_ARGS__);                     \
        if (prof) mfp_prof_end(prof, stream);                \
    } while (0)
    if (n == 0) return 0;
    size_t shmem = tls_format ? (size_t)mfp::MAX_LDS_EXT * mfp::TILE * 6 : 0;
    mfp::KParams P;
    P.cfg.select = select; P.cfg.tls_format = tls_format; P.cfg.mode = mode; P.cfg.classify = 0;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.fp_cap = fp_cap;
    P.fp_used = fp_used;
    P.idx = nullptr; P.count = nullptr;
    const uint64_t tiles = (n + mfp::TILE - 1) / mfp::TILE;
    if (strategy == MFP_STRATEGY_LANE) {
        MFP_LAUNCH("k_fingerprint", mfp::k_fingerprint, dim3((uint32_t)tiles), dim3(mfp::TILE), shmem, stream, P);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    mfpw::WParams W;
    W.cfg.select = select; W.cfg.tls_format = tls_format; W.cfg.mode = mode;
    W.arena = arena; W.desc = desc; W.n = n; W.rec = rec; W.fp_arena = fp_arena; W.fp_cap = fp_cap;
    W.fp_used = fp_used; W.fallback = work + (strategy == MFP_STRATEGY_BINNED ? (uint64_t)mfp::NBINS * n : 0);
    W.idx = nullptr; W.count = nullptr;
    uint64_t groups = (n + 63) / 64;
    if (strategy == MFP_STRATEGY_BINNED) {
        // classify, then one launch per protocol bin: the lane-per-packet
        // walker or the wave-per-packet walker, whichever is faster for
        // that protocol (bin_wave_mask bit b = wave kernel for bin b)
        const uint64_t cblocks = tiles < 2048 ? tiles : 2048;
        MFP_LAUNCH("k_classify", mfp::k_classify, dim3((uint32_t)cblocks), dim3(mfp::TILE), 0, stream, P, work, n, bin_count,
                   (uint8_t *)(work + (uint64_t)(mfp::NBINS + 1) * n + 1));
        if (hipGetLastError() != hipSuccess) return -1;
        uint64_t fblocks = tiles < 2048 ? tiles : 2048;
        uint64_t wblocks = (groups + mfpw::WAVES - 1) / mfpw::WAVES;
        if (wblocks > (uint64_t)MFP_WAVE_GRID) wblocks = MFP_WAVE_GRID;
        bool any_wave = false;
        for (int b = 0; b < mfp::NBINS; b++) {
            static const char *const wave_name[mfp::NBINS] = {"k_wave_fp/tls_ch", "k_wave_fp/http_req",
                "k_wave_fp/tcp_syn", "k_wave_fp/http_resp", "k_wave_fp/other", "k_wave_fp/tls_sh",
                "k_wave_fp/ssh", "k_wave_fp/dtls"};
            static const char *const lane_name[mfp::NBINS] = {"k_fingerprint/tls_ch", "k_fingerprint/http_req",
                "k_fingerprint/tcp_syn", "k_fingerprint/http_resp", "k_fingerprint/other", "k_fingerprint/tls_sh",
                "k_fingerprint/ssh", "k_fingerprint/dtls"};
            static const char *const seg_name[mfp::NBINS] = {"k_fp_seg/tls_ch", "k_fp_seg/http_req",
                "k_fp_seg/tcp_syn", "k_fp_seg/http_resp", "k_fp_seg/other", "k_fp_seg/tls_sh",
                "k_fp_seg/ssh", "k_fp_seg/dtls"};
            if (bin_seg_mask & (1u << b)) {
                // lane walk + wave expansion (HTTP; anything else -> fallback lane)
                P.idx = work + (uint64_t)b * n;
                P.count = bin_count + b;
                MFP_LAUNCH(seg_name[b], mfp::k_fp_seg, dim3((uint32_t)fblocks), dim3(mfp::TILE), 0, stream, P,
                           W.fallback);
                any_wave = true;
            } else if (bin_wave_mask & (1u << b)) {
                W.idx = work + (uint64_t)b * n;
                W.count = bin_count + b;
                // the bin's protocol families only (others -> fallback lane)
                auto kw = (b == 0 || b == 5) ? mfpw::k_wave_fp<mfpw::SPEC_TLS>
                        : (b == 1 || b == 3) ? mfpw::k_wave_fp<mfpw::SPEC_HTTP>
                        : b == 6 ? mfpw::k_wave_fp<mfpw::SPEC_SSH>
                        : b == 7 ? mfpw::k_wave_fp<mfpw::SPEC_DTLS>
                        : b == 2 ? mfpw::k_wave_fp<0u> : mfpw::k_wave_fp<mfpw::SPEC_ALL>;
                MFP_LAUNCH(wave_name[b], kw, dim3((uint32_t)wblocks), dim3(64 * mfpw::WAVES), 0, stream, W);
                any_wave = true;
            } else {
                P.idx = work + (uint64_t)b * n;
                P.count = bin_count + b;
                MFP_LAUNCH(lane_name[b], mfp::k_fingerprint, dim3((uint32_t)fblocks), dim3(mfp::TILE), shmem, stream, P);
            }
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (any_wave) {
            // fallback lane for packets the wave kernel handed back
            P.idx = W.fallback;
            P.count = fp_used + 3;
            uint64_t fb = tiles < 1024 ? tiles : 1024;
            MFP_LAUNCH("k_fingerprint/fallback", mfp::k_fingerprint, dim3((uint32_t)fb), dim3(mfp::TILE), shmem, stream, P);
        }
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    uint64_t wblocks = (groups + mfpw::WAVES - 1) / mfpw::WAVES;
    if (wblocks > (uint64_t)MFP_WAVE_GRID) wblocks = MFP_WAVE_GRID;
    MFP_LAUNCH("k_wave_fp", mfpw::k_wave_fp<mfpw::SPEC_ALL>, dim3((uint32_t)wblocks), dim3(64 * mfpw::WAVES), 0, stream, W);
    if (hipGetLastError() != hipSuccess) return -1;
    // fallback lane over the packets the wave kernel handed back
    P.idx = work;
    P.count = fp_used + 3;
    uint64_t fblocks = tiles < 1024 ? tiles : 1024;
    MFP_LAUNCH("k_fingerprint/fallback", mfp::k_fingerprint, dim3((uint32_t)fblocks), dim3(mfp::TILE), shmem, stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#undef MFP_LAUNCH
