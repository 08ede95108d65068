// mfp_kernels.hpp -- gfx950 kernels of the fingerprint path (the per-packet walkers).
//
// Included by one translation unit per parser family (mfp_k_*.hip), each of
// which instantiates and launches its family's kernels, so the families
// compile in parallel; mfp_kernels.hip holds k_classify and the launcher.
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
#pragma once
#include <hip/hip_runtime.h>

#include "mfp_device.hpp"
#include "mfp_internal.h"

#include "mfp_kphase.hpp"

namespace mfp {

constexpr int TILE = 256;

// Tile order by length (k_fp_tls1).  A
// lane-per-packet wave runs every loop for its longest packet and every
// branch its lanes take, so the tile's packets are handed to its lanes in
// caplen order: packets of one length are mostly one client's hello or one
// request template, so a wave's lanes walk and emit alike.  The rank of each
// packet is the count of smaller (caplen, lane) keys, read four at a time
// from LDS (every lane reads the same words: broadcast, no bank conflict);
// the tile's live packets stay the first lanes.  Output placement does not
// change meaning: the records address their strings.
// (The same order for the HTTP request bin was slower, 9.91 -> 10.18 ms, and
// an order over two tiles gained 0.08 ms only: neither is kept, r05_ab/r05s*.)
struct TileSort {
    uint32_t key[TILE] __attribute__((aligned(16)));
    uint32_t idx[TILE];
    mfp_pkt_desc desc[TILE];
};
template <bool ALIASED = false>   // ALIASED: s overlays LDS the walk writes (a barrier after the reads)
DEV void tile_take(const KParams &P, uint64_t tile, uint64_t count, TileSort &s, int tid, uint64_t &i,
                   mfp_pkt_desc &dsc, bool &live) {
    const uint64_t t = tile * TILE + tid;
    live = t < count;
    const uint32_t i0 = live ? P.idx[t] : 0u;
    mfp_pkt_desc d0;
    if (live) d0 = P.desc[i0];
    else { d0.offset = 0; d0.caplen = 0; d0.linktype = 0xffff; d0.flags = 0; }
    const uint32_t cl = d0.caplen < 0xfffffeu ? d0.caplen : 0xfffffeu;
    const uint32_t mk = ((live ? cl : 0xffffffu) << 8) | (uint32_t)tid;
    s.key[tid] = mk;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll 8
    for (int j = 0; j < TILE; j += 4) {
        const uint4 v = *(const uint4 *)&s.key[j];
        r += (v.x < mk ? 1u : 0u) + (v.y < mk ? 1u : 0u) + (v.z < mk ? 1u : 0u) + (v.w < mk ? 1u : 0u);
    }
    s.idx[r] = i0;
    s.desc[r] = d0;
    __syncthreads();
    i = s.idx[tid];
    dsc = s.desc[tid];
    if (ALIASED) __syncthreads();
    // (otherwise the caller's end-of-tile barrier orders these reads before the next tile's writes)
}

// k_fingerprint -- lane-per-packet walker straight from HBM, grid-stride
// over tiles of TILE packets.  The fallback lane of the other bin kernels
// (packets larger than k_fp_lds's stage, segment lists that overflow); with
// idx == nullptr it processes the whole batch (MFP_STRATEGY=lane).
#ifndef MFP_LANE_MINW
#define MFP_LANE_MINW 4      // 4 waves per SIMD: measured best for the TLS CH and mixed bins
#endif
#ifndef MFP_TLS_PLAN_ONLY
#define MFP_TLS_PLAN_ONLY 1
#endif
#ifndef MFP_TLS_MINW
#define MFP_TLS_MINW 3       // the TLS parser wants ~200 VGPRs: 3 waves/SIMD measured best (4: spills, 2: latency)
#endif
template <uint32_t FAM>
__global__ __launch_bounds__(TILE, FAM == FAM_TLS ? MFP_TLS_MINW : MFP_LANE_MINW) void k_fingerprint(KParams P,
                                                                                                     uint32_t *fallback) {
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

    // pass 1: walk + length (+ the ClientHello plan pass 2 emits from)
    Out o;
    uint32_t len = 0;
    bool punt = false;
    TlsPlan plan;
    plan.ok = false;
    {
        Em<false> e;
        e.plan = &plan;
        packet_walk<FAM>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
        punt = live && e.punt;
        if (o.fp_type && !punt) {
            if (e.valid()) len = e.n;
            else o.fp_type = 0;       // fingerprint::final drops truncated fingerprints
        }
        // the TLS lane kernel emits from a ClientHello plan only: a fingerprint
        // without one (server messages, extension lists the plan cannot hold)
        // goes to the fallback lane, so this kernel carries no second walker
        if (FAM == FAM_TLS && MFP_TLS_PLAN_ONLY && live && len && !plan.ok) { punt = true; len = 0; }
    }
    {
        // a parser this instance lacks: the fallback lane; QUIC and OpenVPN
        // (which only k_quic parses): the k_quic list
        const bool to_quic = punt && (o.msg == MFP_MSG_QUIC || o.msg == MFP_MSG_OPENVPN);
        const bool to_fb = punt && !to_quic && FAM != FAM_ALL;
        const uint64_t pm = __ballot(to_fb);
        if (pm) {
            uint32_t b = 0;
            if ((tid & 63) == 0) b = (uint32_t)atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(pm));
            b = (uint32_t)__shfl((int)b, 0, 64);
            if (to_fb) fallback[b + __builtin_popcountll(pm & ((1ull << (tid & 63)) - 1))] = (uint32_t)i;
        }
        const uint64_t qm = __ballot(to_quic);
        if (qm) {
            uint32_t b = 0;
            if ((tid & 63) == 0) b = (uint32_t)atomicAdd(P.quic_count, (unsigned long long)__builtin_popcountll(qm));
            b = (uint32_t)__shfl((int)b, 0, 64);
            if (to_quic) P.quic_idx[b + __builtin_popcountll(qm & ((1ull << (tid & 63)) - 1))] = (uint32_t)i;
        }
    }

    // workgroup exclusive scan of the 64-byte slots (strings start 64-byte
    // aligned; each is followed by its 8-byte hash at round_up(len, 8))
    const int lane = tid & 63, wid = tid >> 6;
    const uint32_t slot = len ? (((len + 7) & ~7u) + 8 + 63) & ~63u : 0u;
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
#ifdef MFP_PROBE_NOPASS2
    if (0) {
#else
    if (len && fits) {
#endif
        Em<true> e;
        e.begin(P.fp_arena + base + excl, out_line[tid]);
        if (plan.ok) {
            tls_ch_emit(e, plan);
        } else if constexpr (!(FAM == FAM_TLS && MFP_TLS_PLAN_ONLY)) {
            Out o2;
            packet_walk<FAM>(e, P.cfg, o2, data, dsc.caplen, dsc.linktype);
        }
        e.finish();
        *(uint64_t *)(P.fp_arena + base + excl + ((len + 7) & ~7u)) = e.hash();
    }

    if (live && !punt) {
        mfp_record r;
        r.fp_offset = fits ? base + excl : 0;
        r.fp_len = fits ? len : 0;
        r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
        r.msg = (uint8_t)o.msg;
        r.flags = (uint8_t)(o.flags | (fits && len ? MFP_FLAG_HASHED : 0));
        r.xflags = (uint8_t)o.xflags;
        r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
        r.sni_len = (uint16_t)o.sni_len;
        r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
        r.ua_len = (uint16_t)o.ua_len;
        r.src_port = (uint16_t)o.src_port;
        r.dst_port = (uint16_t)o.dst_port;
        r.net = o.net;
        P.rec[i] = r;
            write_seg(P, i, o);
    }
    __syncthreads();   // tile_base / wave_tot reuse
    }
}

// k_fp_tls1 -- the TLS ClientHello bin in one pass.  Each string's slot is
// reserved BEFORE the walk, from an upper bound on its length: 2 characters
// per byte of the frame plus 64 (hex doubles the bytes it prints; the
// ClientHello's unprinted headers, random and session id outweigh the
// parentheses), at most 8192.  So a lane emits its fingerprint from the plan
// right after building it, while the ClientHello's bytes are still in the
// cache, instead of after the tile's scan of exact lengths.  Strings are spaced
// by their bound, not packed (within mfp_fp_arena_bound).  A string longer than
// its bound, or one without a plan, goes to the fallback lane.
#ifndef MFP_TLS_ONEPASS
#define MFP_TLS_ONEPASS 1
#endif
template <int FMT>
__global__ __launch_bounds__(TILE, MFP_TLS_MINW) void k_fp_tls1(KParams P, uint32_t *fallback) {
    __shared__ uint32_t wave_tot[TILE / 64];
    __shared__ __attribute__((aligned(16))) uint64_t out_line[TILE][8];   // emission staging, one 64-byte line per lane
    __shared__ uint32_t ext_off[TILE][FAST_EXT + 1];   // the plan's rows: ext_row entries by wire index (odd stride)
    __shared__ uint8_t ext_ord[FMT ? TILE : 1][FAST_EXT + 4];   // emission order (formats 1/2)
    __shared__ unsigned long long tile_base;
#if MFP_EXT_WIN == 2 && MFP_EXT_WIN_BLOCKS > 4
    __shared__ __attribute__((aligned(16))) uint8_t ext_win2[TILE / 64][1024 * (MFP_EXT_WIN_BLOCKS - 4)];
#endif
    // the tile order over the emission lines (the extension windows are written right after the take)
    static_assert(sizeof(TileSort) <= sizeof(out_line), "TileSort in out_line");
    TileSort &tsort = *reinterpret_cast<TileSort *>(&out_line[0][0]);
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const uint64_t count = (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    KPH_DECL
    for (uint64_t tile = blockIdx.x; tile * TILE < count; tile += gridDim.x) {
        uint64_t i;
        bool live;
        mfp_pkt_desc dsc;
        tile_take<true>(P, tile, count, tsort, tid, i, dsc, live);

        // reservation from the bound: one atomic per tile
        const uint32_t bound = live ? (2 * dsc.caplen + 64 < FP_MAX ? 2 * dsc.caplen + 64 : FP_MAX) : 0u;
        const uint32_t slot = bound ? (((bound + 7) & ~7u) + 8 + 63) & ~63u : 0u;
        uint32_t incl = slot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wave_tot[wid] = incl;
        __syncthreads();
        uint32_t wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < TILE / 64; w++) {
            const uint32_t tt = wave_tot[w];
            if (w < wid) wbase += tt;
            total += tt;
        }
        const uint32_t excl = wbase + incl - slot;
        if (tid == 0) {
            unsigned long long b = total ? atomicAdd(&P.fp_used[0], (unsigned long long)total) : 0ull;
            if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
            tile_base = b;
        }
        __syncthreads();
        const unsigned long long base = tile_base;
        const bool fits = base != ~0ull;
        KPH(0);

        // walk + plan
        Out o;
        uint32_t len = 0;
        bool punt = false;
        TlsPlan plan;
        plan.ok = false;
        plan.off_row = ext_off[tid];
        plan.ord_row = ext_ord[FMT ? tid : 0];
        // free until the emission: the extension-header window (ExtWin)
        const uint8_t *data = P.arena + dsc.offset;
        plan.win = MFP_EXT_WIN == 2 ? (uint8_t *)&out_line[0][0] + 4096 * wid : (uint8_t *)out_line[tid];
        plan.win_lane = (uint32_t)lane;
#if MFP_EXT_WIN == 2 && MFP_EXT_WIN_BLOCKS > 4
        plan.win2 = ext_win2[wid];
#endif
        {
            Em<false, FMT> e;
            e.plan = &plan;
            packet_walk<FAM_TLS>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
            punt = live && e.punt;
            if (o.fp_type && !punt) {
                if (e.valid()) len = e.n;
                else o.fp_type = 0;       // fingerprint::final drops truncated fingerprints
            }
            if (live && len && (!plan.ok || ((len + 7) & ~7u) + 8 > slot)) { punt = true; len = 0; }
        }
        KPH(1);
        {
            const bool to_quic = punt && (o.msg == MFP_MSG_QUIC || o.msg == MFP_MSG_OPENVPN);
            const bool to_fb = punt && !to_quic;
            const uint64_t pm = __ballot(to_fb);
            if (pm) {
                uint32_t b = 0;
                if (lane == 0) b = (uint32_t)atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(pm));
                b = (uint32_t)__shfl((int)b, 0, 64);
                if (to_fb) fallback[b + __builtin_popcountll(pm & ((1ull << lane) - 1))] = (uint32_t)i;
            }
            const uint64_t qm = __ballot(to_quic);
            if (qm) {
                uint32_t b = 0;
                if (lane == 0) b = (uint32_t)atomicAdd(P.quic_count, (unsigned long long)__builtin_popcountll(qm));
                b = (uint32_t)__shfl((int)b, 0, 64);
                if (to_quic) P.quic_idx[b + __builtin_popcountll(qm & ((1ull << lane) - 1))] = (uint32_t)i;
            }
        }
        KPH(2);
        // emit from the plan, the ClientHello still in the cache
#ifdef MFP_PROBE_NOEMIT   // (profiling probe only: the walk and plan alone)
        if (len && fits && dsc.caplen == 0xffffffffu) {
#else
        if (len && fits) {
#endif
            Em<true> e;                                          // the packet is in HBM
            e.begin(P.fp_arena + base + excl, out_line[tid]);
            tls_ch_emit_fast<FMT>(e, plan);
            e.finish();
            *(uint64_t *)(P.fp_arena + base + excl + ((len + 7) & ~7u)) = e.hash();
        }
        KPH(3);
        {   // bytes written (fp_used[2]): the exact lengths
            uint32_t lsum = fits ? len : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lsum += __shfl_xor(lsum, d, 64);
            if (lane == 0 && lsum) atomicAdd(&P.fp_used[2], (unsigned long long)lsum);
        }
        if (live && !punt) {
            mfp_record r;
            r.fp_offset = fits ? base + excl : 0;
            r.fp_len = fits ? len : 0;
            r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
            r.msg = (uint8_t)o.msg;
            r.flags = (uint8_t)(o.flags | (fits && len ? MFP_FLAG_HASHED : 0));
            r.xflags = (uint8_t)o.xflags;
            r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
            r.sni_len = (uint16_t)o.sni_len;
            r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
            r.ua_len = (uint16_t)o.ua_len;
            r.src_port = (uint16_t)o.src_port;
            r.dst_port = (uint16_t)o.dst_port;
            r.net = o.net;
            P.rec[i] = r;
            write_seg(P, i, o);
        }
        __syncthreads();   // tile_base / wave_tot reuse
        KPH(4);
    }
    KPH_FLUSH();
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
// MFP_SEG_LANE (default): each lane writes its own string from its list
// (seg_emit_lane: 64 strings per wave at once, 4-word LDS lines); 0: the
// wave expands the strings one after another (seg_expand)
#ifndef MFP_SEG_LANE
#define MFP_SEG_LANE 1
#endif
constexpr int SEG_STRIDE = SEG_MAX + 1;   // odd word stride: lane-private lists are bank-conflict free
constexpr uint32_t SEG_STAGE = 2048;      // packets up to this (minus alignment) are staged in LDS for expansion
#ifndef MFP_SEG_LINEW
#define MFP_SEG_LINEW 4
#endif
constexpr int SEG_LINEW = MFP_SEG_LINEW;  // lane emission: words per LDS line
template <uint32_t FAM = FAM_HTTP>
__global__ __launch_bounds__(TILE, MFP_SEG_MINW) void k_fp_seg(KParams P, uint32_t *fallback) {
    __shared__ uint32_t segs[TILE * SEG_STRIDE];
    __shared__ uint32_t wave_tot[TILE / 64], wave_len[TILE / 64];
    __shared__ unsigned long long tile_base;
    __shared__ uint8_t pool[SEG_POOL_BYTES];
#if MFP_HTTP_NAMEWIN
    __shared__ HdrKey s_keys[N_REQ_NAMES + N_RESP_NAMES];
    __shared__ uint8_t s_slots[(1 << REQ_BITS) + (1 << RESP_BITS)];
#endif
#if MFP_SEG_LANE
    __shared__ __attribute__((aligned(16))) uint64_t out_line[TILE][SEG_LINEW];
#else
    __shared__ uint4 stage[TILE / 64][SEG_STAGE / 16];   // per wave: the packet being expanded
#endif
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63, wid = tid >> 6;
    if (tid < (int)SEG_POOL_BYTES) {
        const char *lp = MFP_SEG_POOL;
        pool[tid] = (uint8_t)(tid < (int)sizeof(MFP_SEG_POOL) ? lp[tid] : 0);
    }
#if MFP_HTTP_NAMEWIN
    if constexpr ((FAM & FAM_HTTP) != 0) {   // the header-name tables, for walkers that parse HTTP
        if (tid < N_REQ_NAMES) s_keys[tid] = k_req_keys[tid];
        else if (tid < N_REQ_NAMES + N_RESP_NAMES) s_keys[tid] = k_resp_keys[tid - N_REQ_NAMES];
        if (tid < (1 << REQ_BITS)) s_slots[tid] = k_req_slots.s[tid];
        else if (tid < (1 << REQ_BITS) + (1 << RESP_BITS)) s_slots[tid] = k_resp_slots.s[tid - (1 << REQ_BITS)];
    }
#endif
    __syncthreads();
    const uint64_t count = (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    KPH_DECL
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
#if MFP_HTTP_NAMEWIN
        e.slots_req = s_slots; e.slots_resp = s_slots + (1 << REQ_BITS);
        e.keys_req = s_keys; e.keys_resp = s_keys + N_REQ_NAMES;
#endif
        packet_walk<FAM>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
        e.finish();
        const bool fb = live && e.ovf;
        uint32_t len = 0;
        if (!fb && o.fp_type) {
            if (e.valid()) len = e.n;
            else o.fp_type = 0;
        }
        KPH(0);

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

        KPH(1);
#if MFP_SEG_LANE
        if (len && fits) {
            Em<true, -1, SEG_LINEW> em;                          // the packet is in HBM
            em.begin(P.fp_arena + base + excl, out_line[tid]);
            seg_emit_lane(em, segs + tid * SEG_STRIDE, e.nseg, data, pool);
            em.finish();
            *(uint64_t *)(P.fp_arena + base + excl + ((len + 7) & ~7u)) = em.hash();
        }
#else
        // wave-cooperative expansion, one packet at a time
        uint64_t todo = fits ? __ballot(len != 0) : 0ull;
#ifdef MFP_PROBE_SEG_NOEXPAND
        todo = 0;
#endif
        const uint64_t dptr = (uint64_t)(uintptr_t)data;
        // packet j's 16-byte blocks (up to SEG_STAGE bytes: two per lane),
        // loaded into registers while the packet before it is expanded, then
        // written to the wave's LDS stage: the stage's memory round trip is
        // off the per-packet critical path
        constexpr uint32_t SPL = SEG_STAGE / 16 / 64;   // blocks per lane
        uint4 pre[SPL];
        auto stage_load = [&](int j) {
            const uint64_t src = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dptr, j) |
                                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(dptr >> 32), j) << 32);
            const uint32_t cl = (uint32_t)__builtin_amdgcn_readlane((int)dsc.caplen, j);
            const uint32_t a16 = (uint32_t)(src & 15);
            const uint32_t nvec = a16 + cl <= SEG_STAGE ? (a16 + cl + 15) >> 4 : 0u;
            const uint4 *s16 = (const uint4 *)(uintptr_t)(src - a16);
#pragma unroll
            for (uint32_t k = 0; k < SPL; k++) {
                const uint32_t v = k * 64 + lane;
                pre[k] = v < nvec ? s16[v] : make_uint4(0, 0, 0, 0);
            }
        };
        if (todo) stage_load(__builtin_ctzll(todo));
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
            const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)excl, j);
            const uint32_t ns = (uint32_t)__builtin_amdgcn_readlane((int)e.nseg, j);
            const uint64_t src = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dptr, j) |
                                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(dptr >> 32), j) << 32);
            uint8_t *out = P.fp_arena + base + ex;
            // the packet from the LDS stage (expansion's byte reads are LDS
            // round trips, not dependent L2 round trips); a packet larger than
            // the stage is read where it lies
            const uint32_t cl = (uint32_t)__builtin_amdgcn_readlane((int)dsc.caplen, j);
            const uint8_t *pk = (const uint8_t *)(uintptr_t)src;
            const uint32_t a16 = (uint32_t)(src & 15);
            __builtin_amdgcn_wave_barrier();
            if (a16 + cl <= SEG_STAGE) {
#pragma unroll
                for (uint32_t k = 0; k < SPL; k++) stage[wid][k * 64 + lane] = pre[k];
                pk = (const uint8_t *)&stage[wid][0] + a16;
            }
            __builtin_amdgcn_wave_barrier();
            if (todo) stage_load(__builtin_ctzll(todo));   // the next packet, in flight during this expansion
            uint64_t h = seg_expand(segs + (wid * 64 + j) * SEG_STRIDE, ns, pk, T, out, pool, lane);
            h = wave_xor64(h);
            if (lane == 0) *(uint64_t *)(out + ((T + 7) & ~7u)) = mfpc::hash_final(h, T);
        }
#endif

        KPH(2);
        if (live && !fb) {
            mfp_record r;
            r.fp_offset = fits ? base + excl : 0;
            r.fp_len = fits ? len : 0;
            r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
            r.msg = (uint8_t)o.msg;
            r.flags = (uint8_t)(o.flags | (fits && len ? MFP_FLAG_HASHED : 0));
            r.xflags = (uint8_t)o.xflags;
            r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
            r.sni_len = (uint16_t)o.sni_len;
            r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
            r.ua_len = (uint16_t)o.ua_len;
            r.src_port = (uint16_t)o.src_port;
            r.dst_port = (uint16_t)o.dst_port;
            r.net = o.net;
            P.rec[i] = r;
            write_seg(P, i, o);
        }
        __syncthreads();   // tile_base / wave_tot / segs reuse
        KPH(3);
    }
    KPH_FLUSH();
}


// k_fp_lds -- the lane walker over packets staged in LDS.  One wave per
// workgroup; a wave takes 64 packets of its bin (one per lane) and copies as
// many of them as fit its LDS stage with direct-to-LDS 16-byte loads
// (global_load_lds_dwordx4: every wave-instruction moves 1 KiB of one packet,
// coalesced), then every lane walks its own packet from LDS.  The walk's
// dependent byte reads are LDS round trips instead of divergent global loads
// that touch 64 cache lines per instruction, and each packet leaves HBM once.
// Packets that do not fit the next sub-round wait for it; a packet larger
// than the whole stage goes to the fallback lane kernel (global walk).
//   SEGMODE = false: two walks (length, then emission through 64-byte LDS
//     lines, k_fingerprint's emitter); the string hash is folded into the
//     emission and stored behind the string.
//   SEGMODE = true (HTTP bins): one walk recording a segment list (SegEm),
//     then the wave expands each string with coalesced stores (seg_expand),
//     reading the hex sources from the staged packet.
template <bool SEGMODE, uint32_t STG, uint32_t FAM>
__global__ __launch_bounds__(64) void k_fp_lds(KParams P, uint32_t *fallback) {
    __shared__ uint4 stage[STG / 16];
    __shared__ uint64_t out_line[SEGMODE ? 1 : 64][8];
    __shared__ uint32_t segs[SEGMODE ? 64 * SEG_STRIDE : 1];
    __shared__ uint8_t pool[SEG_POOL_BYTES];
    const uint32_t lane = threadIdx.x;
    uint8_t *stg = (uint8_t *)&stage[0];
    if (SEGMODE) {
        const char *lp = MFP_SEG_POOL;
        for (uint32_t k = lane; k < SEG_POOL_BYTES; k += 64) pool[k] = (uint8_t)(k < sizeof(MFP_SEG_POOL) ? lp[k] : 0);
    }
    __builtin_amdgcn_wave_barrier();
    // (idx == nullptr: the whole batch, MFP_STRATEGY_SMALL)
    const uint64_t count = P.idx ? (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : P.n;
#ifdef MFP_PROBE_REPEAT   // (latency probe: the whole walk R times in the same wave)
    for (int rep_ = 0; rep_ < MFP_PROBE_REPEAT; rep_++)
#endif
    // (P.idx == nullptr then; only the small-batch all-family instance spreads)
    const bool spread = FAM == FAM_ALL && !SEGMODE && P.cfg.spread != 0;
    for (uint64_t g = blockIdx.x; (spread ? g : g * 64) < count; g += gridDim.x) {
        const uint64_t t = spread ? g : g * 64 + lane;
        const bool live = spread ? lane == 0 : t < count;
        const uint64_t i = live ? (P.idx ? (uint64_t)P.idx[t] : t) : 0;
        mfp_pkt_desc dsc;
        if (live) dsc = P.desc[i];
        else { dsc.offset = 0; dsc.caplen = 0; dsc.linktype = 0xffff; dsc.flags = 0; }
        const uint32_t a16 = (uint32_t)(dsc.offset & 15);
        const uint32_t pk_bytes = (a16 + dsc.caplen + 15) & ~15u;      // whole 16-byte blocks
        // spread (one packet per wave): a packet larger than the stage is
        // walked straight from global memory by its own wave, not handed on
        const bool glob = spread && live && pk_bytes > STG;
        const uint32_t need = glob ? 0u : pk_bytes;
        const bool big = live && need > STG;
        {   // too large for any sub-round: the fallback lane walks it from HBM
            const uint64_t bm = __ballot(big);
            if (bm) {
                uint32_t b = 0;
                if (lane == 0) b = (uint32_t)atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(bm));
                b = (uint32_t)__shfl((int)b, 0, 64);
                if (big) fallback[b + __builtin_popcountll(bm & ((1ull << lane) - 1))] = (uint32_t)i;
            }
        }
        bool todo = live && !big;
        while (__ballot(todo)) {
            // this sub-round: the waiting lanes, in lane order, while they fit
            uint32_t x = todo ? need : 0u, incl = x;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= (uint32_t)d) incl += y;
            }
            const bool in = todo && incl <= STG;
            const uint32_t sbase = incl - x;
            // stage: one packet after the other, 1 KiB per wave-instruction
            for (uint64_t m = __ballot(in && !glob); m; m &= m - 1) {
                const int j = __builtin_ctzll(m);
                const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)sbase, j);
                const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)pk_bytes, j) >> 4;
                const uint64_t o = dsc.offset & ~(uint64_t)15;
                const uint64_t oj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)o, j) |
                                    ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(o >> 32), j) << 32);
                const uint8_t *src = P.arena + oj;
                for (uint32_t k = 0; k * 64 < nb; k++) {
                    const uint32_t blk = k * 64 + lane;
                    if (blk < nb)
                        __builtin_amdgcn_global_load_lds((const void *)(src + 16 * (uint64_t)blk),
                                                         (void __attribute__((address_space(3))) *)(stg + bj + 1024 * k),
                                                         16, 0, 0);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const uint8_t *data = glob ? P.arena + dsc.offset : stg + sbase + a16;
            // spread, a packet that leaves room in the stage for its string:
            // a single walk that emits as it goes (`one`), the wave copying the
            // string out afterwards, instead of a counting walk and an emitting
            // walk one after the other (a lone packet's latency)
            constexpr uint32_t EBUF = FP_MAX + 64;
            constexpr bool ONE_OK = !SEGMODE && FAM == FAM_ALL;   // (the small-batch instance)
            const uint32_t e_at = (sbase + pk_bytes + 63) & ~63u;
            const bool one = ONE_OK && spread && !glob && e_at + EBUF <= STG;
            uint8_t *const ebuf = stg + e_at;
            uint64_t one_hash = 0;

            Out o;
            uint32_t len = 0;
            bool fb = false;
            uint32_t nseg = 0;
            TlsPlan plan;
            plan.ok = false;
            if constexpr (SEGMODE) {
                SegEm e(data, segs + lane * SEG_STRIDE);
                if (in) {
                    packet_walk<FAM>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
                    e.finish();
                    fb = e.ovf;
                    if (!fb && o.fp_type) {
                        if (e.valid()) len = e.n;
                        else o.fp_type = 0;
                    }
                    nseg = e.nseg;
                }
            } else {
                bool walked = false;
                if constexpr (ONE_OK) {
                    if (in && one) {
                        // one pass: the string is written into the stage behind the
                        // packet while the walk counts it (capped at FP_MAX + a line)
                        Em<true> e;
                        e.begin(ebuf, out_line[lane]);
                        e.out_end = ebuf + EBUF;
                        e.spans = true;
                        packet_walk<FAM>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
                        e.finish();
                        fb = e.punt;
                        if (o.fp_type && !fb) {
                            if (e.valid()) len = e.n;
                            else o.fp_type = 0;    // fingerprint::final drops truncated fingerprints
                        }
                        one_hash = e.hash();
                        walked = true;
                    }
                }
                if (in && !walked) {
                    Em<false> e;
                    e.plan = &plan;
                    packet_walk<FAM>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
                    fb = e.punt;
                    if (o.fp_type && !fb) {
                        if (e.valid()) len = e.n;
                        else o.fp_type = 0;    // fingerprint::final drops truncated fingerprints
                    }
                }
            }
            // arena reservation for the sub-round: one atomic per wave
            const uint32_t slot = SEGMODE ? (len ? (len + 8 + 15) & ~15u : 0u)
                                          : (len ? (((len + 7) & ~7u) + 8 + 63) & ~63u : 0u);
            uint32_t sincl = slot, lsum = len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(sincl, d, 64);
                if (lane >= (uint32_t)d) sincl += y;
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lsum += __shfl_xor(lsum, d, 64);
            const uint32_t total = (uint32_t)__shfl((int)sincl, 63, 64);
            unsigned long long b = 0;
            if (lane == 0 && total) {
                b = atomicAdd(&P.fp_used[0], (unsigned long long)total);
                if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
                else atomicAdd(&P.fp_used[2], (unsigned long long)lsum);
            }
            const unsigned long long base = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)b, 0, 64)) |
                                            ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(b >> 32), 0, 64) << 32);
            const bool fits = base != ~0ull;
            const uint32_t excl = sincl - slot;
            if (spread && FAM == FAM_ALL && !SEGMODE) {
                // every family is here: the only punts are QUIC and OpenVPN,
                // for k_quic's list (as the fallback lane would hand them on);
                // so a small batch launches no fallback kernel
                if (fb) P.quic_idx[atomicAdd(P.quic_count, 1ull)] = (uint32_t)i;
            } else {
                const uint64_t fbm = __ballot(fb);
                if (fbm) {
                    uint32_t fb0 = 0;
                    if (lane == 0) fb0 = (uint32_t)atomicAdd(&P.fp_used[3], (unsigned long long)__builtin_popcountll(fbm));
                    fb0 = (uint32_t)__shfl((int)fb0, 0, 64);
                    if (fb) fallback[fb0 + __builtin_popcountll(fbm & ((1ull << lane) - 1))] = (uint32_t)i;
                }
            }
            if (SEGMODE) {
                // wave-cooperative expansion, one packet at a time, from the stage
                uint64_t todo2 = fits ? __ballot(len != 0) : 0ull;
                while (todo2) {
                    const int j = __builtin_ctzll(todo2);
                    todo2 &= todo2 - 1;
                    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
                    const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)excl, j);
                    const uint32_t ns = (uint32_t)__builtin_amdgcn_readlane((int)nseg, j);
                    const uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)(sbase + a16), j);
                    uint8_t *out = P.fp_arena + base + ex;
                    uint64_t h = seg_expand(segs + j * SEG_STRIDE, ns, stg + pj, T, out, pool, lane);
                    h = wave_xor64(h);
                    if (lane == 0) *(uint64_t *)(out + ((T + 7) & ~7u)) = mfpc::hash_final(h, T);
                }
            } else if (ONE_OK && spread && __builtin_amdgcn_readfirstlane((int)one)) {
                // (spread: lane 0 holds the wave's one packet) the string, with
                // its hash behind it, from the stage to the arena by the wave
                const uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane((int)(fits ? len : 0u));
                if (L) {
                    const uint32_t ex = (uint32_t)__builtin_amdgcn_readfirstlane((int)excl);
                    const uint32_t L8 = (L + 7) & ~7u;
                    uint64_t *dw = (uint64_t *)(P.fp_arena + base + ex);
                    const uint64_t *sw = (const uint64_t *)ebuf;
                    for (uint32_t k = lane; 8 * k < L8; k += 64) dw[k] = sw[k];
                    if (lane == 0) dw[L8 / 8] = one_hash;
                }
            } else {
                if (len && fits) {
                    Em<true> e;
                    e.begin(P.fp_arena + base + excl, out_line[lane]);
                    if (plan.ok) {
                        tls_ch_emit(e, plan);
                    } else {
                        Out o2;
                        packet_walk<FAM>(e, P.cfg, o2, data, dsc.caplen, dsc.linktype);
                    }
                    e.finish();
                    *(uint64_t *)(P.fp_arena + base + excl + ((len + 7) & ~7u)) = e.hash();
                }
            }
            if (in && !fb) {
                mfp_record r;
                r.fp_offset = fits ? base + excl : 0;
                r.fp_len = fits ? len : 0;
                r.fp_type = (uint8_t)(fits ? o.fp_type : 0);
                r.msg = (uint8_t)o.msg;
                r.flags = (uint8_t)(o.flags | (fits && len ? MFP_FLAG_HASHED : 0));
                r.xflags = (uint8_t)o.xflags;
                r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
                r.sni_len = (uint16_t)o.sni_len;
                r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
                r.ua_len = (uint16_t)o.ua_len;
                r.src_port = (uint16_t)o.src_port;
                r.dst_port = (uint16_t)o.dst_port;
                r.net = o.net;
                P.rec[i] = r;
            write_seg(P, i, o);
            }
            todo = todo && !in;
            __builtin_amdgcn_wave_barrier();   // the stage is rewritten by the next sub-round
        }
    }
    if (!SEGMODE && FAM == FAM_ALL && P.host_out) {
        // (every wave of the grid gets here: each has at least one packet)
        __threadfence_system();                       // this wave's records and strings
        if (lane == 0 && atomicAdd(P.fin, 1ull) == gridDim.x - 1) {
            __threadfence();
            unsigned long long u[4];
#pragma unroll
            for (int j = 0; j < 4; j++) u[j] = atomicExch(&P.fp_used[j], 0ull);
            atomicExch(P.quic_count, 0ull);
            atomicExch(P.fin, 0ull);
#pragma unroll
            for (int j = 0; j < 4; j++) P.host_out[j] = u[j];
            __threadfence_system();
            __hip_atomic_store(&P.host_out[4], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

#ifndef MFP_LDS_STAGE
#define MFP_LDS_STAGE (36 * 1024)   // per-wave stage of k_fp_lds: 40 KiB of LDS per wave, 4 waves per CU
#endif
#ifndef MFP_LDS_STAGE_SEG
#define MFP_LDS_STAGE_SEG (32 * 1024)
#endif

// A persistent bin kernel's grid as a whole number of resident rounds: its
// blocks take equal shares of the bin's tiles (static stride), so a grid of 2048
// at 3 blocks per CU (k_fp_tls1, 768 resident on 256 CUs) ran its last third of a
// round on two thirds of the CUs.  MFP_GRID_ROUND=0: the grid as given.
template <auto KERN>
inline uint32_t round_grid(uint32_t want) {
    static std::atomic<uint64_t> res_cache[64];
    const uint32_t res = (uint32_t)mfp_per_device(res_cache, [] {
        const char *e = getenv("MFP_GRID_ROUND");
        if (e && e[0] == '0') return 0u;
        int dev = 0, cus = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, KERN, TILE, 0) != hipSuccess || cus <= 0 || nb <= 0) {
            (void)hipGetLastError();
            return 0u;
        }
        return (uint32_t)(cus * nb);
    });
    return res && want > res ? want / res * res : want;
}

// one protocol bin's kernel: the LDS-staged walker (lds) or the HBM lane
// walker of family FAM; the HTTP segment variants are launched by
// mfp_launch_bin_seg (mfp_k_http.hip) whatever the bin
template <uint32_t FAM>
int launch_bin(const KParams &P, uint32_t *fallback, bool lds, const char *name, uint32_t lblocks, uint32_t fblocks,
               hipStream_t stream, mfp_prof *prof) {
    if (prof) mfp_prof_begin(prof, name, stream);
    if (lds) {
        hipLaunchKernelGGL((k_fp_lds<false, MFP_LDS_STAGE, FAM>), dim3(lblocks), dim3(64), 0, stream, P, fallback);
    } else {
        if constexpr (FAM == FAM_TLS && MFP_TLS_ONEPASS) {   // (bin kernels always have a fallback list)
            switch (P.cfg.tls_format) {
            case 1: hipLaunchKernelGGL(k_fp_tls1<1>, dim3(round_grid<k_fp_tls1<1>>(fblocks)), dim3(TILE), 0, stream, P, fallback); break;
            case 2: hipLaunchKernelGGL(k_fp_tls1<2>, dim3(round_grid<k_fp_tls1<2>>(fblocks)), dim3(TILE), 0, stream, P, fallback); break;
            default: hipLaunchKernelGGL(k_fp_tls1<0>, dim3(round_grid<k_fp_tls1<0>>(fblocks)), dim3(TILE), 0, stream, P, fallback); break;
            }
        } else
            hipLaunchKernelGGL(k_fingerprint<FAM>, dim3(round_grid<k_fingerprint<FAM>>(fblocks)), dim3(TILE), 0, stream, P,
                               fallback);
    }
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mfp

// the per-family launchers (mfp_k_*.hip): bin kernel `name` over P->idx / P->count
#define MFP_BIN_LAUNCHER(suffix) \
    extern "C" int mfp_launch_bin_##suffix(const mfp::KParams *P, uint32_t *fallback, int lds, const char *name, \
                                           uint32_t lblocks, uint32_t fblocks, hipStream_t stream, mfp_prof *prof)
MFP_BIN_LAUNCHER(tls);
MFP_BIN_LAUNCHER(http);
MFP_BIN_LAUNCHER(tcp);
MFP_BIN_LAUNCHER(ssh);
MFP_BIN_LAUNCHER(dtls);
MFP_BIN_LAUNCHER(all);
// the HTTP segment-expansion kernels (k_fp_lds<true> when lds, else k_fp_seg), and SSH's
MFP_BIN_LAUNCHER(seg);
MFP_BIN_LAUNCHER(ssh_seg);

