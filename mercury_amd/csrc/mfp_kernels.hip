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

namespace mfp {

constexpr int TILE = 256;

// k_fingerprint -- lane-per-packet walker straight from HBM, grid-stride
// over tiles of TILE packets.  The fallback lane of the other bin kernels
// (packets larger than k_fp_lds's stage, segment lists that overflow); with
// idx == nullptr it processes the whole batch (MFP_STRATEGY=lane).
#ifndef MFP_LANE_MINW
#define MFP_LANE_MINW 4      // 4 waves per SIMD: measured best for the TLS CH and mixed bins
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
        } else {
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
        r.status = 0;
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
        packet_walk<FAM_HTTP>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
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
            write_seg(P, i, o);
        }
        __syncthreads();   // tile_base / wave_tot / segs reuse
    }
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
    __shared__ uint8_t pool[32];
    const uint32_t lane = threadIdx.x;
    uint8_t *stg = (uint8_t *)&stage[0];
    if (SEGMODE && lane < 32) {
        const char *lp = MFP_SEG_POOL;
        pool[lane] = (uint8_t)(lane < sizeof(MFP_SEG_POOL) ? lp[lane] : 0);
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t count = (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t g = blockIdx.x; g * 64 < count; g += gridDim.x) {
        const uint64_t t = g * 64 + lane;
        const bool live = t < count;
        const uint64_t i = live ? (uint64_t)P.idx[t] : 0;
        mfp_pkt_desc dsc;
        if (live) dsc = P.desc[i];
        else { dsc.offset = 0; dsc.caplen = 0; dsc.linktype = 0xffff; dsc.flags = 0; }
        const uint32_t a16 = (uint32_t)(dsc.offset & 15);
        const uint32_t pk_bytes = (a16 + dsc.caplen + 15) & ~15u;      // whole 16-byte blocks
        const uint32_t need = pk_bytes;
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
            for (uint64_t m = __ballot(in); m; m &= m - 1) {
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
            const uint8_t *data = stg + sbase + a16;

            Out o;
            uint32_t len = 0;
            bool fb = false;
            uint32_t nseg = 0;
            TlsPlan plan;
            plan.ok = false;
            if constexpr (SEGMODE) {
                SegEm e(data, segs + lane * SEG_STRIDE);
                if (in) {
                    packet_walk<FAM_HTTP>(e, P.cfg, o, data, dsc.caplen, dsc.linktype);
                    e.finish();
                    fb = e.ovf;
                    if (!fb && o.fp_type) {
                        if (e.valid()) len = e.n;
                        else o.fp_type = 0;
                    }
                    nseg = e.nseg;
                }
            } else {
                if (in) {
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
            {
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
                r.status = 0;
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
}

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

extern "C" int mfp_launch_quic(const void *kparams, uint8_t *scratch, uint32_t quic_format, uint32_t grid,
                               hipStream_t stream, mfp_prof *prof);

// launchers used by the host library (mfp_host.cpp)
#ifndef MFP_LDS_STAGE
#define MFP_LDS_STAGE (36 * 1024)   // per-wave stage of k_fp_lds: 40 KiB of LDS per wave, 4 waves per CU
#endif
#ifndef MFP_LDS_STAGE_SEG
#define MFP_LDS_STAGE_SEG (32 * 1024)
#endif
extern "C" int mfp_launch_fingerprint(uint32_t select, uint32_t tls_format, uint32_t mode, const uint8_t *arena,
                                      const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, mfp_tcp_seg *seg,
                                      uint8_t *fp_arena,
                                      uint64_t fp_cap, unsigned long long *fp_used, uint32_t *work,
                                      unsigned long long *bin_count, int strategy, uint32_t bin_seg_mask,
                                      uint32_t bin_lds_mask, uint32_t quic_format, uint8_t *quic_scratch,
                                      uint32_t quic_grid, hipStream_t stream, mfp_prof *prof) {
#define MFP_LAUNCH(name, ...)                                \
    do {                                                     \
        if (prof) mfp_prof_begin(prof, name, stream);        \
        hipLaunchKernelGGL(__VA_ARGS__);                     \
        if (prof) mfp_prof_end(prof, stream);                \
    } while (0)
    if (n == 0) return 0;
    mfp::KParams P;
    P.cfg.select = select; P.cfg.tls_format = tls_format; P.cfg.mode = mode; P.cfg.classify = 0;
    P.cfg.seg = seg ? 1u : 0u;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.fp_cap = fp_cap;
    P.fp_used = fp_used;
    P.seg = seg;
    P.idx = nullptr; P.count = nullptr;
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
        MFP_LAUNCH("k_fingerprint", mfp::k_fingerprint<mfp::FAM_ALL>, dim3((uint32_t)tiles), dim3(mfp::TILE), 0, stream,
                   P, nullptr);
        if (hipGetLastError() != hipSuccess) return -1;
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
        const dim3 lg((uint32_t)lblocks), fg((uint32_t)fblocks);
#define MFP_BIN(FAMILY)                                                                                          \
        do {                                                                                                     \
            if (lds && seg) MFP_LAUNCH(lds_name[b], (k_fp_lds<true, MFP_LDS_STAGE_SEG, FAM_HTTP>), lg, dim3(64), 0, \
                                       stream, P, fallback);                                                     \
            else if (lds) MFP_LAUNCH(lds_name[b], (k_fp_lds<false, MFP_LDS_STAGE, FAMILY>), lg, dim3(64), 0,     \
                                     stream, P, fallback);                                                       \
            else if (seg) MFP_LAUNCH(seg_name[b], k_fp_seg, fg, dim3(TILE), 0, stream, P, fallback);             \
            else MFP_LAUNCH(lane_name[b], k_fingerprint<FAMILY>, fg, dim3(TILE), 0, stream, P, fallback);       \
        } while (0)
        switch (b) {
        case 0: case 5: MFP_BIN(FAM_TLS); break;      // TLS ClientHello, ServerHello/Certificate
        case 1: case 3: MFP_BIN(FAM_HTTP); break;     // HTTP request, response
        case 2: MFP_BIN(FAM_TCP); break;              // SYN, SYN-ACK
        case 6: MFP_BIN(FAM_SSH); break;
        case 7: MFP_BIN(FAM_DTLS); break;
        default: MFP_BIN(FAM_ALL); break;             // no message of a selected protocol (or misbinned)
        }
#undef MFP_BIN
        if (hipGetLastError() != hipSuccess) return -1;
    }
    {
        // the fallback lane: every parser family, straight from HBM, over the
        // packets the bin kernels handed back (fp_used[3] of them)
        P.idx = fallback;
        P.count = fp_used + 3;
        const uint64_t fb = tiles < 1024 ? tiles : 1024;
        MFP_LAUNCH("k_fingerprint/fallback", k_fingerprint<FAM_ALL>, dim3((uint32_t)fb), dim3(TILE), 0, stream, P,
                   nullptr);
    }
    if (hipGetLastError() != hipSuccess) return -1;
    return launch_quic();
}
#undef MFP_LAUNCH
