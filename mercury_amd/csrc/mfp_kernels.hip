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

struct KParams {
    Cfg cfg;
    const uint8_t *arena;
    const mfp_pkt_desc *desc;
    uint64_t n;
    mfp_record *rec;
    uint8_t *fp_arena;
    uint64_t fp_cap;
    unsigned long long *fp_used;     // [0] bytes used, [1] overflow flag
};

__global__ __launch_bounds__(TILE) void k_fingerprint(KParams P) {
    // per-lane extension scratch for TLS formats 1/2 (dynamic: 0 bytes for
    // format 0, so the default path keeps full occupancy)
    extern __shared__ uint32_t dyn_lds[];
    uint32_t *lds_key = dyn_lds;
    uint16_t *lds_off = (uint16_t *)(dyn_lds + MAX_LDS_EXT * TILE);
    __shared__ uint32_t wave_tot[TILE / 64];
    __shared__ unsigned long long tile_base;

    const int tid = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * TILE + tid;
    const bool live = i < P.n;

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

    // workgroup exclusive scan of len
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t incl = len;
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
        uint32_t t = wave_tot[w];
        if (w < wid) wbase += t;
        total += t;
    }
    const uint32_t excl = wbase + incl - len;
    if (tid == 0) {
        unsigned long long b = total ? atomicAdd(&P.fp_used[0], (unsigned long long)total) : 0ull;
        if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
        tile_base = b;
    }
    __syncthreads();
    const unsigned long long base = tile_base;
    const bool fits = base != ~0ull;

    // pass 2: emit
    if (len && fits) {
        Em<true> e;
        e.begin(P.fp_arena + base + excl);
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
        r.flags = (uint8_t)o.flags;
        r.status = 0;
        r.sni_off = (uint16_t)(o.sni_len == 0xffff ? 0 : o.sni_off);
        r.sni_len = (uint16_t)o.sni_len;
        r.ua_off = (uint16_t)(o.ua_len == 0xffff ? 0 : o.ua_off);
        r.ua_len = (uint16_t)o.ua_len;
        r.src_port = (uint16_t)o.src_port;
        r.dst_port = (uint16_t)o.dst_port;
        r.reserved = 0;
        P.rec[i] = r;
    }
}

}  // namespace mfp

// launcher used by the host library (mfp_host.cpp)
extern "C" int mfp_launch_fingerprint(uint32_t select, uint32_t tls_format, uint32_t mode, const uint8_t *arena,
                                      const mfp_pkt_desc *desc, uint64_t n, mfp_record *rec, uint8_t *fp_arena,
                                      uint64_t fp_cap, unsigned long long *fp_used, hipStream_t stream) {
    if (n == 0) return 0;
    mfp::KParams P;
    P.cfg.select = select; P.cfg.tls_format = tls_format; P.cfg.mode = mode;
    P.arena = arena; P.desc = desc; P.n = n; P.rec = rec; P.fp_arena = fp_arena; P.fp_cap = fp_cap;
    P.fp_used = fp_used;
    uint64_t blocks = (n + mfp::TILE - 1) / mfp::TILE;
    size_t shmem = tls_format ? (size_t)mfp::MAX_LDS_EXT * mfp::TILE * 6 : 0;
    hipLaunchKernelGGL(mfp::k_fingerprint, dim3((uint32_t)blocks), dim3(mfp::TILE), shmem, stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
