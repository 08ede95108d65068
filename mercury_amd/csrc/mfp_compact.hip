// mfp_compact.hip -- packs the fingerprint strings of a batch into a dense
// arena before they leave the device (mfp_process_pipelined / host batches).
//
// The fingerprint kernels place strings in reservation chunks (the wave
// kernel reserves 32 KiB per wave at a time, every string 16-byte aligned),
// so the arena has gaps.  Copying it to the host as is would move the gaps
// over PCIe; instead the strings are moved to offsets given by an exclusive
// prefix sum of the record lengths (packet order) and the records are
// rewritten to point there.  Three launches: per-block scan of fp_len,
// single-block scan of the block totals, then one wave per 64 records copies
// the strings with coalesced byte moves (lane l moves bytes l, l+64, ...).
// A record with a sidecar (MFP_FLAG_SIDECAR, QUIC) keeps it: its packed span
// is string, padding to 8, hash, sidecar (side_len from the sidecar header),
// so the record's spans stay valid; the packed total replaces used[2].
#include <hip/hip_runtime.h>

#include "../../include/mfp.h"
#include "mfp_internal.h"

namespace mfpk {

constexpr int B = 256;   // records per scan block

// bytes a record takes in the packed arena
__device__ __forceinline__ uint32_t packed_len(const mfp_record &r, const uint8_t *src) {
    if (r.flags & MFP_FLAG_SIDECAR) {
        const uint8_t *sc = src + r.fp_offset + ((r.fp_len + 7) & ~7u) + 8;
        return ((r.fp_len + 7) & ~7u) + 8 + ((uint32_t)sc[4] | (uint32_t)sc[5] << 8);
    }
    return r.fp_type ? r.fp_len : 0u;
}

__global__ __launch_bounds__(B) void k_len_scan(const mfp_record *rec, uint64_t n, const uint8_t *src, uint32_t *local,
                                                unsigned long long *block_sum) {
    __shared__ uint32_t wsum[B / 64];
    const uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t len = 0;
    if (i < n) { const mfp_record r = rec[i]; len = packed_len(r, src); }
    uint32_t incl = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < B / 64; w++) {
        if ((uint32_t)w < wid) base += wsum[w];
        tot += wsum[w];
    }
    if (i < n) local[i] = base + incl - len;
    if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

// exclusive scan of the block totals in place (one block; any count)
__global__ __launch_bounds__(1024) void k_block_scan(unsigned long long *block_sum, uint64_t nb,
                                                    unsigned long long *total) {
    __shared__ unsigned long long carry;
    __shared__ unsigned long long wsum[16];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint64_t k = b0 + threadIdx.x;
        const unsigned long long v = k < nb ? block_sum[k] : 0ull;
        unsigned long long incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        unsigned long long base = carry, tot = 0;
        for (uint32_t w = 0; w < 16; w++) {
            if (w < wid) base += wsum[w];
            tot += wsum[w];
        }
        if (k < nb) block_sum[k] = base + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(256) void k_compact_copy(mfp_record *rec, uint64_t n, const uint32_t *local,
                                                      const unsigned long long *block_sum, const uint8_t *src,
                                                      uint8_t *dst) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t g = wave; g * 64 < n; g += nw) {
        const uint64_t i = g * 64 + lane;
        uint64_t so = 0, dof = 0;
        uint32_t len = 0;
        if (i < n) {
            const mfp_record r = rec[i];
            len = packed_len(r, src);
            so = r.fp_offset;
            dof = block_sum[i / B] + local[i];
        }
        for (int j = 0; j < 64; j++) {
            const uint32_t lj = (uint32_t)__shfl((int)len, j, 64);
            if (!lj) continue;
            const uint64_t sj = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(so >> 32), j, 64) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)so, j, 64);
            const uint64_t dj = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dof >> 32), j, 64) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)dof, j, 64);
            for (uint32_t k = lane; k < lj; k += 64) dst[dj + k] = src[sj + k];
        }
        if (i < n && len) {
            rec[i].fp_offset = dof;
            rec[i].flags &= (uint8_t)~MFP_FLAG_HASHED;   // (a sidecar keeps the hash's 8 bytes as padding)
        }
    }
}

}  // namespace mfpk

// scratch: local = u32[n], block_sum = u64[(n + 255) / 256]; *total (device) =
// the packed bytes
extern "C" int mfp_launch_compact(mfp_record *rec, uint64_t n, const uint8_t *src, uint8_t *dst, uint32_t *local,
                                  unsigned long long *block_sum, unsigned long long *total, hipStream_t stream,
                                  mfp_prof *prof) {
    if (n == 0) return 0;
    const uint64_t nb = (n + mfpk::B - 1) / mfpk::B;
    if (prof) mfp_prof_begin(prof, "k_compact", stream);
    hipLaunchKernelGGL(mfpk::k_len_scan, dim3((uint32_t)nb), dim3(mfpk::B), 0, stream, rec, n, src, local, block_sum);
    hipLaunchKernelGGL(mfpk::k_block_scan, dim3(1), dim3(1024), 0, stream, block_sum, nb, total);
    uint64_t cb = (n + 255) / 256;
    if (cb > 2048) cb = 2048;
    hipLaunchKernelGGL(mfpk::k_compact_copy, dim3((uint32_t)cb), dim3(256), 0, stream, rec, n, local, block_sum, src, dst);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
