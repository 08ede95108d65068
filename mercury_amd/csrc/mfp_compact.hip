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

// A small batch (the per-packet API, n <= 1024) in one launch: the scan in
// LDS, then the packed strings, the re-pointed records, the classifier's
// results and the counters written straight into the caller's page-locked
// host buffers (no device-to-host copies after it).  Strings are copied only
// when the packed total fits `cap` (the host reports the overflow).
__global__ __launch_bounds__(1024) void k_compact_small(const mfp_record *rec, uint32_t n, const uint8_t *src,
                                                        uint8_t *dst, uint64_t cap, mfp_record *rec_out,
                                                        const unsigned long long *used, unsigned long long *used_out,
                                                        const uint64_t *an, uint64_t *an_out, uint32_t an_words,
                                                        const uint64_t *ap, uint64_t *ap_out, uint32_t ap_words) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t s_off[1024], s_len[1024];
    __shared__ uint64_t s_src[1024];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    mfp_record r;
    uint32_t len = 0;
    if (tid < n) { r = rec[tid]; len = packed_len(r, src); }
    uint32_t incl = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) {
        if ((uint32_t)w < wid) base += wsum[w];
        total += wsum[w];
    }
    const uint32_t off = base + incl - len;
    if (tid < n) {
        s_off[tid] = off; s_len[tid] = len; s_src[tid] = r.fp_offset;
        if (len) { r.fp_offset = off; r.flags &= (uint8_t)~MFP_FLAG_HASHED; }
        rec_out[tid] = r;
    }
    __syncthreads();
    if ((uint64_t)total <= cap)
        for (uint32_t j = wid; j < n; j += 16) {
            const uint32_t L = s_len[j];
            const uint8_t *sj = src + s_src[j];
            uint8_t *dj = dst + s_off[j];
            for (uint32_t k = lane; k < L; k += 64) dj[k] = sj[k];
        }
    for (uint32_t k = tid; k < an_words; k += 1024) an_out[k] = an[k];
    for (uint32_t k = tid; k < ap_words; k += 1024) ap_out[k] = ap[k];
    if (tid == 0) { used_out[0] = used[0]; used_out[1] = used[1]; used_out[2] = total; used_out[3] = used[3]; }
    // used_out[4]: done -- every thread's host writes made visible first
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&used_out[4], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace mfpk

// k_compact_small's launch: every *_out pointer is page-locked host memory
// (hipHostMalloc) the device writes directly; an / ap may be null; used_host
// holds 5 words, [4] set last (the host polls it)
extern "C" int mfp_launch_compact_small(const mfp_record *rec, uint64_t n, const uint8_t *src, uint8_t *dst_host,
                                        uint64_t cap, mfp_record *rec_host, const unsigned long long *used,
                                        unsigned long long *used_host, const mfp_analysis *an, mfp_analysis *an_host,
                                        const double *ap, double *ap_host, hipStream_t stream, mfp_prof *prof) {
    static_assert(sizeof(mfp_analysis) % 8 == 0, "mfp_analysis copied as 8-byte words");
    if (n == 0 || n > 1024) return -1;
    const uint32_t an_words = an ? (uint32_t)(n * sizeof(mfp_analysis) / 8) : 0u;
    const uint32_t ap_words = ap ? (uint32_t)(n * MFP_ATTR_DB_TAGS) : 0u;
    if (prof) mfp_prof_begin(prof, "k_compact_small", stream);
    hipLaunchKernelGGL(mfpk::k_compact_small, dim3(1), dim3(1024), 0, stream, rec, (uint32_t)n, src, dst_host, cap,
                       rec_host, used, used_host, (const uint64_t *)an, (uint64_t *)an_host, an_words,
                       (const uint64_t *)ap, (uint64_t *)ap_host, ap_words);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

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

