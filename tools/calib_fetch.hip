// calib_fetch.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for
// the access widths and patterns of the fingerprint kernels (the MI355X guide
// calibrates only 16-B-per-lane streaming reads).  Each kernel reads (or
// writes) a known byte count from a buffer far larger than the 256 MiB
// Infinity Cache; the profiled counter divided by the known count is the
// correction factor for that pattern.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -- tools/calib_fetch      (then WRITE_SIZE)
//
// Patterns (one dispatch each, in this order):
//   c_stream16   16 B/lane, consecutive lanes consecutive (the guide's case)
//   c_stream4     4 B/lane, coalesced
//   c_lane4      lane per 512-B segment, the lane walks its segment with
//                dword loads (the lane walker's LeStream / ld_be32n pattern)
//   c_lane8      same with 8-byte loads (swar_find's pattern)
//   c_write16    16 B/lane coalesced stores
//   c_write8lane lane per 512-B segment, 8-byte stores (Em<true> line flush
//                is 16 B; k_fp_seg expansion is 8 B/lane coalesced)
//   c_write8     8 B/lane coalesced stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = (size_t)2 << 30;   // 2 GiB per pattern: ~8x the Infinity Cache
constexpr uint32_t SEG = 512;

__global__ void c_stream16(const uint4 *p, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void c_stream4(const uint32_t *p, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void c_lane4(const uint8_t *p, size_t nseg, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < nseg; s += (size_t)gridDim.x * blockDim.x) {
        const uint32_t *q = (const uint32_t *)(p + s * SEG);
        for (uint32_t k = 0; k < SEG / 4; k++) acc ^= q[k] + k;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void c_lane8(const uint8_t *p, size_t nseg, uint32_t *sink) {
    uint64_t acc = 0;
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < nseg; s += (size_t)gridDim.x * blockDim.x) {
        const uint64_t *q = (const uint64_t *)(p + s * SEG);
        for (uint32_t k = 0; k < SEG / 8; k++) acc ^= q[k] + k;
    }
    if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}
__global__ void c_write16(uint4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void c_write8lane(uint8_t *p, size_t nseg) {
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < nseg; s += (size_t)gridDim.x * blockDim.x) {
        uint64_t *q = (uint64_t *)(p + s * SEG);
        for (uint32_t k = 0; k < SEG / 8; k++) q[k] = s + k;
    }
}
__global__ void c_write8(uint64_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = i;
}

int main() {
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) { fprintf(stderr, "alloc\n"); return 1; }
    (void)hipMemset(buf, 1, BYTES);
    const dim3 grid(256 * 8), block(256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    auto run = [&](const char *name, auto launch) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("%-14s %10zu bytes %8.3f ms %8.1f GB/s\n", name, BYTES, ms, BYTES / (ms * 1e-3) / 1e9);
    };
    run("c_stream16", [&] { hipLaunchKernelGGL(c_stream16, grid, block, 0, 0, (const uint4 *)buf, BYTES / 16, sink); });
    run("c_stream4", [&] { hipLaunchKernelGGL(c_stream4, grid, block, 0, 0, (const uint32_t *)buf, BYTES / 4, sink); });
    run("c_lane4", [&] { hipLaunchKernelGGL(c_lane4, grid, block, 0, 0, (const uint8_t *)buf, BYTES / SEG, sink); });
    run("c_lane8", [&] { hipLaunchKernelGGL(c_lane8, grid, block, 0, 0, (const uint8_t *)buf, BYTES / SEG, sink); });
    run("c_write16", [&] { hipLaunchKernelGGL(c_write16, grid, block, 0, 0, (uint4 *)buf, BYTES / 16); });
    run("c_write8lane", [&] { hipLaunchKernelGGL(c_write8lane, grid, block, 0, 0, buf, BYTES / SEG); });
    run("c_write8", [&] { hipLaunchKernelGGL(c_write8, grid, block, 0, 0, (uint64_t *)buf, BYTES / 8); });
    (void)hipDeviceSynchronize();
    (void)hipFree(buf); (void)hipFree(sink);
    return 0;
}
