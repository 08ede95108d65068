// h2d_probe.hip -- PCIe copy rates on the GPU box (tools/, never shipped):
// hipMemcpyAsync host->device and device->host from page-locked memory,
// both directions at once on two streams, and a copy kernel that pulls
// page-locked host memory into HBM (every lane 16-byte loads of host memory).
//   hipcc --offload-arch=gfx950 -O3 tools/h2d_probe.hip -o tools/h2d_probe && tools/h2d_probe [MB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

__global__ __launch_bounds__(256) void k_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = i + k < n16 ? src[i + k] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) if (i + k < n16) dst[i + k] = v[k];
    }
}
__global__ __launch_bounds__(256) void k_push(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const size_t bytes = mb << 20;
    uint8_t *h1, *h2, *d1, *d2;
    CK(hipHostMalloc((void **)&h1, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&h2, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&d2, bytes));
    memset(h1, 1, bytes);
    memset(h2, 2, bytes);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto rate = [&](const char *what, auto fn, double gb) {
        fn(); CK(hipDeviceSynchronize());
        double best = 1e9;
        for (int r = 0; r < 5; r++) {
            const double t0 = now();
            fn();
            CK(hipDeviceSynchronize());
            best = std::min(best, now() - t0);
        }
        printf("{\"what\": \"%s\", \"GB\": %.3f, \"ms\": %.3f, \"GB_per_s\": %.2f}\n", what, gb, best * 1e3, gb / best);
        fflush(stdout);
    };
    const double gb = bytes / 1e9;
    rate("memcpy_h2d", [&] { CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1)); }, gb);
    rate("memcpy_d2h", [&] { CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s1)); }, gb);
    rate("memcpy_h2d_d2h_two_streams", [&] {
        CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
    }, 2 * gb);
    rate("memcpy_h2d_4_pieces_2_streams", [&] {
        for (int k = 0; k < 4; k++)
            CK(hipMemcpyAsync(d1 + k * (bytes / 4), h1 + k * (bytes / 4), bytes / 4, hipMemcpyHostToDevice, k & 1 ? s2 : s1));
    }, gb);
    for (int grid : {256, 1024, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "pull_kernel_h2d_grid%d", grid);
        rate(nm, [&] { hipLaunchKernelGGL(k_pull, dim3(grid), dim3(256), 0, s1, (const uint4 *)h1, (uint4 *)d1, bytes / 16); }, gb);
        snprintf(nm, sizeof nm, "push_kernel_d2h_grid%d", grid);
        rate(nm, [&] { hipLaunchKernelGGL(k_push, dim3(grid), dim3(256), 0, s1, (const uint4 *)d2, (uint4 *)h2, bytes / 16); }, gb);
    }
    rate("pull_h2d_and_push_d2h_kernels", [&] {
        hipLaunchKernelGGL(k_pull, dim3(1024), dim3(256), 0, s1, (const uint4 *)h1, (uint4 *)d1, bytes / 16);
        hipLaunchKernelGGL(k_push, dim3(1024), dim3(256), 0, s2, (const uint4 *)d2, (uint4 *)h2, bytes / 16);
    }, 2 * gb);
    return 0;
}
