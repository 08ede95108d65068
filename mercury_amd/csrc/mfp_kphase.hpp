// mfp_kphase.hpp -- phase clocks of the walker kernels (probe builds only).
#pragma once
#include <hip/hip_runtime.h>

// MFP_K_PHASES (probe builds): clock sums per phase of k_fp_tls1 / k_fp_seg in
// this translation unit's mfp_kphase[] (read by mfp_probe_read_<tu>)
#ifdef MFP_K_PHASES
static __device__ unsigned long long mfp_kphase[8];
#define KPH_DECL uint64_t kph_t = clock64(); uint64_t kph[5] = {0, 0, 0, 0, 0};
#define KPH(k) do { const uint64_t t_ = clock64(); kph[k] += t_ - kph_t; kph_t = t_; } while (0)
#define KPH_FLUSH() do { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 5; k_++) atomicAdd(&mfp_kphase[k_], (unsigned long long)kph[k_]); } while (0)
#define KPH_READER(suffix) \
    extern "C" MFP_EXPORT int mfp_probe_read_##suffix(unsigned long long *out) { \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(mfp_kphase), sizeof(mfp_kphase)) == hipSuccess ? 0 : -1; }
#else
#define KPH_DECL
#define KPH(k) do { } while (0)
#define KPH_FLUSH() do { } while (0)
#define KPH_READER(suffix)
#endif
