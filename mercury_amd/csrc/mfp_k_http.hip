// mfp_k_http.hip -- instantiates and launches the walkers of the FAM_HTTP parser family
// (mfp_kernels.hpp); compiled on its own so the families build in parallel.
#include "mfp_kernels.hpp"

MFP_BIN_LAUNCHER(http) {
    return mfp::launch_bin<mfp::FAM_HTTP>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}

MFP_BIN_LAUNCHER(seg) {
    if (prof) mfp_prof_begin(prof, name, stream);
    if (lds)
        hipLaunchKernelGGL((mfp::k_fp_lds<true, MFP_LDS_STAGE_SEG, mfp::FAM_HTTP>), dim3(lblocks), dim3(64), 0, stream, *P,
                           fallback);
    else
        hipLaunchKernelGGL(mfp::k_fp_seg<>, dim3(fblocks), dim3(mfp::TILE), 0, stream, *P, fallback);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

KPH_READER(http)
