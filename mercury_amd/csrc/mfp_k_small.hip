// mfp_k_small.hip -- instantiates and launches the walkers of the FAM_TCP, FAM_SSH, FAM_DTLS parser families
// (mfp_kernels.hpp); compiled on its own so the families build in parallel.
#include "mfp_kernels.hpp"

MFP_BIN_LAUNCHER(tcp) {
    return mfp::launch_bin<mfp::FAM_TCP>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}

MFP_BIN_LAUNCHER(ssh) {
    return mfp::launch_bin<mfp::FAM_SSH>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}

MFP_BIN_LAUNCHER(dtls) {
    return mfp::launch_bin<mfp::FAM_DTLS>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}

// the SSH bin as segment lists: one walk, then each lane writes its string
// (k_fp_seg<FAM_SSH>), or the LDS-staged variant
MFP_BIN_LAUNCHER(ssh_seg) {
    if (prof) mfp_prof_begin(prof, name, stream);
    if (lds)
        hipLaunchKernelGGL((mfp::k_fp_lds<true, MFP_LDS_STAGE_SEG, mfp::FAM_SSH>), dim3(lblocks), dim3(64), 0, stream, *P,
                           fallback);
    else
        hipLaunchKernelGGL(mfp::k_fp_seg<mfp::FAM_SSH>, dim3(fblocks), dim3(mfp::TILE), 0, stream, *P, fallback);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
