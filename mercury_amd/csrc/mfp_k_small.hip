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
