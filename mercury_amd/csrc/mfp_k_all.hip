// mfp_k_all.hip -- instantiates and launches the walkers of the FAM_ALL parser family
// (mfp_kernels.hpp); compiled on its own so the families build in parallel.
#include "mfp_kernels.hpp"

MFP_BIN_LAUNCHER(all) {
    return mfp::launch_bin<mfp::FAM_ALL>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}
