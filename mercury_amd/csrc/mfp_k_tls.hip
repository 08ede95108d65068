// mfp_k_tls.hip -- instantiates and launches the walkers of the FAM_TLS parser family
// (mfp_kernels.hpp); compiled on its own so the families build in parallel.
#include "mfp_kernels.hpp"

MFP_BIN_LAUNCHER(tls) {
    return mfp::launch_bin<mfp::FAM_TLS>(*P, fallback, lds != 0, name, lblocks, fblocks, stream, prof);
}

KPH_READER(tls)
