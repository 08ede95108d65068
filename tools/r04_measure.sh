#!/bin/bash
# GPU box: suite + smoke + default bench (tools/suite_and_bench.sh), then the
# end-to-end copy-engine A/B (tools/gpu_e2e_sdma.sh).   tools/r04_measure.sh <outdir>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tools/suite_and_bench.sh "$1" || exit $?
TAG=${1#gpurun_out/}_sdma tools/gpu_e2e_sdma.sh
