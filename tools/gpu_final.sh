#!/bin/bash
# Round-end measurement: the default bench line (config 4), then the
# kernel-trace + FETCH/WRITE passes over the same configuration (TAG).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r02v}
mkdir -p gpurun_out/$T
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json | head -c 400; echo
TAG=$T bash tools/gpu_traffic.sh
