#!/bin/bash
# Round-end measurement: smoke(), the default bench line (config 4), then the
# kernel-trace + FETCH/WRITE passes over the same configuration (TAG).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r02w}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
head -c 300 gpurun_out/$T/bench.json; echo
TAG=$T bash tools/gpu_traffic.sh
