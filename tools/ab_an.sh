#!/bin/bash
# GPU box: classifier parity (tests/test_analysis.py, test_gpu_parity analysis
# mode) of each probe variant, then the A/B bench.  PV, AB, TAG as tools/ab_sort.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r05an}
mkdir -p gpurun_out/$T
for v in $PV; do
  MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_analysis.py tests/test_json_analysis.py tests/test_gpu_parity.py -k "analysis or Analysis or classif or json" > gpurun_out/$T/parity_$v.log 2>&1 || { tail -20 gpurun_out/$T/parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/$T/parity_$v.log)"
done
TAG=$T VARIANTS="$AB" bash tools/gpu_ab_lib.sh
