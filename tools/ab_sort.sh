#!/bin/bash
# GPU box: parity (tests/test_gpu_parity.py) of each probe variant, then the
# A/B bench of the variants (tools/gpu_ab_lib.sh).  PV="v1 v2", AB="base v1 v2 base", TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r05s}
mkdir -p gpurun_out/$T
for v in $PV; do
  MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/$T/parity_$v.log 2>&1 || { tail -20 gpurun_out/$T/parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/$T/parity_$v.log)"
done
TAG=$T VARIANTS="$AB" bash tools/gpu_ab_lib.sh
