#!/bin/bash
# GPU box: parity of the wide-load probe build (MFP_LIB) on the walker tests,
# then the A/B of the wide-load variants on config 4
#   TAG=r04w tools/r04_wide_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04w}
O=gpurun_out/$T
mkdir -p $O
MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_wide_all.so timeout -k 10 600 python -u -m pytest -x -q -m gpu \
  --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_tunnel.py tests/test_all.py > $O/parity_wide.log 2>&1 \
  || { tail -30 $O/parity_wide.log; exit 1; }
tail -2 $O/parity_wide.log
TAG=$T VARIANTS="${VARIANTS:-base http_fast http_wide tls_lb16 wide_all}" tools/gpu_ab_lib.sh
