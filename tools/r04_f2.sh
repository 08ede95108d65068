#!/bin/bash
# GPU box: the GPU tests on the in-tree library, the walker parity tests on
# the MFP_HTTP_FAST=2 probe, then the A/B of the HTTP variants on config 4
#   TAG=r04x tools/r04_f2.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tests.log 2>&1 \
  || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_http_f2.so timeout -k 10 600 python -u -m pytest -x -q -m gpu \
  --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_tunnel.py tests/test_all.py > $O/parity_f2.log 2>&1 \
  || { tail -30 $O/parity_f2.log; exit 1; }
tail -2 $O/parity_f2.log
TAG=$T VARIANTS="${VARIANTS:-base http_f2 http_f2w3}" tools/gpu_ab_lib.sh
