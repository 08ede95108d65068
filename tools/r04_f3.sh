#!/bin/bash
# GPU box: walker parity on the http_f3 probe, then the A/B against the in-tree library
#   TAG=r04y tools/r04_f3.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04y}
O=gpurun_out/$T
mkdir -p $O
MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_http_f3.so timeout -k 10 600 python -u -m pytest -x -q -m gpu \
  --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_tunnel.py tests/test_all.py > $O/parity_f3.log 2>&1 \
  || { tail -30 $O/parity_f3.log; exit 1; }
tail -2 $O/parity_f3.log
TAG=$T VARIANTS="${VARIANTS:-base http_f3 base http_f3}" tools/gpu_ab_lib.sh
