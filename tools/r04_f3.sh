#!/bin/bash
# GPU box: walker parity on the HTTP probes (PROBES), then their A/B against
# the in-tree library on config 4
#   TAG=r04y tools/r04_f3.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04y}
O=gpurun_out/$T
mkdir -p $O
for pr in ${PROBES:-http_f3nw http_nw}; do
  MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$pr.so timeout -k 10 600 python -u -m pytest -x -q -m gpu \
    --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_tunnel.py tests/test_all.py > $O/parity_$pr.log 2>&1 \
    || { tail -30 $O/parity_$pr.log; exit 1; }
  echo "$pr: $(tail -1 $O/parity_$pr.log)"
done
TAG=$T VARIANTS="${VARIANTS:-base http_f3 http_nw http_f3nw base http_nw http_f3nw}" tools/gpu_ab_lib.sh
