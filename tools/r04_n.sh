#!/bin/bash
# GPU box: the round-4 closing profiles (tools/r04_final_b.sh) for the in-tree
# library, then the QUIC occupancy probe: its parity on the QUIC suites and the
# other-paths legs against the in-tree library
#   TAG=r04n tools/r04_n.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04n}
O=gpurun_out/$T
mkdir -p $O
TAG=$T tools/r04_final_b.sh || exit 1
MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_quic_w2.so timeout -k 10 300 python -u -m pytest -x -q -m gpu \
  --timeout 200 --timeout-method thread tests/test_quic.py tests/test_quic_reassembly.py > $O/parity_quic_w2.log 2>&1 \
  || { tail -30 $O/parity_quic_w2.log; exit 1; }
echo "quic_w2: $(tail -1 $O/parity_quic_w2.log)"
QUIC_LIBS="base quic_w2" tools/quic_phases.sh $O/quic
