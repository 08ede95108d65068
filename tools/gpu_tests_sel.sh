#!/bin/bash
# GPU-box: the -m gpu tests of the files given in $TESTS (default: all)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-sel}
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -40
exit $rc
