#!/bin/bash
# GPU box: full -m gpu suite, then smoke(); results under gpurun_out/$TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-round}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?
tail -3 $O/smoke.log
exit $rc
