set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02an1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -60 $O/pytest.log | grep -E "PASS|FAIL|ERROR|passed|failed" | tail -70
exit $rc
