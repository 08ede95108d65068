#!/bin/bash
# GPU box: the GPU test suite, then (if it ended normally) smoke() and the
# default bench line.   tools/suite_and_bench.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
tail -3 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 560 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 400 $O/bench.json; echo
