#!/bin/bash
# GPU-box iteration: -m gpu tests (TESTS selects a subset), then one short bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-tb}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
timeout -k 10 600 python -u bench.py --no-cpu-baseline --e2e-total 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print('  %-28s %8.3f ms  %s GB/s'%(k, v['ms_per_step'], v['achieved_gb_s']))
"
