#!/bin/bash
# A/B bench lines on one box: tests first (unless SKIP_TESTS), then one short
# bench per "name=ENVSPEC" argument (ENVSPEC: space-separated VAR=value, e.g.
# "MFP_LIB=mercury_amd/_variants/libmercury_amd_x.so MFP_BIN_LDS_MASK=0x1").
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-total 0 --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$name.json'))
print('== $name', 'value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print('  %-28s %8.3f ms  %s GB/s'%(k, v['ms_per_step'], v['achieved_gb_s']))
"
done
