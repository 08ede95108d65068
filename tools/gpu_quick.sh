#!/bin/bash
# quick GPU iteration: selected parity tests (TESTS, default all gpu tests), then
# one bench line (BENCH args), no profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py --no-cpu-baseline ${BENCH:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'])
for k,v in d['kernels'].items(): print(f'  {k:28s} {v[\"ms_per_step\"]:9.3f} ms')
print(d.get('analysis'))"
fi
