#!/bin/bash
# parity tests (default strategy) + bench for each strategy in $STRATS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for s in ${STRATS:-binned wave lane}; do
  MFP_STRATEGY=$s timeout -k 10 300 python bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline $BARGS > gpurun_out/bench_$s.json 2> gpurun_out/bench_$s.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_$s.json'));print('$s', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
