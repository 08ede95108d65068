#!/bin/bash
# GPU-box round check: parity tests, bench lines, rocprofv3 kernel-trace stats
# and the HBM counter passes (FETCH_SIZE / WRITE_SIZE in separate runs).
#   TAG=name  output directory gpurun_out/<TAG>
#   BENCH_ARGS extra bench.py arguments for the profiled runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-round}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
timeout -k 10 600 python -u bench.py ${BENCH_MAIN:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -n "$BENCH_AN" ]; then
  timeout -k 10 600 python -u bench.py --no-analysis --no-cpu-baseline --e2e-total 0 > $O/bench_fp.json 2> $O/bench_fp.err || { tail -20 $O/bench_fp.err; exit 1; }
  cat $O/bench_fp.json
fi
P="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-total 0 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- $P > $O/kt.out 2>&1 || { tail -20 $O/kt.out; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o fetch -- $P > $O/fetch.out 2>&1 || { tail -20 $O/fetch.out; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o write -- $P > $O/write.out 2>&1 || { tail -20 $O/write.out; exit 1; }
python tools/pmc_traffic.py $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv "${TRAFFIC_KEY:-mixed/50000000/analysis}" $O/traffic.json || exit 1
echo done
