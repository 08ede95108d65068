#!/bin/bash
# One gpurun call, steps chosen by STEPS (space separated, run in order, the
# first failure ends the call):
#   tests   python -m pytest tests -m gpu (TESTS= to select, e.g. "tests/test_tunnel.py -k json")
#   smoke   __graft_entry__.smoke()
#   bench   python bench.py $BENCH  -> gpurun_out/$TAG/bench.json
#   prof    rocprofv3 --kernel-trace --stats over a short bench run (PK packets)
# Output: gpurun_out/$TAG/.  Usage (from the dev container):
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'TAG=r03a STEPS="tests bench" bash tools/gpu_run.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-run}
O=gpurun_out/$T
mkdir -p $O
for s in ${STEPS:-tests}; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 \
        --timeout-method thread > $O/pytest.log 2>&1
      rc=$?; grep -E "passed|failed|error" $O/pytest.log | tail -3
      [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
      head -c 600 $O/bench.json; echo ;;
    prof)
      B="python3 bench.py --packets ${PK:-50000000} --steps 4 --warmup 1 --no-cpu-baseline --e2e-total 0 --no-other-paths ${BENCH:-}"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- $B > $O/kt.out 2>&1 || { tail -20 $O/kt.out; exit 1; }
      head -12 $O/kt/kt_kernel_stats.csv | cut -c1-160 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done"
