#!/bin/bash
# one GPU iteration: parity tests, bench (wave), kernel trace + SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_wave.json 2> gpurun_out/bench_wave.err || exit $?
cat gpurun_out/bench_wave.json
[ -n "$NOPROF" ] && exit 0
TAG=${TAG:-it} bash tools/prof_wave.sh
