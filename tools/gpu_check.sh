#!/bin/bash
# GPU-box check: parity tests, then a short bench (A: wave kernel, B: lane-only kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_wave.json 2> gpurun_out/bench_wave.err || exit $?
cat gpurun_out/bench_wave.json
MFP_LANE_ONLY=1 timeout -k 10 300 python bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_lane.json 2> gpurun_out/bench_lane.err || exit $?
cat gpurun_out/bench_lane.json
