#!/bin/bash
# GPU box: the FETCH/WRITE calibration kernels and the default bench line of
# a closing profile set whose traffic passes already ran (tools/r06_final.sh).  TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r06p}
O=gpurun_out/$T
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/cal_f -o cal_f -- tools/calib_fetch > $O/cal_f.out 2>&1 || { tail -5 $O/cal_f.out; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/cal_w -o cal_w -- tools/calib_fetch > $O/cal_w.out 2>&1 || { tail -5 $O/cal_w.out; exit 1; }
echo "calibration done"
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
echo "bench done"
tail -c 600 $O/bench.json
