#!/bin/bash
# GPU box, round-6 closing profiles on the final tree: rocprofv3 kernel-trace
# stats + FETCH_SIZE / WRITE_SIZE passes over config 4 (tools/gpu_traffic.sh),
# two SQ counter passes over 10 M packets, the FETCH/WRITE calibration
# kernels (tools/calib_fetch), then the default bench line.
#   TAG=r06g bash tools/r06_final.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r06g}
O=gpurun_out/$T
mkdir -p $O
TAG=$T BENCH="--diverse-leg 0" bash tools/gpu_traffic.sh || exit 1
cp $O/traffic.json profiles/${T}_traffic_50M_analysis_survey.json   # (the box copy: the bench below reports it)
B="python3 bench.py --packets 10000000 --steps 3 --warmup 1 --no-cpu-baseline --e2e-total 0 --diverse-leg 0 --no-other-paths"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SMEM -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || { tail -5 $O/p1.out; exit 1; }
echo "sq pass 1 done"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -f csv -d $O/p2 -o p2 -- $B > $O/p2.out 2>&1 || { tail -5 $O/p2.out; exit 1; }
echo "sq pass 2 done"
python tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/cal_f -o cal_f -- tools/calib_fetch > $O/cal_f.out 2>&1 || { tail -5 $O/cal_f.out; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/cal_w -o cal_w -- tools/calib_fetch > $O/cal_w.out 2>&1 || { tail -5 $O/cal_w.out; exit 1; }
echo "calibration done"
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
echo "bench done"
tail -c 600 $O/bench.json
