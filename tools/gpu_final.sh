#!/bin/bash
# Round-end measurement on one MI355X: smoke(), the default bench line
# (config 4), the rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE
# passes of the same configuration (tools/gpu_traffic.sh, the diversity leg
# off so each step is one group of kernels), and two SQ counter passes.
#   TAG=name -> gpurun_out/<TAG>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r03z}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
TAG=$T BENCH="--diverse-leg 0" bash tools/gpu_traffic.sh || exit 1
B="python3 bench.py --packets 10000000 --steps 3 --warmup 1 --no-cpu-baseline --e2e-total 0 --diverse-leg 0 --no-other-paths"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SMEM -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || { tail -5 $O/p1.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -f csv -d $O/p2 -o p2 -- $B > $O/p2.out 2>&1 || { tail -5 $O/p2.out; exit 1; }
python tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
echo done
