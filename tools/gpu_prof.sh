#!/bin/bash
# Profiling pass over a short bench run: kernel-trace stats, SQ instruction /
# wait counters, FETCH_SIZE and WRITE_SIZE (separate passes), and the
# FETCH/WRITE calibration microbench (tools/calib_fetch).
#   TAG=name  output directory gpurun_out/<TAG>; PK packets; BENCH extra args
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-prof}
mkdir -p $O
B="python3 bench.py --packets ${PK:-10000000} --steps 3 --warmup 1 --no-cpu-baseline --e2e-total 0 ${BENCH:-}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- $B > $O/kt.out 2>&1 || { tail -20 $O/kt.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SMEM -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || { tail -5 $O/p1.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -f csv -d $O/p2 -o p2 -- $B > $O/p2.out 2>&1 || { tail -5 $O/p2.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/p3 -o p3 -- $B > $O/p3.out 2>&1 || { tail -5 $O/p3.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/p4 -o p4 -- $B > $O/p4.out 2>&1 || { tail -5 $O/p4.out; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum -f csv -d $O/p5 -o p5 -- $B > $O/p5.out 2>&1 || { tail -5 $O/p5.out; exit 1; }
if [ -x tools/calib_fetch ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/c1 -o c1 -- tools/calib_fetch > $O/c1.out 2>&1 || { tail -5 $O/c1.out; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/c2 -o c2 -- tools/calib_fetch > $O/c2.out 2>&1 || { tail -5 $O/c2.out; exit 1; }
fi
python tools/pmc_kernels.py $O/pmc.json $O/p1/p1_counter_collection.csv $O/p2/p2_counter_collection.csv $O/p3/p3_counter_collection.csv $O/p4/p4_counter_collection.csv $O/p5/p5_counter_collection.csv > $O/pmc.txt 2>&1
cat $O/pmc.txt
cat $O/c1.out | grep "^c_" || true
echo done
