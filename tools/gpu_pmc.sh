#!/bin/bash
# SQ / TA counter passes over a short bench run (one pass per counter group),
# summarised per kernel by tools/pmc_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-pmc}
mkdir -p $O
B="python3 bench.py --packets ${PK:-10000000} --steps 2 --warmup 1 --no-cpu-baseline ${BENCH:-}"
if [ -n "$LIST" ]; then timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1; fi
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || { tail -5 $O/p1.out; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -f csv -d $O/p2 -o p2 -- $B > $O/p2.out 2>&1 || { tail -5 $O/p2.out; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum -f csv -d $O/p3 -o p3 -- $B > $O/p3.out 2>&1 || { tail -5 $O/p3.out; exit 1; }
python tools/pmc_summary.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
