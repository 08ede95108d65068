#!/bin/bash
# rocprofv3 kernel trace + SQ counters for the wave kernel (separate --pmc passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_${TAG:-x}
mkdir -p $O
B="python bench.py --packets ${PK:-5000000} --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- $B > $O/kt.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -f csv -d $O/p2 -o p2 -- $B > $O/p2.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/p3 -o p3 -- $B > $O/p3.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/p4 -o p4 -- $B > $O/p4.out 2>&1 || exit $?
echo done
