#!/bin/bash
# per-dispatch kernel trace of one strategy (MFP_STRATEGY), plus SQ counters per dispatch
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/trace_${TAG:-x}
mkdir -p $O
B="python bench.py --packets ${PK:-5000000} --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/kt -o kt -- $B > $O/kt.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH -f csv -d $O/p1 -o p1 -- $B > $O/p1.out 2>&1 || exit $?
echo done
