set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof
B="python bench.py --packets 5000000 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/kt -o kt -- $B > gpurun_out/prof/kt.out 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d gpurun_out/prof/p1 -o p1 -- $B > gpurun_out/prof/p1.out 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD -f csv -d gpurun_out/prof/p2 -o p2 -- $B > gpurun_out/prof/p2.out 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/prof/p3 -o p3 -- $B > gpurun_out/prof/p3.out 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/prof/p4 -o p4 -- $B > gpurun_out/prof/p4.out 2>&1
echo done
