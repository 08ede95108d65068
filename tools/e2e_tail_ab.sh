#!/bin/bash
# A/B of the pipeline's shrinking tail (MFP_PIPE_TAIL) on tools/e2e_probe.py, twice each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e_tail
for v in 0 1 0 1; do
  MFP_PIPE_TAIL=$v timeout -k 10 300 python tools/e2e_probe.py --chunk 1000000 --passes 3 > gpurun_out/e2e_tail/t$v.txt 2>&1 || { tail -3 gpurun_out/e2e_tail/t$v.txt; exit 1; }
  echo "tail=$v $(tail -n 1 gpurun_out/e2e_tail/t$v.txt)"
done
