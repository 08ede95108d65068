#!/bin/bash
# End-to-end (host-resident, config 5) A/B of the host-to-device copy split
# (MFP_COPY_SPLIT=1: large copies over two streams / DMA engines; 0: one).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-e2e_ab}
mkdir -p $O
for v in 1 0; do
  MFP_COPY_SPLIT=$v timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --diverse-leg 0 \
    --no-json-leg > $O/split$v.json 2> $O/split$v.err || { tail -5 $O/split$v.err; exit 1; }
  python -c "import json,sys; o=json.loads(open('$O/split$v.json').read().strip().splitlines()[-1]); e=o['end_to_end']; print('split=$v', e['value'], 'Mpkt/s H2D', e['h2d_gb_per_s_per_gpu'], 'GB/s D2H', e['d2h_gb_per_s_per_gpu'])"
done
