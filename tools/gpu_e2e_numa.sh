#!/bin/bash
# End-to-end (host-resident, config 5) A/B: host threads and page-locked
# buffers anywhere vs on the GPU's NUMA node (MFP_E2E_NUMA=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-e2e_numa}
mkdir -p $O
for v in 0 1; do
  MFP_E2E_NUMA=$v timeout -k 10 400 python bench.py --packets 20000000 --steps 2 --warmup 1 --no-cpu-baseline \
    --diverse-leg 0 --no-other-paths > $O/numa$v.json 2> $O/numa$v.err || { tail -5 $O/numa$v.err; exit 1; }
  python -c "import json,sys; o=json.loads(open('$O/numa$v.json').read().strip().splitlines()[-1]); e=o['end_to_end']; print('numa=$v', e['value'], 'Mpkt/s H2D', e['h2d_gb_per_s_per_gpu'], 'GB/s D2H', e['d2h_gb_per_s_per_gpu'], 'json', e['json']['value'], e.get('numa'))"
done
