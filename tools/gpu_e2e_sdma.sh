#!/bin/bash
# End-to-end (host-resident, config 5) A/B of the copy engine: SDMA (default)
# against HIP's blit kernels (HSA_ENABLE_SDMA=0: shader copies over PCIe).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-e2e_sdma}
mkdir -p $O
for v in 1 0; do
  HSA_ENABLE_SDMA=$v timeout -k 10 400 python bench.py --packets 20000000 --steps 2 --warmup 1 --no-cpu-baseline \
    --diverse-leg 0 --no-json-leg --no-other-paths > $O/sdma$v.json 2> $O/sdma$v.err || { tail -5 $O/sdma$v.err; exit 1; }
  python -c "import json,sys; o=json.loads(open('$O/sdma$v.json').read().strip().splitlines()[-1]); e=o['end_to_end']; print('sdma=$v', e['value'], 'Mpkt/s H2D', e['h2d_gb_per_s_per_gpu'], 'GB/s D2H', e['d2h_gb_per_s_per_gpu'])"
done
