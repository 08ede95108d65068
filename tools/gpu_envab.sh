#!/bin/bash
# A/B of environment knobs at 50 M packets (config 4): ENVS="name=VAR=value ..." (default first)
mkdir -p gpurun_out
for spec in default ${ENVS}; do
  name=${spec%%=*}; kv=${spec#*=}
  if [ "$spec" = default ]; then envs=""; else envs="$kv"; fi
  env $envs timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-total 0 \
      > gpurun_out/env_$name.json 2> gpurun_out/env_$name.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/env_$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], k['k_fingerprint/tls_ch' if 'k_fingerprint/tls_ch' in k else [x for x in k if 'tls_ch' in x][0]]['ms_per_step'], k['k_analyze']['ms_per_step'])"
done
