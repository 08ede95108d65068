#!/bin/bash
# fp-only bench with each probe variant of the library (tools/build_probes.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-probes}
mkdir -p $O
for v in base ${PROBES}; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/mercury_amd/${PRDIR:-_probe}/libmercury_amd_$v.so; fi
  MFP_LIB=$lib timeout -k 10 300 python -u bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline ${BENCH:---no-analysis} > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench_$v.json'))
print('$v', d['value'], 'Mpkt/s', d['ms_per_step'], 'ms', ' '.join(f'{k}={v[\"ms_per_step\"]:.2f}' for k,v in d['kernels'].items()))"
done
