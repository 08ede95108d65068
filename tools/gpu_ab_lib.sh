#!/bin/bash
# A/B of library variants (tools/build_probes.sh -> mercury_amd/_probe/) on
# one bench configuration: per variant the step rate and the per-kernel times.
#   VARIANTS="base an_noverify ..."  (base = the in-tree library), BENCH args, TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ab}
mkdir -p $O
B="--packets ${PK:-50000000} --steps ${ST:-4} --warmup 1 --no-cpu-baseline --e2e-total 0 ${BENCH:-}"
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset MFP_LIB; else export MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so; fi
  timeout -k 10 300 python bench.py $B > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python - "$v" "$O/$v.json" <<'PY'
import json, sys
o = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {k: v["ms_per_step"] for k, v in o["kernels"].items()}
top = sorted(ks.items(), key=lambda x: -x[1])[:7]
print(f"{sys.argv[1]:14s} {o['value']:8.1f} Mpkt/s {o['ms_per_step']:8.2f} ms  " + "  ".join(f"{k}={v:.2f}" for k, v in top))
PY
done
echo done
