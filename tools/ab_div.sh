#!/bin/bash
# GPU box: parity of the probe variants (classifier + prevalence tests), then
# the realistic-diversity leg per variant.  PV, AB, TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r05dv}
O=gpurun_out/$T
mkdir -p $O
for v in $PV; do
  MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_analysis.py tests/test_prevalence.py tests/test_shard.py > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
for v in $AB; do
  case $v in base) unset MFP_LIB ;; *) export MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so ;; esac
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-total 0 --no-other-paths > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python - "$v" "$O/$v.json" <<'PY'
import json, sys
o = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
d = o["diversity"]
print(f"{sys.argv[1]:10s} main {o['value']:7.1f}  diversity {d['value']:7.1f} Mpkt/s {d['ms_per_step']:6.2f} ms  kernels {d['kernel_ms']:6.2f}  " + " ".join(f"{k}={v:.2f}" for k, v in d["classifier_ms"].items()))
PY
done
