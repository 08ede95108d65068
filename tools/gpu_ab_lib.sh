#!/bin/bash
# A/B of library variants (tools/build_probes.sh -> mercury_amd/_probe/) on
# one bench configuration: per variant the step rate and the per-kernel times.
#   VARIANTS="base an_noverify env:MFP_BIN_LDS_MASK=0xea ..."  (base = the in-tree library; env:...
#   the in-tree library under those variables), BENCH args, TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ab}
mkdir -p $O
B="--packets ${PK:-50000000} --steps ${ST:-4} --warmup 1 --no-cpu-baseline --e2e-total 0 ${BENCH:-}"
for v in ${VARIANTS:-base}; do
  envs=""
  case $v in
    base) unset MFP_LIB ;;
    env:*) unset MFP_LIB; envs=${v#env:} ;;   # the in-tree library under NAME=VALUE[,NAME=VALUE]
    *) export MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so ;;
  esac
  v=${v//[:=,]/_}
  env ${envs//,/ } timeout -k 10 300 python bench.py $B > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python - "$v" "$O/$v.json" <<'PY'
import json, sys
o = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {k: v["ms_per_step"] for k, v in o["kernels"].items()}
top = sorted(ks.items(), key=lambda x: -x[1])[:7]
print(f"{sys.argv[1]:14s} {o['value']:8.1f} Mpkt/s {o['ms_per_step']:8.2f} ms  " + "  ".join(f"{k}={v:.2f}" for k, v in top))
for key in ("wave_phase_clocks", "tls_phase_clocks", "http_phase_clocks"):
    ph = (o.get("analysis_counters") or {}).get(key)
    if ph:
        t = sum(ph) or 1
        print(f"   {key} (% of clocks): " + " ".join(f"{k}:{100 * v / t:.1f}" for k, v in enumerate(ph)))
PY
done
echo done
