# GPU box: the parity files $PT (default test_gpu_parity.py) for each probe variant
# in $PV, then the A/B bench of $AB (tools/gpu_ab_lib.sh).  TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-ab}
mkdir -p gpurun_out/$T
PT=${PT:-tests/test_gpu_parity.py}
for v in $PV; do
  MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $PT > gpurun_out/$T/parity_$v.log 2>&1 || { tail -20 gpurun_out/$T/parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/$T/parity_$v.log)"
done
PK=${PK:-50000000} ST=${ST:-3} BENCH=${BENCH:-"--diverse-leg 0 --no-other-paths"} TAG=$T VARIANTS="$AB" bash tools/gpu_ab_lib.sh
