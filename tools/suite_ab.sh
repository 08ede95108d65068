# GPU box: the whole GPU suite on the in-tree library, then the parity + A/B of probe variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-suite_ab}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
[ -n "$PV$AB" ] && TAG=$T bash tools/run_par_ab.sh
