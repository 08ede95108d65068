#!/bin/bash
# GPU suite + optional follow-up command, for gpurun: the follow-up runs only
# when pytest ended normally (all passed, or test failures: rc 0/1), never
# after a timeout, abort or crash.
#   tools/gpu_suite.sh <outdir> [pytest selection...] [-- follow-up command]
out=$1; shift
sel=(); follow=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; follow=("$@"); break; fi
  sel+=("$1"); shift
done
[ ${#sel[@]} -eq 0 ] && sel=(tests)
mkdir -p "$out"
timeout -k 10 1100 python -u -m pytest "${sel[@]}" -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$out/pytest.log"
if [ $rc -gt 1 ]; then exit $rc; fi
if [ ${#follow[@]} -gt 0 ]; then "${follow[@]}"; fi
