#!/bin/bash
# follow-up of tools/gpu_suite.sh: the per-packet shim leg, then an A/B of
# library variants (VARIANTS, see tools/gpu_ab_lib.sh) on config 4
#   tools/after_suite.sh <outdir>
out=$1
tools/shim_bench.sh "$out" || exit $?
[ -n "$VARIANTS" ] && TAG=${out#gpurun_out/}_ab tools/gpu_ab_lib.sh
exit 0
