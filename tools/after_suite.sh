#!/bin/bash
# follow-up of tools/gpu_suite.sh: the per-packet shim leg, then an A/B of
# library variants (VARIANTS, see tools/gpu_ab_lib.sh) on config 4, then
# k_quic's phase clocks when QUIC_PHASES is set, then the end-to-end NUMA A/B
# when E2E_NUMA is set
#   tools/after_suite.sh <outdir>
out=$1
tools/shim_bench.sh "$out" || exit $?
if [ -n "$VARIANTS" ]; then TAG=${out#gpurun_out/}_ab tools/gpu_ab_lib.sh || exit $?; fi
if [ -n "$QUIC_PHASES" ]; then tools/quic_phases.sh "$out" || exit $?; fi
if [ -n "$E2E_NUMA" ]; then TAG=${out#gpurun_out/}_numa tools/gpu_e2e_numa.sh || exit $?; fi
exit 0
