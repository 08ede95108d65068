#!/bin/bash
# GPU box: the other-paths legs (QUIC Initials, STUN/OpenVPN, reassembly) per
# library in QUIC_LIBS (probe names under mercury_amd/_probe, or "base"); the
# phase-clock probe (quic_phases, MFP_K_PHASES) reports k_quic's phases.
#   QUIC_LIBS="quic_phases base" tools/quic_phases.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$1
mkdir -p $O
for v in ${QUIC_LIBS:-quic_phases}; do
  if [ "$v" = base ]; then unset MFP_LIB; else export MFP_LIB=$PWD/mercury_amd/_probe/libmercury_amd_$v.so; fi
  MFP_REPORT_PHASES=1 timeout -k 10 300 python -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
print(json.dumps(bench.other_paths(torch, 3)))" > $O/other_$v.json 2> $O/other_$v.err || { tail -5 $O/other_$v.err; exit 1; }
  python -c "
import json
o = json.loads(open('$O/other_$v.json').read())
q = o['quic_initials']; ph = q.get('quic_phase_clocks'); t = sum(ph) if ph else 1
print('$v', 'quic', q['value'], 'k_quic', q['kernel_ms'].get('k_quic'), 'cpu', q.get('cpu_baseline'),
      'phases%', [round(100 * x / t, 1) for x in ph] if ph else None)
print('   stun', o['stun_openvpn']['value'], 'reasm', o['reassembly']['value'], 'cpu', o['reassembly'].get('cpu_baseline'))"
done
