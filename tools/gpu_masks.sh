#!/bin/bash
# parity tests, then fp-only bench per MFP_BIN_WAVE_MASK value in $MASKS
# (bit b: bin b on the wave kernel; bins: 0 tls_ch 1 http_req 2 tcp_syn 3 http_resp 4 other)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-masks}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for m in ${MASKS:-0x2}; do
  MFP_BIN_WAVE_MASK=$m timeout -k 10 300 python -u bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline ${BENCH:---no-analysis} > $O/bench_$m.json 2> $O/bench_$m.err || { tail -5 $O/bench_$m.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench_$m.json'))
print('mask $m', d['value'], 'Mpkt/s', d['ms_per_step'], 'ms', ' '.join(f'{k}={v[\"ms_per_step\"]:.2f}' for k,v in d['kernels'].items()))"
done
