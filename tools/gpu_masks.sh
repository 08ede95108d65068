#!/bin/bash
# parity tests, then fp-only bench per entry of $MASKS: WAVE or WAVE/SEG
# (MFP_BIN_WAVE_MASK / MFP_BIN_SEG_MASK; bit b = bin b on that kernel; bins:
# 0 tls_ch 1 http_req 2 tcp_syn 3 http_resp 4 other 5 tls_sh 6 ssh 7 dtls)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-masks}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for m in ${MASKS:-0x2}; do
  wm=${m%/*}; sm=0x0; case $m in */*) sm=${m#*/};; esac
  tag=${m//\//_}
  MFP_BIN_WAVE_MASK=$wm MFP_BIN_SEG_MASK=$sm timeout -k 10 300 python -u bench.py --packets ${PK:-10000000} --steps 5 --warmup 2 --no-cpu-baseline ${BENCH:---no-analysis} > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -5 $O/bench_$tag.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench_$tag.json'))
print('mask $m', d['value'], 'Mpkt/s', d['ms_per_step'], 'ms', ' '.join(f'{k}={v[\"ms_per_step\"]:.2f}' for k,v in d['kernels'].items()))"
done
