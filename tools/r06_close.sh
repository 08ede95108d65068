#!/bin/bash
# round 6: the whole GPU suite and smoke on the final tree, the driver's
# file -> JSON rate, then the default bench line; stop at the first failure
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u tools/drv_rate.py --loops 20 --batch 131072 524288 > $out/drv_rate.jsonl 2> $out/drv_rate.err || { tail -5 $out/drv_rate.err; exit 1; }
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 300 $out/bench.json
exit $rc
