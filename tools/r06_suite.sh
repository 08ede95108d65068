#!/bin/bash
# round 6: the whole GPU suite, then the reassembly probe and the two-rank
# rehearsal (MFP_BENCH_DEVICE0: never a bench line); stop at the first failure
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/reasm_probe.py > $out/reasm_probe.json 2> $out/reasm_probe.err || { tail -5 $out/reasm_probe.err; exit 1; }
cat $out/reasm_probe.json
MFP_BENCH_DEVICE0=1 timeout -k 10 700 python -u bench.py --gpus 2 --packets 25000000 --steps 5 --warmup 2 --e2e-total 0 --no-other-paths --no-cpu-baseline > $out/bench2.json 2> $out/bench2.err; rc=$?
echo "bench2 rc=$rc"
exit $rc
