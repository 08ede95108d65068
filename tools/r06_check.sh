#!/bin/bash
# round 6: processor tests, then the default bench line with its reference
# output checks (each step under its own limit; stop at the first failure)
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_pkt_proc.py -m gpu -q -x --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 700 python -u bench.py > $out/bench.json 2> $out/bench.err; rc=$?
echo "bench rc=$rc"; tail -5 $out/bench.err
exit $rc
