#!/bin/bash
# round 6: the driver's file -> JSON / pcap rate, then the two-rank bench
# rehearsed on one GPU (MFP_BENCH_DEVICE0: never a bench line)
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 600 python -u tools/drv_rate.py --loops 20 --batch 131072 524288 > $out/drv_rate.jsonl 2> $out/drv_rate.err || { echo "drv_rate failed"; tail -20 $out/drv_rate.err; exit 1; }
cat $out/drv_rate.jsonl
MFP_BENCH_DEVICE0=1 timeout -k 10 700 python -u bench.py --gpus 2 --packets 25000000 --steps 5 --warmup 2 --e2e-total 0 --no-other-paths --no-cpu-baseline > $out/bench2.json 2> $out/bench2.err; rc=$?
echo "bench2 rc=$rc"; tail -5 $out/bench2.err
exit $rc
