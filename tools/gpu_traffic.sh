#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes (one
# pass each) over a short config-4 bench run, summarised per launch by
# tools/pmc_traffic.py into profiles/${TAG}_traffic_*.json (which bench.py
# then reports as roofline.traffic).  TAG, PK (packets), BENCH (extra args).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r02t}
O=gpurun_out/$T
mkdir -p $O
PKN=${PK:-50000000}
B="python3 bench.py --packets $PKN --steps 4 --warmup 1 --no-cpu-baseline --e2e-total 0 --no-other-paths ${BENCH:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- $B > $O/kt.out 2>&1 || { tail -20 $O/kt.out; exit 1; }
echo "kernel-trace done"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o fetch -- $B > $O/fetch.out 2>&1 || { tail -5 $O/fetch.out; exit 1; }
echo "fetch done"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o write -- $B > $O/write.out 2>&1 || { tail -5 $O/write.out; exit 1; }
echo "write done"
KEY=${KEY:-mixed/$PKN/analysis/survey}
python tools/pmc_traffic.py $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv $KEY $O/traffic.json
tail -1 $O/kt.out
