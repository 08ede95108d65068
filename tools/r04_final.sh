#!/bin/bash
# GPU box, round-4 final: smoke(), the default bench line, then the
# profiles (tools/r04_final_b.sh: kernel-trace stats, FETCH/WRITE, SQ counters)
#   TAG=r04z tools/r04_final.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r04z}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 560 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
TAG=$T tools/r04_final_b.sh
