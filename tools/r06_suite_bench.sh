#!/bin/bash
# GPU box: the whole GPU suite, smoke(), then the default bench line.  TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-r06s}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; o=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(o['value'], o['ms_per_step'], o['roofline']['frac'], o['roofline']['kernel_ms_per_launch'], o.get('output_check',{}).get('ok'))"
