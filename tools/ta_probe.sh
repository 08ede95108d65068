#!/bin/bash
# GPU box: texture-address / L1 counters per kernel over 10 M packets (is the
# lane walkers' vector-memory pipe, not HBM, the limit?).  TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ta}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
B="python3 bench.py --packets 10000000 --steps 3 --warmup 1 --no-cpu-baseline --e2e-total 0 --diverse-leg 0 --no-other-paths"
pick() { local out=""; for c in "$@"; do grep -qw "${c%_sum}" $O/counters.txt && out="$out $c"; done; echo $out; }
P1=$(pick TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT)
P2=$(pick TD_TD_BUSY_sum TD_SPI_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum)
P3=$(pick TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum)
echo "P1=$P1"; echo "P2=$P2"; echo "P3=$P3"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1)); [ -z "$P" ] && continue
  timeout -s KILL 240 rocprofv3 --pmc $P -f csv -d $O/p$i -o p$i -- $B > $O/p$i.out 2>&1 || { tail -5 $O/p$i.out; exit 1; }
  echo "pass $i done"
done
python3 tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
grep -A12 "k_fp_tls1\|k_fp_seg<4" $O/pmc_summary.txt | head -60
