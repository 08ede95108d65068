#!/bin/bash
# per-packet API latency on the GPU box: tests/c/per_packet_bench (1 thread,
# write_json and get_analysis_context) plain, then under rocprofv3 kernel +
# memory-copy traces (no counters) for the device-side breakdown.
#   ENTRIES="json an" THREADS="1" SECS=2 PROF=1 TAG=pp
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-pp}
mkdir -p $O
python - $O/pkts.pcap <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
import bench
from tests import pcaplib, synth
a, d = synth.batch(20_000, seed=bench.TEMPLATE_SEED["mixed"], workload="mixed", n_templates=bench.N_TEMPLATES)
pk = [a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes() for x in d]
pcaplib.write_pcap(sys.argv[1], pk, linktype=1)
PY
LIB=${MFP_LIB:-$PWD/mercury_amd/libmercury_amd.so}
CFG="tls,dtls,ssh,http,tcp,tcp.syn_ack"
RES=$PWD/tests/golden/synth_resources.tgz
for e in ${ENTRIES:-json an}; do
  r=-; [ $e = an ] && r=$RES
  for t in ${THREADS:-1}; do
    MFP_SHIM_STATS=1 timeout -k 10 120 tests/c/per_packet_bench $LIB $O/pkts.pcap $CFG $r $t ${SECS:-2} $e \
      > $O/$e.$t.out 2> $O/$e.$t.err || { tail -5 $O/$e.$t.err; exit 1; }
    echo "$e threads=$t: $(tail -1 $O/$e.$t.out)"
    grep -h shim_ $O/$e.$t.err
  done
  if [ "${PROF:-1}" = 1 ]; then
    timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_$e -o run -- \
      tests/c/per_packet_bench $LIB $O/pkts.pcap $CFG $r 1 1 $e > $O/prof_$e.log 2>&1 || { tail -5 $O/prof_$e.log; exit 1; }
    for f in $(find $O/prof_$e -name '*stats.csv'); do echo "== $f"; head -25 $f; done
  fi
done
echo done
