#!/bin/bash
# reassembly + STUN/OpenVPN tests, the whole GPU suite, then k_analyze occupancy A/B at 10 M packets
mkdir -p gpurun_out
FIRST="tests/test_reassembly.py tests/test_stun_ovpn.py" bash tools/gpu_round.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in default an2 an3; do
  lib=""; [ $v != default ] && lib=mercury_amd/_variants/libmercury_amd_$v.so
  MFP_LIB=$lib timeout -k 10 300 python bench.py --packets 10000000 --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));k=d['kernels'];print('$v', d['value'], d['ms_per_step'], k['k_analyze']['ms_per_step'], k['k_analyze_wave']['ms_per_step'])"
done
