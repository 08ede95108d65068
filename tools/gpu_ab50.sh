#!/bin/bash
# new-feature tests, then an A/B of library variants at 50 M packets (config 4)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${FIRST:-tests/test_stun_ovpn.py} -q --timeout 300 --timeout-method thread > gpurun_out/first.log 2>&1
rc=$?; tail -3 gpurun_out/first.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${VARS:-default an4}; do
  lib=""; [ $v != default ] && lib=mercury_amd/_variants/libmercury_amd_$v.so
  MFP_LIB=$lib timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-total 0 \
      > gpurun_out/ab50_$v.json 2> gpurun_out/ab50_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab50_$v.json'));k=d['kernels'];print('$v', d['value'], d['ms_per_step'], k['k_analyze']['ms_per_step'], k['k_fingerprint/tls_ch']['ms_per_step'], k['k_classify']['ms_per_step'])"
done
