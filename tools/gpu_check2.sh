#!/bin/bash
# new tests first, then a config-4 bench (k_analyze_wave regression check), then the whole suite
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${FIRST} -q --timeout 300 --timeout-method thread > gpurun_out/first.log 2>&1
rc=$?; tail -3 gpurun_out/first.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-total 0 > gpurun_out/chk.json 2> gpurun_out/chk.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/chk.json'));k=d['kernels'];print(d['value'], d['ms_per_step'], k['k_analyze']['ms_per_step'], k['k_analyze_wave']['ms_per_step'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu.log 2>&1
rc=$?; tail -3 gpurun_out/gpu.log; exit $rc
