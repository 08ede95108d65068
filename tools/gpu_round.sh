#!/bin/bash
# GPU check: new-feature tests first (their failures do not stop the run),
# then the whole -m gpu suite; stops on a fault, abort or timeout.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${FIRST:-tests/test_stun_ovpn.py} -v --timeout 200 --timeout-method thread > gpurun_out/first.log 2>&1
rc=$?
echo "first exit $rc" >> gpurun_out/first.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu.log 2>&1
rc=$?
echo "gpu exit $rc" >> gpurun_out/gpu.log
exit $rc
