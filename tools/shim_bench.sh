#!/bin/bash
# the per-packet shim leg of bench.py on its own (tests/c/per_packet_bench)
out=$1
mkdir -p "$out"
timeout -k 10 300 python -u -c "
import json, sys; sys.path.insert(0, '.')
import bench
print(json.dumps(bench.per_packet_shim(2.0)))" > "$out/shim.json" 2> "$out/shim.err"
