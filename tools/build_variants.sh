#!/bin/bash
# Variant builds of libmercury_amd.so for A/B runs on the GPU box (MFP_LIB=<path>):
#   tools/build_variants.sh NAME "-DFLAG=..." [NAME2 "-D..."] ...
# Only $SRC (default mfp_kernels.hip) is rebuilt with the flags; the other
# objects are the default build's (run __graft_entry__.build() first).
set -e
cd "$(dirname "$0")/.."
mkdir -p mercury_amd/_variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  src=${SRC:-mfp_kernels.hip}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $flags -c mercury_amd/csrc/$src -o /tmp/var_$name.o
  objs=$(ls mercury_amd/_obj/*.o | grep -v "/$src.o")
  hipcc --offload-arch=gfx950 -shared -fPIC -o mercury_amd/_variants/libmercury_amd_$name.so /tmp/var_$name.o $objs -lz -lcrypto
  echo "built mercury_amd/_variants/libmercury_amd_$name.so ($flags)"
done
