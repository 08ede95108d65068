#!/bin/bash
# profiling variants of libmercury_amd.so (never shipped: mercury_amd/_probe/)
# usage: tools/build_probes.sh NAME:MACRO[,MACRO] ...
#   an_*: mfp_analysis.hip only; tls_* / http_*: that family's walker TU only (tlsk_* / httpk_*: and
#   mfp_kernels.hip, k_classify); quic_*: mfp_quic.hip;
#   anything else: every walker TU
set -e
cd "$(dirname "$0")/.."
mkdir -p mercury_amd/_probe
OBJ=mercury_amd/_obj
for spec in "$@"; do
  name=${spec%%:*}; macros=${spec#*:}
  defs=""; for m in ${macros//,/ }; do defs="$defs -D$m"; done
  if [[ $name == an_* ]]; then   # classifier probes: recompile mfp_analysis.hip only
    ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $defs -c mercury_amd/csrc/mfp_analysis.hip -o mercury_amd/_probe/a_$name.o &&
      hipcc --offload-arch=gfx950 -shared -fPIC -o mercury_amd/_probe/libmercury_amd_$name.so \
        mercury_amd/_probe/a_$name.o $(ls $OBJ/*.o | grep -v mfp_analysis.hip.o) -lz -lcrypto && echo built $name ) &
    continue
  fi
  (  # fingerprint probes: recompile the walker translation units
    objs=""
    tus="mfp_kernels mfp_k_tls mfp_k_http mfp_k_small mfp_k_all"
    case $name in tls_*) tus=mfp_k_tls ;; tlsk_*) tus="mfp_k_tls mfp_kernels" ;; http_*) tus=mfp_k_http ;;
                  httpk_*) tus="mfp_k_http mfp_kernels" ;; quic_*) tus=mfp_quic ;; esac   # probes of one family (+ k_classify)
    for k in $tus; do
      hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $defs -c mercury_amd/csrc/$k.hip \
        -o mercury_amd/_probe/k_${name}_$k.o & objs="$objs mercury_amd/_probe/k_${name}_$k.o"
    done
    wait
    hipcc --offload-arch=gfx950 -shared -fPIC -o mercury_amd/_probe/libmercury_amd_$name.so $objs \
      $(for o in $OBJ/*.o; do b=$(basename $o .hip.o); case " $tus " in *" $b "*) ;; *) echo $o ;; esac; done) \
      -lz -lcrypto && echo built $name ) &
done
wait
