# GPU box: parity + A/B of the LDS-staged ClientHello bin, then TA counters
PV="tls_stg" AB="base tls_stg env:MFP_BIN_LDS_MASK=0xa1" TAG=ab_stg1 PK=50000000 ST=3 BENCH="--diverse-leg 0 --no-other-paths" bash tools/ab_sort.sh && TAG=ta1 bash tools/ta_probe.sh
