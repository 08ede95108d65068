# GPU box: parity of probe variants $PV, then the A/B bench of $AB (tools/ab_sort.sh)
PK=${PK:-50000000} ST=${ST:-3} BENCH=${BENCH:-"--diverse-leg 0 --no-other-paths"} bash tools/ab_sort.sh
