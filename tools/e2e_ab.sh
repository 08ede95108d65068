# A/B of the host pipeline's settings (tools/e2e_probe.py under environment variants)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { name=$1; shift; env "$@" timeout -k 10 300 python tools/e2e_probe.py $EXTRA > gpurun_out/e2e_$name.txt 2>&1 || { tail -3 gpurun_out/e2e_$name.txt; exit 1; }; echo "$name $(tail -n 1 gpurun_out/e2e_$name.txt)"; }
for v in ${VARIANTS:-A}; do
  case $v in
    A) run A MFP_PIPE_SLOTS=2 ;;
    D) run D MFP_PIPE_SLOTS=2 MFP_PIPE_INSTREAM=1 ;;
    C) run C MFP_PIPE_SLOTS=3 MFP_PIPE_INSTREAM=1 ;;
    D1) EXTRA="--chunk 1000000" run D1 MFP_PIPE_SLOTS=2 MFP_PIPE_INSTREAM=1 ;;
    D50) EXTRA="--packets 50000000 --passes 1" run D50 MFP_PIPE_SLOTS=2 MFP_PIPE_INSTREAM=1 ;;
    A50) EXTRA="--packets 50000000 --passes 1" run A50 MFP_PIPE_SLOTS=2 ;;
    C1) EXTRA="--chunk 1000000" run C1 MFP_PIPE_SLOTS=3 ;;
    D05) EXTRA="--chunk 500000" run D05 MFP_PIPE_SLOTS=2 ;;
    N1) EXTRA="--chunk 1000000" run N1 MFP_PIPE_SLOTS=2 MFP_PIPE_INSTREAM=0 ;;
    DP) MFP_PIPE_SLOTS=2 MFP_PIPE_INSTREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_profD -o run -- python tools/e2e_probe.py --passes 1 > gpurun_out/e2e_profD.log 2>&1 || exit 1 ;;
  esac
done
