#!/bin/bash
# k_dp phase clock (throwaway build from profiles/diag/kdp_phases.py, copied
# to _v6/phases) on C2, then the C4 and C5 bench lines (collect_r06.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06/phases
timeout -k 10 300 env MICALL_HIP_LIB=$PWD/_v6/phases/libmicall_hip.so python -u bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-parity > gpurun_out/r06/phases/bench.json 2> gpurun_out/r06/phases/bench.err
rc=$?; echo "phases rc=$rc"; [ $rc = 0 ] || exit $rc
bash profiles/collect_r06.sh c4 && bash profiles/collect_r06.sh c5
