#!/bin/bash
# Round-6 checkpoint on one MI355X: the fast-path probe against the previous
# ungapped_wide (_v6/old, expected to show fast-path cells the full DP
# beats), then the whole GPU suite on this build, then a C2 bench line.
# Every GPU step has its own limit; a fault / abort / signal ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 env MICALL_HIP_LIB=$PWD/_v6/old/libmicall_hip.so $PYT -x tests/test_gpu_fastpath.py \
    -k two_diagonals > gpurun_out/r06/probe_old.log 2>&1; rc=$?; echo "old build probe: rc=$rc"; ok $rc
timeout -k 10 900 $PYT -m gpu tests > gpurun_out/r06/gpu_suite.log 2>&1; rc=$?; echo "gpu suite: rc=$rc"; ok $rc
tail -n 3 gpurun_out/r06/gpu_suite.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-e2e > gpurun_out/r06/bench_c2b.json 2> gpurun_out/r06/bench_c2b.err
echo "bench rc=$?"
