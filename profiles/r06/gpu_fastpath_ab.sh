#!/bin/bash
# A/B of the ungapped_wide fix: the low-complexity fast-path test
# against the previous build (_v6/old, expected to fail if the test reaches
# the two-off-diagonal case) and this build, then the parity suites and a C2
# bench line.  Every GPU step has its own time limit; a fault, abort, signal
# or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 env MICALL_HIP_LIB=$PWD/_v6/old/libmicall_hip.so $PYT tests/test_gpu_fastpath.py \
    -k low_complexity > gpurun_out/r06/fast_old.log 2>&1; rc=$?; echo "old build: rc=$rc"; ok $rc
timeout -k 10 600 $PYT tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_parity_scale.py \
    > gpurun_out/r06/fast_new.log 2>&1; rc=$?; echo "new build: rc=$rc"; ok $rc
[ $rc = 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-e2e > gpurun_out/r06/bench_c2.json 2> gpurun_out/r06/bench_c2.err
echo "bench rc=$?"
