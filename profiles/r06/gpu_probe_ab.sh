#!/bin/bash
# The fast-path probe (mh_probe_extend) against the previous ungapped_wide
# (_v6/old: expected to report fast-path cells the full DP beats) and this
# build; then the fast-path, index-cache and bench self-launch GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 env MICALL_HIP_LIB=$PWD/_v6/old/libmicall_hip.so $PYT tests/test_gpu_fastpath.py \
    -k two_diagonals > gpurun_out/r06/probe_old.log 2>&1; rc=$?; echo "old build: rc=$rc"; ok $rc
timeout -k 10 600 $PYT tests/test_gpu_fastpath.py tests/test_gpu_index_cache.py \
    > gpurun_out/r06/probe_new.log 2>&1; rc=$?; echo "new build: rc=$rc"; ok $rc
timeout -k 10 600 $PYT tests/test_gpu_bench_ranks.py -k own_ranks > gpurun_out/r06/ranks.log 2>&1
rc=$?; echo "self-launch: rc=$rc"
