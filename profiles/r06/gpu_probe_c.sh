#!/bin/bash
# The round-5 counterexamples (tests/golden/fastpath_two_diagonal.json)
# through mh_probe_extend on the previous ungapped_wide (_v6/old: expected
# to FAIL, the fast path taking the worse cell) and on this build (pass).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 env MICALL_HIP_LIB=$PWD/_v6/old/libmicall_hip.so $PYT tests/test_gpu_fastpath.py \
    -k "counterexamples or two_diagonals" > gpurun_out/r06/probe_old_c.log 2>&1; rc=$?; echo "old build: rc=$rc"; ok $rc
timeout -k 10 300 $PYT tests/test_gpu_fastpath.py > gpurun_out/r06/probe_new_c.log 2>&1; rc=$?; echo "new build: rc=$rc"; ok $rc
