#!/bin/bash
# Whole GPU suite on this build, then C4-all without the stage breakdown
# (its synchronisations inflate the step).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06/b
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/r06/b/gpu_suite.log 2>&1; rc=$?; echo "gpu suite: rc=$rc"; ok $rc
tail -n 3 gpurun_out/r06/b/gpu_suite.log
timeout -k 10 600 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline \
    > gpurun_out/r06/b/c4all.json 2> gpurun_out/r06/b/c4all.err
echo "c4all rc=$?"
