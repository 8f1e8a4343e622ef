#!/bin/bash
# the run-based traceback walk: gotoh / aln2counts / filter tests, then the
# filter's chain and phase timings
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/tb
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_aln2counts.py tests/test_gpu_retry.py tests/test_gpu_e2e.py \
    tests/test_gpu_bench_parity.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 -u profiles/diag/filter_chain.py 2 > $O/filter_chain.txt 2>&1
timeout -k 10 300 python3 -u profiles/diag/filter_phases.py 2 > $O/filter_phases.txt 2>&1
echo diag ok
