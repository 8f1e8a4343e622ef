#!/bin/bash
# the filter's bound batch: its parity test, the filter's GPU tests, and the
# C4-all line with the pruned filter
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/bound
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "lev_bound or gotoh_distance or planes_need" \
    tests/test_gpu_bench_parity.py tests/test_gpu_parity_scale.py tests/test_gpu_e2e.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 900 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --breakdown \
    > $O/c4all.json 2> $O/c4all.err
echo c4all ok
