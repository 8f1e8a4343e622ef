#!/bin/bash
# the neighbour rows loaded a block ahead in k_gotoh_fwd / k_gotoh_bwd: the gotoh /
# aln2counts / filter tests, the filter timings, C4-all and C4 lines
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/pre
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_aln2counts.py tests/test_gpu_shard_aln2counts.py tests/test_gpu_retry.py \
    tests/test_gpu_e2e.py tests/test_gpu_bench_parity.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 -u profiles/diag/filter_chain.py 2 > $O/filter_chain.txt 2>&1
timeout -k 10 900 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e \
    > $O/c4all.json 2> $O/c4all.err
echo c4all ok
