#!/bin/bash
# mh_pileup_only gated (the kernel's skip test only when a reference is
# skipped; the prelim pass counts the winners only when the others took >= 5 %
# of the mapped lines): tests, C4-all, then C2 A/B against the same build
# counting every reference (_v6/base)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/only2
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_parity_scale.py tests/test_gpu_e2e.py tests/test_gpu_shard.py \
    tests/test_gpu_bench_parity.py tests/test_gpu_chain.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 900 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e > $O/c4all.json 2> $O/c4all.err
echo c4all ok
bash profiles/r06/gpu_ab_only.sh
