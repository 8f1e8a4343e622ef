#!/bin/bash
# one 16-B hash entry per slot: mapper parity tests, then the C2 collection
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/hent
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_parity_scale.py tests/test_gpu_fastpath.py tests/test_gpu_e2e.py \
    tests/test_gpu_bowtie2_cli.py tests/test_gpu_index_cache.py tests/test_gpu_shard.py > $O/tests.log 2>&1
echo tests ok
OUTNAME=c2_hent bash profiles/collect_r06.sh c2
