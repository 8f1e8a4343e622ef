#!/bin/bash
# packed 16-B slot statistics: mapper parity tests, then the C2 collection
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/pack
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_parity_scale.py tests/test_gpu_fastpath.py tests/test_gpu_e2e.py \
    tests/test_gpu_bowtie2_cli.py > $O/tests.log 2>&1
echo tests ok
OUTNAME=c2_pack bash profiles/collect_r06.sh c2
