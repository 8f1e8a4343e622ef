#!/bin/bash
# HIP API + kernel + copy trace of short C2 runs (host gaps between kernels)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/hiptrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MH_INDEX_TRACE=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-parity > $O/bench.json 2> $O/bench.err
echo done
