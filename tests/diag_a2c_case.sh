#!/bin/bash
# diagnostics: one aln2counts shard case (name in $1) with 2 ranks, under a
# short time limit, output under gpurun_out/a2c_case
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/a2c_case
rm -rf $O && mkdir -p $O/cases
cd $R/tests
python3 -c "
import os, shutil, sys
sys.path.insert(0, '$R/micall-lite_amd')
import test_gpu_shard_aln2counts as t
t._cases('$O/all')
shutil.move('$O/all/$1', '$O/cases/$1')
"
cd $R
PORT=$((20000 + RANDOM % 20000))
for r in 0 1; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT WORLD_SIZE=2 RANK=$r LOCAL_RANK=$r MICALL_DIST_BACKEND=gloo \
  MICALL_HIP_DEVICE=0 MICALL_TEST_STACKS=1 timeout -k 5 90 python3 -u tests/gpu_a2c_worker.py --cases $O/cases \
      > $O/rank$r.log 2>&1 &
done
wait
