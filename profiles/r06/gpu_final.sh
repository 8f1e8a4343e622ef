#!/bin/bash
# the round's last build: the whole GPU suite, smoke, the default bench line
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/${OUTNAME:-final}
mkdir -p $O
cd $R
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
echo suite ok
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo smoke ok
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
