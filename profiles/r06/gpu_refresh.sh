#!/bin/bash
# C4, C5 and C3 lines with the round's last build (C3: the 200 000-pair
# parity leg; its whole-input check is profiles/r06/c3/parity_full.json)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/${OUTNAME:-refresh}
mkdir -p $O
cd $R
timeout -k 10 600 python3 bench.py --genomes hiv --pairs 5000000 --steps 3 --warmup 1 --no-e2e > $O/c4.json 2> $O/c4.err
echo c4 ok
timeout -k 10 600 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err
echo c5 ok
timeout -k 10 900 python3 bench.py --pairs 10000000 --iterations 3 --force-iterations --steps 3 --warmup 1 > $O/c3.json 2> $O/c3.err
echo c3 ok
