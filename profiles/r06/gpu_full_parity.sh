#!/bin/bash
# Whole-input record parity (every record of every pass against og_map, in
# 1M-unit chunks) for C2, C4, C4-all and C5 on this build, then the C4 and
# C5 bench lines with their CPU baselines
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/${OUTNAME:-full}
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --parity-full 1000000 > $O/c2_full.json 2> $O/c2_full.err
echo c2 ok
timeout -k 10 400 python3 bench.py --genomes hiv --pairs 5000000 --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --parity-full 1000000 > $O/c4_full.json 2> $O/c4_full.err
echo c4 ok
timeout -k 10 400 python3 bench.py --genomes all --pairs 5000000 --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --parity-full 1000000 > $O/c4all_full.json 2> $O/c4all_full.err
echo c4all ok
timeout -k 10 300 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --parity-full 1000000 > $O/c5_full.json 2> $O/c5_full.err
echo c5 ok
timeout -k 10 600 python3 bench.py --genomes hiv --pairs 5000000 --steps 3 --warmup 1 --no-e2e > $O/c4.json 2> $O/c4.err
echo c4 line ok
timeout -k 10 600 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err
echo c5 line ok
