#!/bin/bash
# C4-all: the committed build (_v6/head: a git archive of HEAD with its own library)
# against the working tree, alternately, with the stage breakdown
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/c4ab
mkdir -p $O
for r in 1 2; do
  timeout -k 10 600 \
      python3 _v6/head/bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-parity --breakdown > $O/head.$r.json 2> $O/head.$r.err
  timeout -k 10 600 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-parity --breakdown > $O/tree.$r.json 2> $O/tree.$r.err
done
