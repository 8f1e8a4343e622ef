#!/bin/bash
# Pileup windows capped so two blocks of 12 waves fit per CU
# (MH_PILE_WIN_HALF=1) against the uncapped windows, same build, alternating:
# C4, C4-all, C2
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/abwinhalf
mkdir -p $O
run() {   # name flag args...
  local name=$1 flag=$2; shift 2
  timeout -k 10 400 env MH_PILE_WIN_HALF=$flag python3 bench.py "$@" --no-cpu-baseline --no-e2e --no-parity > $O/$name.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], d['ms_per_step'], k['k_pileup'])" $O/$name.json $name
}
for r in 1 2; do
  run c4_full.$r 0 --genomes hiv --pairs 5000000 --steps 3 --warmup 1
  run c4_half.$r 1 --genomes hiv --pairs 5000000 --steps 3 --warmup 1
done
run c4all_full 0 --genomes all --pairs 5000000 --steps 3 --warmup 1
run c4all_half 1 --genomes all --pairs 5000000 --steps 3 --warmup 1
run c2_full 0 --steps 20 --warmup 3
run c2_half 1 --steps 20 --warmup 3
