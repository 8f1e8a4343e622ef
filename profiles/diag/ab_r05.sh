#!/bin/bash
# On-box A/B of round-5 k_dp variants (profiles/diag/build_variants_r05.sh):
# alternates the in-tree build with each variant, ROUNDS times, on C2
# (2x251 pairs) and C5 (unpaired 1x300), one bench line per run.
#   bash profiles/diag/ab_r05.sh ROUNDS
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
run() {   # variant, config name, bench args...
  local v=$1 cfg=$2; shift 2
  if [ "$v" = base ]; then unset MICALL_HIP_LIB; else export MICALL_HIP_LIB=$PWD/_ab/$v/libmicall_hip.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-parity --steps 5 --warmup 2 "$@" \
    > gpurun_out/ab/${cfg}_$v.json 2> gpurun_out/ab/${cfg}_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/${cfg}_$v.json'));k=d['kernels_ms_per_step'];print('%-4s %-11s k_dp %7.3f k_dp_rescue %6.3f step %7.3f' % ('$cfg', '$v', k['k_dp'], k['k_dp_rescue'], d['ms_per_step']))"
}
for r in $(seq "${1:-3}"); do
  for v in base noprefetch; do run $v c2; done
  for v in base multiround; do run $v c5 --unpaired --read-len 300 --pairs 2000000; done
done
