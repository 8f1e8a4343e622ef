#!/bin/bash
# A/B of the prelim pileup over the winners only (this build) against the
# build before them (_v6/base): alternating C2 bench lines on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06/abonly
V=$PWD/_v6/base/libmicall_hip.so
for r in 1 2 3; do
  for which in base only; do
    if [ $which = base ]; then L=$V; else L=$PWD/micall-lite_amd/micall_amd/libmicall_hip.so; fi
    timeout -k 10 300 env MICALL_HIP_LIB=$L python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-parity \
        > gpurun_out/r06/abonly/$which.$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], d['ms_per_step'], k['k_seed'], k['k_dp'], k['k_pileup'], round(d['ms_per_step']-sum(k.values()),3))" gpurun_out/r06/abonly/$which.$r.json $which
  done
done
