#!/bin/bash
# A/B timing of libmicall_hip.so builds on one GPU box: alternates the
# in-tree build ("base") with variants/<name>/libmicall_hip.so, ROUNDS times,
# and prints k_dp / k_dp_rescue / k_pileup / step ms per run.
#   bash profiles/diag/ab_bench.sh ROUNDS name1 [name2 ...]
set -e
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset MICALL_HIP_LIB; else export MICALL_HIP_LIB=$PWD/variants/$v/libmicall_hip.so; fi
    timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab_$v.json
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$v.json'));k=d['kernels_ms_per_step'];print('%-10s k_dp %7.3f  k_dp_rescue %6.3f  k_rescue %6.3f  k_pileup %6.3f  k_seed %6.3f  step %7.3f' % ('$v', k['k_dp'], k['k_dp_rescue'], k['k_rescue'], k['k_pileup'], k['k_seed'], d['ms_per_step']))"
  done
done
