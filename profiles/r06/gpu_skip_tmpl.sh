#!/bin/bash
# The skipping k_pileup as its own template instance, and the Gotoh scratch
# kept across calls: C4-all twice as a fresh box's first processes (stage
# breakdown), then C2 A/B against the build without the skip (_v6/base),
# then the pileup and filter GPU tests
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/skiptmpl
mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-parity --breakdown \
      > $O/c4all.$r.json 2> $O/c4all.$r.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4all', d['ms_per_step'], d['kernels_ms_per_step']['k_pileup'])" $O/c4all.$r.json
  grep -o '"host.filter_conseqs": [0-9.]*' $O/c4all.$r.err || true
done
V=$PWD/_v6/base/libmicall_hip.so
for r in 1 2 3; do
  for which in base tmpl; do
    if [ $which = base ]; then L=$V; else L=$PWD/micall-lite_amd/micall_amd/libmicall_hip.so; fi
    timeout -k 10 300 env MICALL_HIP_LIB=$L python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-parity \
        > $O/$which.$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], d['ms_per_step'], k['k_seed'], k['k_dp'], k['k_pileup'], round(d['ms_per_step']-sum(k.values()),3))" $O/$which.$r.json $which
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pileup or filter or gotoh" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
