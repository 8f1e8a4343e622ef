#!/bin/bash
# The prelim pileup's windows for the seed-group winners (skipped references'
# hits zeroed before the most-hit-first order): this build against HEAD's
# (_v6/base) on C4-all, C4 and C2, alternating; then the pileup GPU tests
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/abwin
mkdir -p $O
V=$PWD/_v6/base/libmicall_hip.so
N=$PWD/micall-lite_amd/micall_amd/libmicall_hip.so
run() {   # name lib args...
  local name=$1 lib=$2; shift 2
  timeout -k 10 400 env MICALL_HIP_LIB=$lib python3 bench.py "$@" --no-cpu-baseline --no-e2e --no-parity > $O/$name.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], d['ms_per_step'], k['k_pileup'])" $O/$name.json $name
}
for r in 1 2; do
  run c4all_base.$r $V --genomes all --pairs 5000000 --steps 3 --warmup 1
  run c4all_win.$r $N --genomes all --pairs 5000000 --steps 3 --warmup 1
done
run c4_base $V --genomes hiv --pairs 5000000 --steps 3 --warmup 1
run c4_win $N --genomes hiv --pairs 5000000 --steps 3 --warmup 1
run c2_base $V --steps 20 --warmup 3
run c2_win $N --steps 20 --warmup 3
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pileup" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
