#!/bin/bash
# A/B of the software-pipelined traceback bits in dp_pair's branch-free row
# groups (_v6/pipe) against this build: parity tests on the variant, then
# alternating C2 bench lines (no CPU baseline / e2e / parity).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06/abpipe
V=$PWD/_v6/pipe/libmicall_hip.so
timeout -k 10 600 env MICALL_HIP_LIB=$V python -u -m pytest -q -x --timeout 300 --timeout-method thread \
    tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_parity_scale.py > gpurun_out/r06/abpipe/tests.log 2>&1
rc=$?; echo "variant tests rc=$rc"; [ $rc = 0 ] || exit $rc
for r in 1 2 3; do
  for which in base pipe; do
    if [ $which = pipe ]; then L=$V; else L=$PWD/micall-lite_amd/micall_amd/libmicall_hip.so; fi
    timeout -k 10 300 env MICALL_HIP_LIB=$L python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-parity \
        > gpurun_out/r06/abpipe/$which.$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['kernels_ms_per_step']['k_dp'], d['kernels_ms_per_step']['k_dp_rescue'])" gpurun_out/r06/abpipe/$which.$r.json $which
  done
done
