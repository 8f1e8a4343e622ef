#!/bin/bash
# A/B of the candidate-major slot planes (this build) against HEAD's build
# (_v6/base): alternating C2 bench lines, then the mapping GPU tests and one
# FETCH_SIZE / WRITE_SIZE pass of this build
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/${ABNAME:-abslots}
mkdir -p $O
V=$PWD/_v6/base/libmicall_hip.so
for r in 1 2 3; do
  for which in base ${BNAME:-slots}; do
    if [ $which = base ]; then L=$V; else L=$PWD/micall-lite_amd/micall_amd/libmicall_hip.so; fi
    timeout -k 10 300 env MICALL_HIP_LIB=$L python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-parity \
        > $O/$which.$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], d['ms_per_step'], k)" $O/$which.$r.json $which
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_scale.py tests/test_gpu_retry.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $R/$O/pmc_fetch -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $R/$O/pmc_fetch.out 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $R/$O/pmc_write -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $R/$O/pmc_write.out 2>&1
cd $R
python3 profiles/pmc_summary.py $(ls $O/pmc_fetch/*counter_collection.csv $O/pmc_fetch/*/*counter_collection.csv 2>/dev/null | head -1) \
    $(ls $O/pmc_write/*counter_collection.csv $O/pmc_write/*/*counter_collection.csv 2>/dev/null | head -1) 1000000 $O/pmc_traffic.json
python3 -c "import json; d=json.load(open('$O/pmc_traffic.json'))['kernels']; print({k: round(v['hbm_bytes_per_launch']/1e9,3) for k,v in d.items() if v['hbm_bytes_per_launch']>1e7})"
