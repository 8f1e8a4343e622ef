set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sk; mkdir -p $O; cd $R
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastpath.py tests/test_gpu_e2e.py tests/test_gpu_retry.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/pmc_fetch.out 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/pmc_write.out 2>&1
cd $R
python3 profiles/pmc_summary.py $(ls $O/pmc_fetch/*counter_collection.csv $O/pmc_fetch/*/*counter_collection.csv 2>/dev/null | head -1) $(ls $O/pmc_write/*counter_collection.csv $O/pmc_write/*/*counter_collection.csv 2>/dev/null | head -1) 1000000 $O/pmc_traffic.json
