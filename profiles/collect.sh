# profiles/collect.sh -- how the committed profiles were collected (run on the GPU box
# through gpurun from the repo root): full bench, rocprofv3 kernel trace + stats,
# then one separate --pmc pass per counter (FETCH_SIZE, WRITE_SIZE).
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_r01 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.out 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_write.out 2>&1
