# profiles/collect_remap.sh -- headline (remap) profiles of the current build
# (run on the GPU box through gpurun from the repo root):
#   bash profiles/collect_remap.sh
# bench line, rocprofv3 kernel trace + stats of the same command, the two PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE: one counter per pass) and one pass of
# SQ issue counters, all under gpurun_out/remap/.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/remap
mkdir -p $O
cd $R
timeout -k 10 400 python3 bench.py --breakdown > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/prof.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.out 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.out 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    -T --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_sq.out 2>&1
echo collected
