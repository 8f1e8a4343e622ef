# profiles/collect_r06.sh -- round-6 profiles (run on the GPU box through
# gpurun from the repo root):  bash profiles/collect_r06.sh c2|c4|c4all|c3|c5
# c2: the default bench line, a rocprofv3 kernel trace + stats of the same
#     command, separate PMC passes (FETCH_SIZE, WRITE_SIZE) and one SQ issue
#     pass; the summaries carry the kernel sources' fingerprint that bench.py
#     checks before it divides them by its own launch times.
# c4 / c4all / c5: bench lines with the CPU baseline and the consensus parity
#     leg (the oracle step with the consensus-distance filter).
# c3: 10M pairs, 3 forced remap iterations, --parity-full 1000000 (every
#     record of all 4 passes over the whole input against og_map, in chunks).
# Outputs under gpurun_out/r06/<config>/.  Each GPU step has its own limit;
# set -e ends the script at the first failure.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
WHAT=${1:?config}
O=$R/gpurun_out/r06/${OUTNAME:-$WHAT}
mkdir -p $O
cd $R
first() { ls $1/*$2 $1/*/*$2 2>/dev/null | head -1; }
case $WHAT in
c2)
  timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-parity > $O/bench_under_rocprof.json 2> $O/prof.err
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o run \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/pmc_fetch.out 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o run \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/pmc_write.out 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
      -T --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/pmc_sq.out 2>&1
  cd $R
  cp $(first $O/prof kernel_stats.csv) $O/run_kernel_stats.csv
  python3 profiles/pmc_summary.py $(first $O/pmc_fetch counter_collection.csv) $(first $O/pmc_write counter_collection.csv) 1000000 $O/pmc_traffic.json
  python3 profiles/sq_summary.py $(first $O/pmc_sq counter_collection.csv) $O/sq_issue.json
  python3 profiles/kdp_launches.py $(first $O/prof kernel_trace.csv) $O/k_dp_launches.json
  ;;
c4)
  timeout -k 10 600 python3 bench.py --genomes hiv --pairs 5000000 --steps 3 --warmup 1 --no-e2e --breakdown \
      > $O/bench.json 2> $O/bench.err
  ;;
c4all)
  timeout -k 10 1000 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --no-e2e --breakdown \
      > $O/bench.json 2> $O/bench.err
  ;;
c5)
  timeout -k 10 600 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --steps 10 --warmup 2 \
      > $O/bench.json 2> $O/bench.err
  ;;
c3)
  timeout -k 10 1100 python3 bench.py --pairs 10000000 --iterations 3 --force-iterations --steps 3 --warmup 1 \
      --parity-full 1000000 > $O/bench.json 2> $O/bench.err
  ;;
esac
echo collected $WHAT
