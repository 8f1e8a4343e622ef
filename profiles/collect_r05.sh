# profiles/collect_r05.sh -- round-5 profiles (run on the GPU box through gpurun
# from the repo root):  bash profiles/collect_r05.sh [c2|c3|c5|c4|all]
# C2 (headline): bench line, rocprofv3 kernel trace + stats of the same
# command, separate PMC passes (FETCH_SIZE, WRITE_SIZE: one counter each) and
# one SQ issue pass.  C3 (10M pairs, 3 forced remap iterations) and C5's
# mapping half (2M unpaired 300-nt reads): bench lines with the stage
# breakdown.  C4: breakdown bench line + kernel stats.
# Outputs under gpurun_out/r05/.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
WHAT=${1:-all}
O=$R/gpurun_out/r05
mkdir -p $O/c2 $O/c3 $O/c4 $O/c4all $O/c5
cd $R
if [ "$WHAT" = c2 ] || [ "$WHAT" = all ]; then
  timeout -k 10 500 python3 bench.py --steps 20 --warmup 3 > $O/c2/bench.json 2> $O/c2/bench.err
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/c2/prof -o run \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-parity > $O/c2/bench_under_rocprof.json 2> $O/c2/prof.err
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/c2/pmc_fetch -o run \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/c2/pmc_fetch.out 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/c2/pmc_write -o run \
      -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/c2/pmc_write.out 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
      -T --output-format csv -d $O/c2/pmc_sq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity > $O/c2/pmc_sq.out 2>&1
  cd $R
  cp $(ls $O/c2/prof/*kernel_stats.csv $O/c2/prof/*/*kernel_stats.csv 2>/dev/null | head -1) $O/c2/run_kernel_stats.csv
  python3 profiles/pmc_summary.py $(ls $O/c2/pmc_fetch/*counter_collection.csv $O/c2/pmc_fetch/*/*counter_collection.csv 2>/dev/null | head -1) \
      $(ls $O/c2/pmc_write/*counter_collection.csv $O/c2/pmc_write/*/*counter_collection.csv 2>/dev/null | head -1) 1000000 $O/c2/pmc_traffic.json
  python3 profiles/sq_summary.py $(ls $O/c2/pmc_sq/*counter_collection.csv $O/c2/pmc_sq/*/*counter_collection.csv 2>/dev/null | head -1) $O/c2/sq_issue.json
  python3 profiles/kdp_launches.py $(ls $O/c2/prof/*kernel_trace.csv $O/c2/prof/*/*kernel_trace.csv 2>/dev/null | head -1) $O/c2/k_dp_launches.json
fi
if [ "$WHAT" = c3 ] || [ "$WHAT" = all ]; then
  timeout -k 10 600 python3 bench.py --pairs 10000000 --iterations 3 --force-iterations --steps 3 --warmup 1 \
      > $O/c3/bench.json 2> $O/c3/bench.err
fi
if [ "$WHAT" = c5 ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --steps 10 --warmup 2 \
      > $O/c5/bench.json 2> $O/c5/bench.err
fi
if [ "$WHAT" = c4all ] || [ "$WHAT" = all ]; then
  timeout -k 10 500 python3 bench.py --genomes all --pairs 5000000 --steps 3 --warmup 1 --breakdown \
      > $O/c4all/bench.json 2> $O/c4all/bench.err
fi
if [ "$WHAT" = c4 ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 python3 bench.py --genomes hiv --pairs 5000000 --steps 3 --warmup 1 --breakdown > $O/c4/bench.json 2> $O/c4/bench.err
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/c4/prof -o run \
      -- python3 $R/bench.py --genomes hiv --pairs 5000000 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-parity > $O/c4/bench_under_rocprof.json 2> $O/c4/prof.err
fi
echo collected
