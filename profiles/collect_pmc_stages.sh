# profiles/collect_pmc_stages.sh -- HBM traffic of every stage's kernels: two
# separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of one bench step
# per stage, summarised by profiles/pmc_summary.py into
# gpurun_out/pmc_stages/pmc_traffic_<stage>.json (committed under profiles/).
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_stages
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for st in remap sam2aln censor aln2counts; do
  mkdir -p $O/$st
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d $O/$st/$c -o run \
        -- python3 $R/bench.py --stage $st --steps 1 --warmup 0 --no-cpu-baseline > $O/$st/$c.log 2>&1
  done
  python3 $R/profiles/pmc_summary.py $O/$st/FETCH_SIZE/run_counter_collection.csv \
      $O/$st/WRITE_SIZE/run_counter_collection.csv 1000000 $O/pmc_traffic_$st.json
  echo "pmc $st done"
done
