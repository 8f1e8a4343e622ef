# profiles/collect_stages.sh -- per-stage kernel profiles (run on the GPU box
# through gpurun from the repo root):
#   bash profiles/collect_stages.sh
# For the headline remap bench and each --stage bench: the bench JSON line and
# a rocprofv3 --kernel-trace --stats run of the same command (csv), collected
# under gpurun_out/stages/<stage>/.  The committed copies live in profiles/r01/.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stages
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for st in remap sam2aln censor aln2counts; do
  mkdir -p $O/$st
  timeout -k 10 400 python3 $R/bench.py --stage $st --steps 3 --warmup 1 > $O/$st/bench.json 2> $O/$st/bench.err
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$st/prof -o run \
      -- python3 $R/bench.py --stage $st --steps 3 --warmup 1 --no-cpu-baseline > $O/$st/bench_under_rocprof.json 2> $O/$st/prof.err
  echo "stage $st done"
done
