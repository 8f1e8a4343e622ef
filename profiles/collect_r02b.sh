# profiles/collect_r02b.sh -- the C3, C4 and C5 bench lines of the current
# build (run on the GPU box through gpurun from the repo root).  Outputs
# under gpurun_out/r02b/; the committed copies go to profiles/r02/{c3,c4,c5}.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02b
mkdir -p $O/c3 $O/c4 $O/c5
cd $R
timeout -k 10 400 python3 bench.py --genomes hiv --pairs 5000000 --steps 3 --warmup 1 --breakdown --no-cpu-baseline --no-e2e > $O/c4/bench.json 2> $O/c4/bench_breakdown.txt
echo c4 done
timeout -k 10 300 python3 bench.py --unpaired --read-len 300 --pairs 2000000 --no-cpu-baseline --no-e2e > $O/c5/bench.json 2> $O/c5/bench.err
echo c5 done
timeout -k 10 600 python3 bench.py --pairs 10000000 --iterations 3 --force-iterations --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/c3/bench.json 2> $O/c3/bench.err
echo c3 done
