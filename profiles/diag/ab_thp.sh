# profiles/diag/ab_thp.sh -- end-to-end C2 with the large host buffers on
# 4 KiB pages (MICALL_NO_THP=1) and on transparent huge pages, alternated.
set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/thp; mkdir -p $O; cd $R
for i in 1 2; do
  MICALL_NO_THP=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/nothp_$i.json 2> $O/nothp_$i.err
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/thp_$i.json 2> $O/thp_$i.err
done
