# A/B timing of library variants built into variants/: one bench line per
# variant, same workload; a failing variant is reported and skipped.
cd $GRAFT_REPO_ROOT
for lib in variants/lib_*.so; do
  n=$(basename $lib .so)
  if MICALL_HIP_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err; then
    python -c "import json; d=json.load(open('gpurun_out/var_$n.json')); print('$n', d['value'], d['kernels_ms_per_step'])"
  else
    echo "$n failed: $(tail -1 gpurun_out/var_$n.err)"
    [ $? -ge 124 ] && break
  fi
done
