# A/B of C4 k_pileup: the in-tree build against variants/w2 (windows limited to
# what fits two 12-wave blocks per CU); run on the GPU box from the repo root.
set -e
for v in base w2 base w2; do
  if [ $v = base ]; then unset MICALL_HIP_LIB; else export MICALL_HIP_LIB=$PWD/variants/$v/libmicall_hip.so; fi
  timeout -k 10 300 python3 bench.py --genomes hiv --pairs 5000000 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/c4_$v.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/c4_$v.json'));k=d['kernels_ms_per_step'];print('$v', k['k_pileup'], k['k_dp'], d['ms_per_step'])"
done
