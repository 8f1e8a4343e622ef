# One SQ PMC pass over one C2 step (LDS / issue counters of k_pileup and
# k_dp); run on the GPU box from the repo root.  Output under
# gpurun_out/pmc_pileup/.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_pileup
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    -T --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/pmc.out 2>&1
echo done
