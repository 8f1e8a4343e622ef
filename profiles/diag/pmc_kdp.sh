# profiles/diag/pmc_kdp.sh -- SQ counters of the remap kernels (k_dp first),
# two separate rocprofv3 --pmc passes of one short bench step.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -T --output-format csv -d $R/gpurun_out/pmc/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --pairs 300000 > $R/gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -T --output-format csv -d $R/gpurun_out/pmc/p2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --pairs 300000 > $R/gpurun_out/pmc/p2.log 2>&1
