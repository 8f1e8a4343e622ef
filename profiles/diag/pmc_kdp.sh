# profiles/diag/pmc_kdp.sh -- issue/occupancy counters of the mapping kernels
# (run on the GPU box through gpurun from the repo root).
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_kdp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
   -T --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p1.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU \
   -T --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p2.out 2>&1
