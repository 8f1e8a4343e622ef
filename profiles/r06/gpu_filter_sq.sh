#!/bin/bash
# SQ instruction mix of the filter batch's kernels (one PMC pass each)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/filter_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    -T --output-format csv -d $O/sq -o run -- python3 $R/profiles/diag/filter_batch_once.py > $O/sq.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR \
    -T --output-format csv -d $O/mix -o run -- python3 $R/profiles/diag/filter_batch_once.py > $O/mix.out 2>&1
echo done
