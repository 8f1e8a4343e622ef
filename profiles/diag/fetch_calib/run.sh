#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (and the raw request counters) per pattern kernel,
# one counter set per run; outputs under gpurun_out/r06/fetch_calib
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/fetch_calib
mkdir -p $O
B=$R/profiles/diag/fetch_calib/fetch_calib
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $B > $O/bytes.json
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/fetch -o run -- $B > $O/fetch.out 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/write -o run -- $B > $O/write.out 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -T --output-format csv -d $O/req -o run -- $B > $O/req.out 2>&1
echo calib ok
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum -T --output-format csv -d $O/req32 -o run -- $B > $O/req32.out 2>&1 || echo "req32 failed"
echo done
