#!/bin/bash
# cProfile of the host side of C2 and C4-all steps (profiles/diag/step_profile.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06/stepprof
timeout -k 10 300 python -u profiles/diag/step_profile.py 1000000 10 pol > gpurun_out/r06/stepprof/c2.txt 2>&1
rc=$?; echo "c2 rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u profiles/diag/step_profile.py 5000000 3 all > gpurun_out/r06/stepprof/c4all.txt 2>&1
echo "c4all rc=$?"
