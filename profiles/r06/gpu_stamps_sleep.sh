#!/bin/bash
# SARS-CoV-2 strip stamps and the filter chain timings: this build against a
# variant whose poll loop sleeps 12 x 64 cycles between polls (not 2 x 64)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/stamps
mkdir -p $O
V=$PWD/_v6/sleep/libmicall_hip.so
timeout -k 10 300 env MICALL_HIP_LIB=$V python3 -u profiles/diag/gotoh_sars_stamps.py > $O/sars_sleep.json 2> $O/sars_sleep.err
timeout -k 10 300 env MICALL_HIP_LIB=$V python3 -u profiles/diag/filter_chain.py 2 > $O/chain_sleep.txt 2>&1
echo done
