#!/bin/bash
# rocprofv3 kernel stats of the Minimize line alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/min_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/min_prof -o run -- python3 scripts/min_only.py > gpurun_out/min_prof/log 2>&1
echo "[minprof] exit $?"
