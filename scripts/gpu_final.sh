#!/bin/bash
# End-of-round check: every GPU test, smoke(), the default bench line, and the
# headline's rocprofv3 profile (trace + FETCH/WRITE/L2 passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-final}
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/${T}_status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "[smoke] exit $rc" | tee -a gpurun_out/${T}_status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "[bench] exit $rc" | tee -a gpurun_out/${T}_status.log; [ $rc -ne 0 ] && exit $rc
[ -n "${NO_PROF:-}" ] && exit 0
PROF_TAG=${T}_prof bash scripts/profile.sh
