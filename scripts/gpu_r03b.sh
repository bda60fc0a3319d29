#!/bin/bash
# Round-3: remaining GPU tests (TESTS), bench, then the triage-line profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
if [ -n "${TESTS:-}" ]; then
	timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_tests.log 2>&1
	rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "[bench] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
[ -n "${NO_PROF:-}" ] && exit 0
PROF_TAG=${TAG}_prof bash scripts/profile.sh
