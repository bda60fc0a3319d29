#!/bin/bash
# Round-3 GPU session: the given test files (TESTS), then a short bench.
# Each GPU step has its own time limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "[bench] exit $rc" | tee -a gpurun_out/${TAG}_status.log
exit $rc
