#!/bin/bash
# Quick GPU iteration: triage/shard parity tests, then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py} > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "[quick_tests] exit $rc" | tee -a gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1
rc=$?; echo "[quick_bench] exit $rc" | tee -a gpurun_out/status.log
exit $rc
