#!/bin/bash
# Minimize on the aggregation path: its tests, the triage tests (shared scatter), C3, then a bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_minimize_shard.py tests/test_gpu_triage.py tests/test_gpu_dist.py > gpurun_out/exp_j_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_j.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_configs.py -k c3 > gpurun_out/exp_j_c3.log 2>&1
rc=$?; echo "[c3] exit $rc" | tee -a gpurun_out/status_j.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/exp_j_bench.log 2>&1
rc=$?; echo "[bench] exit $rc" | tee -a gpurun_out/status_j.log; [ $rc -ne 0 ] && exit $rc
bash scripts/exp_r02k.sh
