#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_poll.py tests/test_gpu_minimize_shard.py tests/test_gpu_dist.py tests/test_gpu_signal.py > gpurun_out/exp_h_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_h.log
exit $rc
