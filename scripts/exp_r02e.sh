#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py tests/test_gpu_configs.py tests/test_ingest.py > gpurun_out/exp_e_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_e.log; [ $rc -ne 0 ] && exit $rc
bash scripts/sweep.sh
