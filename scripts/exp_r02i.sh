#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_triage.py > gpurun_out/exp_i_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_i.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/exp_i_smoke.log 2>&1
rc=$?; echo "[smoke] exit $rc" | tee -a gpurun_out/status_i.log; [ $rc -ne 0 ] && exit $rc
bash scripts/sweep.sh
