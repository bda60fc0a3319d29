#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_triage.py tests/test_gpu_edge.py tests/test_gpu_configs.py::test_c2_full_batch_vs_oracle > gpurun_out/exp_b_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_b.log; [ $rc -ne 0 ] && exit $rc
SYZSIG_EDGE_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_edge.py > gpurun_out/exp_b_edge8.log 2>&1
rc=$?; echo "[edge8 tests] exit $rc" | tee -a gpurun_out/status_b.log; [ $rc -ne 0 ] && exit $rc
printf 'SYZSIG_EDGE_WAVES=4\nSYZSIG_EDGE_WAVES=8\nSYZSIG_EDGE_WAVES=4\nSYZSIG_EDGE_WAVES=8\n' > /tmp/sw.txt
SWEEP_FILE=/tmp/sw.txt bash scripts/sweep.sh
