#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_triage.py tests/test_gpu_configs.py::test_c2_full_batch_vs_oracle > gpurun_out/exp_d_tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/status_d.log; [ $rc -ne 0 ] && exit $rc
bash scripts/sweep.sh || exit $?

