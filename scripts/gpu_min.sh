#!/bin/bash
# Minimize: its GPU tests, then the line alone twice, then a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-min}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_minimize_shard.py "tests/test_gpu_configs.py::test_c3_minimize_vs_oracle" tests/test_gpu_dist.py > gpurun_out/$T/tests.log 2>&1
rc=$?; echo "[tests] exit $rc" | tee -a gpurun_out/$T/status.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
	timeout -k 10 120 python -u scripts/min_only.py > gpurun_out/$T/min_$i.log 2>&1
	rc=$?; echo "[min $i] exit $rc" | tee -a gpurun_out/$T/status.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$T/trace -o run -- python3 scripts/min_only.py > gpurun_out/$T/trace.log 2>&1
rc=$?; echo "[trace] exit $rc" | tee -a gpurun_out/$T/status.log
exit $rc
