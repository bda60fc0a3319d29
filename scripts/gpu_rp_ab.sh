#!/bin/bash
# The owner side's LDS records kernels (k_rp_*) on the C4 rank line (kernel
# trace), after the records-mode and sharded-step GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/rpab
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py \
	tests/test_gpu_configs.py::test_c4_sharded_1b_vs_unsharded "tests/test_gpu_triage.py::test_records_mode_vs_oracle" \
	tests/test_gpu_minimize_shard.py > $O/tests.log 2>&1
rc=$?; echo "[tests] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/default -o run -- python3 scripts/line_only.py c4 > $O/default.log 2>&1
rc=$?; echo "[trace] exit $rc" >> $O/status.log
exit $rc
