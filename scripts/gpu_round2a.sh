#!/bin/bash
# New config/concurrency tests first (each with its own limit), then the rest of -m gpu, then a bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a gpurun_out/status.log
	return $rc
}
step new_tests 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_concurrency.py tests/test_gpu_configs.py
rc=$?; [ $rc -gt 1 ] && exit $rc
step old_tests 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_concurrency.py
rc=$?; [ $rc -gt 1 ] && exit $rc
step bench 400 python -u bench.py --steps 10 --warmup 2
exit $?
