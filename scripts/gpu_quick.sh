#!/bin/bash
# Quick loop: the triage / minimize / edge GPU tests, smoke, then a short bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/quick
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "gpurun_out/quick/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a gpurun_out/quick/status.log
	return $rc
}
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
	tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py tests/test_gpu_edge.py ${QUICK_TESTS:-} || exit $?
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 300 python -u bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_EXTRA:-}
