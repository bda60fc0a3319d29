#!/bin/bash
# Round 6, first pass: the ADVICE fixes' tests (edge mark-all clear, poll
# fallback atomicity), the edge and poll suites, and a short bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r06a
mkdir -p $out
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$out/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a $out/status.log
	return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
	tests/test_gpu_edge.py tests/test_gpu_poll.py || exit $?
step bench 300 python -u bench.py --steps 10 --warmup 2 --no-cpu || exit $?
