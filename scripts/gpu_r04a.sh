#!/bin/bash
# Round 4, first GPU pass: the tests touched by the stream-ordered step, the
# LDS records path and the advisor fixes; smoke; a short bench with every line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04a
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "gpurun_out/r04a/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a gpurun_out/r04a/status.log
	return $rc
}
step tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
	${TESTS:-tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py tests/test_gpu_dist.py tests/test_gpu_poll.py \
	tests/test_gpu_configs.py} || exit $?
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python -u bench.py --steps 10 --warmup 2 --no-cpu || exit $?
