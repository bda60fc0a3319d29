#!/bin/bash
# One GPU pass: the GPU tests in TESTS (none if empty), smoke (SMOKE=1), a
# bench run (BENCH_ARGS), and with PROF=1 a kernel trace of a short bench.
# Every step has its own time limit; the first failure ends the pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pass}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
if [ -n "${TESTS:-}" ]; then
	step tests 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS || exit $?
fi
if [ "${SMOKE:-0}" = 1 ]; then
	step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ -n "${BENCH_ARGS:-}" ]; then
	step bench 500 python -u bench.py $BENCH_ARGS || exit $?
fi
if [ "${PROF:-0}" = 1 ]; then
	step prof 500 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 bench.py ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu} || exit $?
fi
exit 0
