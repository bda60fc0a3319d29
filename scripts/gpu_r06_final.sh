#!/bin/bash
# Round 6 final pass on one GPU: the whole GPU test suite, smoke, the default
# bench line.  Each step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_final}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
	step tests 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests || exit $?
fi
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python -u bench.py ${BENCH_ARGS:-} || exit $?
exit 0
