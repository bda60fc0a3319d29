#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> short bench.  Each GPU step has its
# own time limit; a crash/timeout (exit > 1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-5}
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a gpurun_out/status.log
	return $rc
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
rc=$?; [ $rc -gt 1 ] && exit $rc
step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
rc=$?; [ $rc -gt 1 ] && exit $rc
step bench 600 python -u bench.py --steps "$STEPS" --warmup 1
exit $?
