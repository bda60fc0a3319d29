#!/bin/bash
# Checkpoint A: every -m gpu test, smoke, a default bench line (with the CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ckpt
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "gpurun_out/ckpt/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a gpurun_out/ckpt/status.log
	return $rc
}
step tests 700 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests || exit $?
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 300 python -u bench.py
