#!/bin/bash
# Round 6: Minimize's work items through k_scat3 (exp/libsyzsig_ment{10,8}.so:
# per-record levels, 128-B blocks) -- the Minimize tests on it, then the
# Minimize line against the default, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06l}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step tests 600 env SYZSIG_LIB=exp/libsyzsig_ment10.so python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
	tests/test_gpu_minimize_shard.py tests/test_gpu_configs.py -k "minimize or c3" || exit $?
for rep in 1 2; do
	for v in base ment10 ment8; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "min_${v}_$rep" 200 env $E python -u scripts/min_only.py || exit $?
	done
done
exit 0
