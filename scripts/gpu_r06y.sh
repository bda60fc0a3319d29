#!/bin/bash
# Round 6: the tile-fill threshold that sends a work item to k_scat3 instead of
# k_agg_scatter_blk, re-swept after the scatter changes (exp/libsyzsig_fill60,
# fill40.so: SYZ_SCAT3_FILL=60, 40; default 85) -- the K3 tests on fill40,
# then the Minimize line, the region-walk line and the K3 chain, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06y}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step tests 700 env SYZSIG_LIB=exp/libsyzsig_fill40.so python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
	tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py tests/test_gpu_configs.py || exit $?
A="--steps 10 --warmup 3 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for rep in 1 2; do
	for v in base fill60 fill40; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "min_${v}_$rep" 200 env $E python -u scripts/min_only.py || exit $?
		step "rw_${v}_$rep" 200 env $E python -u scripts/line_only.py rw || exit $?
		step "k3_${v}_$rep" 240 env $E python -u bench.py $A || exit $?
	done
done
exit 0
