#!/bin/bash
# Round 6: k_scat3 with one slot claim per record, a claim past the block
# written at slot - kB after each flush (exp/libsyzsig_carry.so:
# SYZ_SCAT3_CARRY=1; the same sub-rounds and barriers, no second claim) -- the
# K3 tests on it, then the K3 chain and the Minimize line against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06x}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step tests 700 env SYZSIG_LIB=exp/libsyzsig_carry.so python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
	tests/test_gpu_triage.py tests/test_gpu_minimize_shard.py tests/test_gpu_configs.py || exit $?
A="--steps 10 --warmup 3 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for rep in 1 2; do
	for v in base carry; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "k3_${v}_$rep" 240 env $E python -u bench.py $A || exit $?
	done
	for v in base carry; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "min_${v}_$rep" 200 env $E python -u scripts/min_only.py || exit $?
	done
done
exit 0
