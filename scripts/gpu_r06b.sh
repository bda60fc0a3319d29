#!/bin/bash
# Round 6: the ADVICE fixes' tests, then the K3 chain A/B of the scatter's
# workgroup shape: 2048 partitions (default), 1024 partitions with 128-B
# blocks (one 1024-thread workgroup per CU), 1024 with 64-B blocks in two
# workgroups per CU (w2b: 512 threads each; w2: 1024 threads each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06b}
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
	step tests "${TEST_LIMIT:-600}" python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS || exit $?
fi
A="--steps 10 --warmup 3 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for rep in 1 2; do
	for v in ${VARIANTS:-base s3a s3b p1024 w2b}; do
		case $v in
		base) E="" ;;
		p1024) E="SYZSIG_AGG_PARTS=1024" ;;
		w2|w2b) E="SYZSIG_AGG_PARTS=1024 SYZSIG_LIB=exp/libsyzsig_$v.so" ;;
		*) E="SYZSIG_LIB=exp/libsyzsig_$v.so" ;;
		esac
		step "k3_${v}_$rep" 240 env $E python -u bench.py $A || exit $?
	done
done
exit 0
