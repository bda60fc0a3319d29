#!/bin/bash
# Round 6: triage tests with the per-item scatter split, the K3 A/B of the
# flush-list / flush-batch variants, and the region-walk line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06g}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_triage.py \
	tests/test_gpu_configs.py tests/test_gpu_minimize_shard.py tests/test_gpu_dist.py} || exit $?
A="--steps 10 --warmup 3 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for v in ${VARIANTS:-base}; do
	case $v in
	base) E="" ;;
	*) E="SYZSIG_LIB=exp/libsyzsig_$v.so" ;;
	esac
	step "k3_${v}_1" 240 env $E python -u bench.py $A || exit $?
done
step rw 200 python -u scripts/line_only.py rw || exit $?
step c5 200 python -u scripts/line_only.py c5 || exit $?
step c1 200 python -u scripts/line_only.py c1 || exit $?
exit 0
