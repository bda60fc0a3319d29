#!/bin/bash
# Round 6: decomposition of the new default scatter (k_scat3) -- timing-only
# builds d1 (nothing placed) and d2 (blocks not stored) against the default and
# the round-5 scatter (old), then one SQ-counter pass of the default's K3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
A="--steps 10 --warmup 3 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for v in ${VARIANTS:-base old d1 d2}; do
	case $v in
	base) E="" ;;
	*) E="SYZSIG_LIB=exp/libsyzsig_$v.so" ;;
	esac
	step "k3_${v}_1" 240 env $E python -u bench.py $A || exit $?
done
if [ -n "${SQ:-1}" ]; then
	step sq 300 env PROF_TAG=$(basename $O)/sq PMC_KERNELS="k_scat3|k_agg<|k_agg_scatter" \
		BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll" \
		scripts/pmc_sq.sh || exit $?
fi
exit 0
