#!/bin/bash
# Round 6, after the scatter's flush changes: smoke, the default bench line,
# and one SQ counter pass over the K3 kernels of the headline (wave-cycle
# breakdown, VALU/LDS instructions) for comparison with profiles/r06/sq_k3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06s}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python -u bench.py || exit $?
step sq 300 env PROF_TAG=r06s/sq PMC_KERNELS="k_scat3|k_agg<" \
	BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll" \
	scripts/pmc_sq.sh || exit $?
exit 0
