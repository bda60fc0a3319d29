#!/bin/bash
# Round 6: the default bench line (all lines) with the final library against
# the one before k_agg's 32-bit indices (exp/libsyzsig_base72.so), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06w}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
for rep in 1 2; do
	for v in base base72; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "bench_${v}_$rep" 400 env $E python -u bench.py || exit $?
	done
done
exit 0
