#!/bin/bash
# Round 6: is the scatter's bimodal per-process time the workspace's backing?
# Large workspaces sized in whole 2 MiB units (exp/libsyzsig_a2m.so:
# SYZ_WS_ALIGN2M=1) against the default, six alternating K3-only processes each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06z}
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
for rep in 1 2 3 4 5 6; do
	for v in base a2m; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "k3_${v}_$rep" 240 env $E python -u bench.py $A || exit $?
	done
done
exit 0
