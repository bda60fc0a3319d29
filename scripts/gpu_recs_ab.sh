#!/bin/bash
# A/B of records mode's sorted walk on the C4 rank line: the default
# one-thread-per-run k_recs_walk against k_recs_walk_wave (SYZSIG_AGG_DBG=512 =
# SYZSIG_DEBUG_RECS_WAVE), alternating, then a kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/recs_ab
O=gpurun_out/recs_ab
A="--steps 3 --warmup 1 --no-min --no-c5 --no-c1 --no-cpu"
for r in 1 2; do
	for v in 0 512; do
		SYZSIG_AGG_DBG=$v timeout -k 10 300 python -u bench.py $A > $O/run_${v}_$r.log 2>&1
		rc=$?; echo "[dbg=$v run $r] exit $rc" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
	done
done
export TMPDIR=/tmp
for v in 0 512; do
	SYZSIG_AGG_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py $A > $O/prof_$v.log 2>&1
	rc=$?; echo "[prof dbg=$v] exit $rc" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
