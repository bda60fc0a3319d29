#!/bin/bash
# k_agg knobs on the headline (global walk) and the region walk: agg_ms per build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/aggab
mkdir -p $O
A="--steps 10 --warmup 4 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe"
for rep in 1 2; do
	for v in base ${VARIANTS}; do
		L=syzkaller_amd/libsyzsig.so; [ $v != base ] && L=exp/libsyzsig_$v.so
		for w in global region; do
			SYZSIG_LIB=$L timeout -k 10 300 python -u bench.py $A --walk $w > $O/${v}_${w}_$rep.log 2>&1
			rc=$?; echo "[$v $w $rep] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
		done
	done
done
exit 0
