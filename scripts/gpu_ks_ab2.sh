#!/bin/bash
# Edge kernel signals per lane (exp builds ks2, ks3) on the slot-resolution
# rounds: the executor goldens and full-C2 edge tests per build, then the edge
# line on both trace distributions, alternating with the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ks2
mkdir -p $O
for v in ${VARIANTS:-ks2 ks3}; do
	SYZSIG_LIB=exp/libsyzsig_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu \
		tests/test_gpu_edge.py tests/test_gpu_edge_c2.py > $O/tests_$v.log 2>&1
	rc=$?; echo "[tests $v] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
done
A="--steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --batches 1"
for rep in 1 2; do
	for v in base ${VARIANTS:-ks2 ks3}; do
		L=syzkaller_amd/libsyzsig.so; [ $v != base ] && L=exp/libsyzsig_$v.so
		for w in global region; do
			SYZSIG_LIB=$L timeout -k 10 200 python -u bench.py $A --walk $w > $O/${v}_${w}_$rep.log 2>&1
			rc=$?; echo "[$v $w $rep] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
		done
	done
done
exit 0
