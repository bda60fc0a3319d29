#!/bin/bash
# Edge dedup conflicts by decision slot (default build) vs by window (exp
# build dec0): the executor goldens and the full-C2 edge tests on the default
# build, then the edge line on both trace distributions, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dec
mkdir -p $O
[ "${SKIP_TESTS:-0}" = 1 ] || SYZSIG_LIB=${TEST_LIB:-syzkaller_amd/libsyzsig.so} timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_edge.py \
	tests/test_gpu_edge_c2.py > $O/tests.log 2>&1
rc=$?; echo "[tests] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
A="--steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --batches 1"
for rep in 1 2; do
	for v in ${VARIANTS:-dec dec0}; do
		L=syzkaller_amd/libsyzsig.so; [ $v != dec ] && L=exp/libsyzsig_$v.so
		for w in global region; do
			SYZSIG_LIB=$L timeout -k 10 200 python -u bench.py $A --walk $w > $O/${v}_${w}_$rep.log 2>&1
			rc=$?; echo "[$v $w $rep] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
		done
	done
done
exit 0
