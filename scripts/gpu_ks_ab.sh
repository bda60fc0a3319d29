#!/bin/bash
# Edge kernel signals-per-lane variants: the executor goldens for each build,
# the full-C2 edge test for KS=2, then the edge line per build, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ks
mkdir -p $O
st() { echo "[$1] exit $2" >> $O/status.log; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_edge.py > $O/t1.log 2>&1; rc=$?; st t1 $rc; [ $rc -ne 0 ] && exit $rc
for k in ${KS_LIST:-ks2 ks3}; do
	SYZSIG_LIB=exp/libsyzsig_$k.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_edge.py > $O/t_$k.log 2>&1; rc=$?; st t_$k $rc; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
	for k in base ${KS_LIST:-ks2 ks3}; do
		if [ $k = base ]; then L=syzkaller_amd/libsyzsig.so; else L=exp/libsyzsig_$k.so; fi
		SYZSIG_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe > $O/b_${k}_$rep.log 2>&1; rc=$?; st b_${k}_$rep $rc; [ $rc -ne 0 ] && exit $rc
	done
done
exit 0
