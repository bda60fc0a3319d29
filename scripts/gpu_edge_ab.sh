#!/bin/bash
# K1+K2 implementations: the edge tests under SYZSIG_EDGE_IMPL=$IMPL, then the
# bench's edge line for impl 0 and $IMPL, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-edge}
IMPL=${IMPL:-1}
if [ -z "${NO_TESTS:-}" ]; then
	SYZSIG_EDGE_IMPL=$IMPL timeout -k 10 ${TEST_LIMIT:-500} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_edge.py} > gpurun_out/${TAG}_tests.log 2>&1
	rc=$?; echo "[tests impl $IMPL] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
	for im in 0 $IMPL; do
		SYZSIG_EDGE_IMPL=$im timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_e${im}_${rep}.log 2>&1
		rc=$?; echo "[edge impl $im rep $rep] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
	done
done
exit 0
