#!/bin/bash
# A/B of library variants on one box: bench.py's triage line (no CPU, no
# Minimize) once per env setting in AB (space-separated VAR=VAL, "-" = none),
# alternating twice.  Output gpurun_out/${TAG}_ab_<i>_<rep>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
for rep in 1 2; do
	i=0
	for v in ${AB:--}; do
		i=$((i + 1))
		if [ "$v" = "-" ]; then
			timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-min ${BENCH_ARGS:-} > gpurun_out/${TAG}_ab_${i}_${rep}.log 2>&1
		else
			timeout -k 10 200 env $v python -u bench.py --steps 20 --warmup 3 --no-cpu --no-min ${BENCH_ARGS:-} > gpurun_out/${TAG}_ab_${i}_${rep}.log 2>&1
		fi
		rc=$?; echo "[ab $i $v rep $rep] exit $rc" | tee -a gpurun_out/${TAG}_status.log; [ $rc -ne 0 ] && exit $rc
	done
done
exit 0
