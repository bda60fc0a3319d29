#!/bin/bash
# A/B of records mode on the C4 rank line (VS: SYZSIG_AGG_DBG values; default
# k_recs_walk (one thread per compacted run head) against k_recs_walk_scan
# (SYZSIG_AGG_DBG=512 = SYZSIG_DEBUG_RECS_SCAN, one thread per sorted
# position), after the records-mode oracle tests; alternating runs, then a
# kernel trace of each (only the stats kept).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/recs_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "records_mode or restore_keys" tests/test_gpu_triage.py > $O/tests.log 2>&1
rc=$?; echo "[tests] exit $rc $(tail -1 $O/tests.log)" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
A="--steps 3 --warmup 1 --no-min --no-c5 --no-c1 --no-cpu"
c4() { tail -1 "$1" | python3 -c "import json,sys; c=json.loads(sys.stdin.read())['lines']['c4_rank']; print('c4_rank ms %.3f source %.3f owner %.3f' % (c['ms'], c['source_ms'], c['owner_ms']))"; }
for r in ${RUNS-1 2}; do
	for v in ${VS:-0 1024}; do
		SYZSIG_AGG_DBG=$v timeout -k 10 300 python -u bench.py $A > $O/run_${v}_$r.log 2>&1
		rc=$?; echo "[dbg=$v run $r] exit $rc $(c4 $O/run_${v}_$r.log)" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
	done
done
export TMPDIR=/tmp
for v in ${VS:-0 1024}; do
	SYZSIG_AGG_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/recs_prof_$v -o run -- python3 bench.py $A > $O/prof_$v.log 2>&1
	rc=$?; echo "[prof dbg=$v] exit $rc" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
	find /tmp/recs_prof_$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
	grep -h "k_recs\|Radix\|radix\|Onesweep" $O/kernel_stats_$v.csv | cut -c1-70 | tee -a $O/status.log
done
exit 0
