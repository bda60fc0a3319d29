#!/bin/bash
# Round 6 profiles (rocprofv3 kernel trace + stats, then separate FETCH_SIZE /
# WRITE_SIZE / TCC hit passes) of the final code, one workload each:
# the headline (C2 global walk), Minimize, Poll, C5, the C4 rank line and
# the region walk.  Output: gpurun_out/r06_prof*/ (summarize_prof.py turns
# them into profiles/r06_prof*/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() {
	local tag=$1
	shift
	env PROF_TAG=$tag "$@" timeout -k 10 900 scripts/profile.sh
	local rc=$?
	echo "[$tag] exit $rc" | tee -a gpurun_out/r06_prof_status.log
	return $rc
}
for w in ${WHICH:-head min poll c5 c4 rw}; do
	case $w in
	head) run r06_prof BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll" || exit $? ;;
	min) run r06_prof_min PROF_CMD=scripts/min_only.py || exit $? ;;
	poll) run r06_prof_poll PROF_CMD=scripts/line_only.py BENCH_ARGS=poll PMC_KERNELS="k_poll|k_rp_" || exit $? ;;
	c5) run r06_prof_c5 PROF_CMD=scripts/line_only.py BENCH_ARGS=c5 || exit $? ;;
	c4) run r06_prof_c4 PROF_CMD=scripts/line_only.py BENCH_ARGS=c4 PMC_KERNELS="k_agg|k_scat3|k_fast_prep|k_cell_plan|k_stair|k_step|k_rp_" || exit $? ;;
	rw) run r06_prof_rw PROF_CMD=scripts/line_only.py BENCH_ARGS=rw || exit $? ;;
	esac
done
exit 0
