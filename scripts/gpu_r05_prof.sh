#!/bin/bash
# Round-5 profiles of the final tree, one workload per profile (kernel trace +
# separate FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes, scripts/profile.sh):
#   PART=1  the headline triage line (C2, global walk) with K1+K2, the Minimize
#           line (C3), the C5 line (Zipf(1.1) global walks)
#   PART=2  the C4 rank line, the region-walk C2 line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${PROF_ROUND:-r05}
K3="k_agg|k_fin|k_ns_def|k_edge|k_fast_prep|k_cell_plan"
case ${PART:-1} in
1)
	PROF_TAG=${R}_prof BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll" \
		bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_prof_min PROF_CMD=scripts/min_only.py bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_prof_c5 PROF_CMD=scripts/line_only.py BENCH_ARGS=c5 PMC_KERNELS="$K3" bash scripts/profile.sh || exit $?
	;;
2)
	PROF_TAG=${R}_prof_c4 PROF_CMD=scripts/line_only.py BENCH_ARGS="c4 global" \
		PMC_KERNELS="k_agg|k_fast_prep|k_cell_plan|k_stair|k_step|k_rp_" bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_prof_rw PROF_CMD=scripts/line_only.py BENCH_ARGS=rw PMC_KERNELS="$K3" bash scripts/profile.sh || exit $?
	;;
esac
exit 0
