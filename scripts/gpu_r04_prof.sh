#!/bin/bash
# Round-4 profiles of the final tree, one workload per profile (kernel trace +
# separate FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes each, scripts/profile.sh),
# in parts that each fit one gpurun call:
#   PART=1  the headline triage line (C2) and the Minimize line (C3)
#   PART=2  the C4 rank line and the C5 line
#   PART=3  the C2 global-walk line, and SQ counter passes of the K3 chain
#   PART=4  (after the headline moved to SURVEY 8(d)'s global walk) the headline
#           and the C4 rank line on it
#   PART=5  the region-walk C2 line (rounds 1-3's headline), SQ of the new headline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${PROF_ROUND:-r04}
K3="k_agg|k_fin|k_ns_def|k_edge|k_fast_prep|k_cell_plan"
case ${PART:-1} in
1)
	PROF_TAG=${R}_prof BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe" \
		bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_prof_min PROF_CMD=scripts/min_only.py bash scripts/profile.sh || exit $?
	;;
2)
	PROF_TAG=${R}_prof_c4 PROF_CMD=scripts/line_only.py BENCH_ARGS=c4 \
		PMC_KERNELS="k_agg|k_fast_prep|k_cell_plan|k_stair|k_step|k_rp_" bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_prof_c5 PROF_CMD=scripts/line_only.py BENCH_ARGS=c5 PMC_KERNELS="$K3" bash scripts/profile.sh || exit $?
	;;
3)
	PROF_TAG=${R}_prof_gw PROF_CMD=scripts/line_only.py BENCH_ARGS=gw PMC_KERNELS="$K3" bash scripts/profile.sh || exit $?
	PROF_TAG=${R}_sq_k3 PMC_KERNELS="k_agg|k_fin" \
		BENCH_ARGS="--steps 1 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe" \
		bash scripts/pmc_sq.sh || exit $?
	PROF_TAG=${R}_sq_k3b PMC_KERNELS="k_agg|k_fin" \
		BENCH_ARGS="--steps 1 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe" \
		SQ_CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES" \
		bash scripts/pmc_sq.sh || exit $?
	;;
4)
	PROF_TAG=${R}g_prof BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe" \
		bash scripts/profile.sh || exit $?
	PROF_TAG=${R}g_prof_c4 PROF_CMD=scripts/line_only.py BENCH_ARGS="c4 global" \
		PMC_KERNELS="k_agg|k_fast_prep|k_cell_plan|k_stair|k_step|k_rp_" bash scripts/profile.sh || exit $?
	;;
5)
	PROF_TAG=${R}g_prof_rw PROF_CMD=scripts/line_only.py BENCH_ARGS=rw PMC_KERNELS="$K3" bash scripts/profile.sh || exit $?
	PROF_TAG=${R}g_sq_k3 PMC_KERNELS="k_agg|k_fin" \
		BENCH_ARGS="--steps 1 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe" \
		bash scripts/pmc_sq.sh || exit $?
	;;
esac
exit 0
