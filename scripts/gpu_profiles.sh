#!/bin/bash
# Checkpoint B: rocprofv3 summaries of the triage line and of the Minimize line
# (kernel trace + separate FETCH/WRITE/L2 PMC passes each), and one SQ pass of
# k_edge_dedup.  PROF_ROUND names the profiles (e.g. r02b).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${PROF_ROUND:-rxx}
PROF_TAG=${R}_prof bash scripts/profile.sh || exit $?
PROF_TAG=${R}_prof_min PROF_CMD=scripts/min_only.py bash scripts/profile.sh || exit $?
PROF_TAG=${R}_pmc_edge PMC_KERNELS=k_edge_dedup BENCH_ARGS="--steps 1 --warmup 0 --no-cpu --no-min" bash scripts/pmc_sq.sh || exit $?
PROF_TAG=${R}_pmc_edge2 PMC_KERNELS=k_edge_dedup BENCH_ARGS="--steps 1 --warmup 0 --no-cpu --no-min" \
	SQ_CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES" \
	bash scripts/pmc_sq.sh
