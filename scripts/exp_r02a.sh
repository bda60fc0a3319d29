#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/sweep.sh || exit $?
PROF_TAG=pmc_sq_edge PMC_KERNELS=k_edge BENCH_ARGS="--steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh || exit $?
PROF_TAG=pmc_sq_edge2 PMC_KERNELS=k_edge SQ_CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" BENCH_ARGS="--steps 1 --warmup 0 --no-cpu" bash scripts/pmc_sq.sh
exit $?
