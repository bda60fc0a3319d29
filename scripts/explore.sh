#!/bin/bash
# Exploration session: scatter write-pattern microbenchmark, partition-count
# sweep, SQ counters of the K3 partitioning kernels.  Each GPU step has its own
# limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o build/mb_scatter scripts/mb_scatter.hip || exit 1
timeout -k 10 120 ./build/mb_scatter > gpurun_out/mb_scatter.log 2>&1
rc=$?; echo "[mb_scatter] exit $rc" | tee -a gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
if [ -n "${SWEEP_FILE:-}" ]; then bash scripts/sweep.sh || exit $?; fi
PROF_TAG=pmc_sq_scat PMC_KERNELS="k_agg_scatter|k_agg_count|k_agg<" BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-min" bash scripts/pmc_sq.sh
