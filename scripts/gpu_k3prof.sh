#!/bin/bash
# K3 chain at C2: kernel trace (timeline) + SQ counter pass + LDS counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-k3}
A="--steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1"
mkdir -p gpurun_out/$T
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$T/trace -o run -- python3 bench.py $A > gpurun_out/$T/trace.log 2>&1
rc=$?; echo "[trace] exit $rc" | tee -a gpurun_out/$T/status.log; [ $rc -ne 0 ] && exit $rc
PROF_TAG=$T/sq1 PMC_KERNELS="k_agg|k_fin" BENCH_ARGS="$A" bash scripts/pmc_sq.sh || exit $?
PROF_TAG=$T/sq2 PMC_KERNELS="k_agg|k_fin" BENCH_ARGS="$A" SQ_CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES" bash scripts/pmc_sq.sh
