#!/bin/bash
# One rocprofv3 PMC pass of SQ counters (wave-cycle breakdown, LDS) over a short
# bench run, for the kernels in PMC_KERNELS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-pmc_sq}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu}
CTRS=${SQ_CTRS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT}
timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "${PMC_KERNELS:-k_agg|k_edge}" -f csv \
	-d "$OUT/pmc" -o run -- python3 bench.py $ARGS > "$OUT/pmc.log" 2>&1
rc=$?
echo "[pmc_sq] exit $rc" | tee -a "$OUT/status.log"
exit $rc
