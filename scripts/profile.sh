#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run, then separate PMC passes
# (one counter group per run, as MI355X_MICROARCH.md prescribes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p "$OUT"
# the program profiled: bench.py's triage line (PROF_CMD unset), or e.g.
# PROF_CMD=scripts/min_only.py for the Minimize line alone -- one workload per
# profile, so per-kernel averages never mix two workloads' launches
CMD=${PROF_CMD:-bench.py}
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1}
[ "$CMD" != bench.py ] && ARGS=${BENCH_ARGS:-}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $CMD $ARGS > "$OUT/trace.log" 2>&1
echo "[trace] exit $?" | tee -a "$OUT/status.log"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PMC:-}; do
	tag=$(echo "$grp" | tr ' ' '_')
	timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_KERNELS:-k_agg|k_scat3|k_fin|k_ns_def|k_edge|k_min|k_chunk_sizes|k_cell_plan|k_fast_prep|k_count_u8}" -f csv \
		-d "$OUT/pmc_$tag" -o run -- python3 $CMD $ARGS > "$OUT/pmc_$tag.log" 2>&1
	rc=$?
	echo "[pmc $grp] exit $rc" | tee -a "$OUT/status.log"
	[ $rc -ne 0 ] && exit $rc
done
exit 0
