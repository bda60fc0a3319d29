#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-trace}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --no-min} > "$OUT/trace.log" 2>&1
rc=$?; echo "[trace] exit $rc" | tee -a "$OUT/status.log"; exit $rc
