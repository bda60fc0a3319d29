#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_f.log 2>&1
rc=$?; echo "[bench] exit $rc" | tee -a gpurun_out/status_f.log; [ $rc -ne 0 ] && exit $rc
PROF_TAG=r02_prof_a BENCH_ARGS="--steps 3 --warmup 1 --no-cpu" bash scripts/profile.sh
