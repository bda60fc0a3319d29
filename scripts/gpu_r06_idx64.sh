#!/bin/bash
# Round 6: k_agg's 64-bit record-index path (SYZSIG_DEBUG_AGG_IDX64) against
# the oracle in both cell layouts, with the other layout cases beside it, and
# the whole triage file.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_idx64}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_triage.py > "$O/tests.log" 2>&1
rc=$?
echo "[tests] exit $rc" | tee -a "$O/status.log"
exit $rc
