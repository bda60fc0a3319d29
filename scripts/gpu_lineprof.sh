#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE/L2 PMC passes of one extra bench line
# (scripts/line_only.py LINE) -> gpurun_out/<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for LINE in ${LINES:-c5 c4}; do
	PROF_TAG=${TAG:-r03}_prof_$LINE PROF_CMD=scripts/line_only.py BENCH_ARGS=$LINE \
		PMC_KERNELS="k_agg|k_fin|k_fast|k_cell|k_chunk|k_stair|k_recs|k_probe|k_decide|k_rehash" bash scripts/profile.sh || exit $?
done
