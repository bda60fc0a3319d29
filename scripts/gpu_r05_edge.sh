#!/bin/bash
# K2 A/B: edge tests with the default library, then line_only.py edge on both
# walks for the default and each exp/libsyzsig_<v>.so in VARIANTS, REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05e}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
if [ -n "${TESTS:-}" ]; then
	step tests "${TEST_LIMIT:-600}" python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS || exit $?
fi
for rep in $(seq 1 "${REPS:-2}"); do
	for v in default ${VARIANTS:-}; do
		for walk in global region; do
			if [ "$v" = default ]; then
				step "edge_${v}_${walk}_$rep" 200 python -u scripts/line_only.py edge $walk || exit $?
			else
				step "edge_${v}_${walk}_$rep" 200 env SYZSIG_LIB=exp/libsyzsig_$v.so python -u scripts/line_only.py edge $walk || exit $?
			fi
		done
	done
done
exit 0
