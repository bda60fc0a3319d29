#!/bin/bash
# Round 5 loop: GPU tests in TESTS, then an A/B of the default library against
# the experiment builds in VARIANTS (exp/libsyzsig_<name>.so), alternating
# REPS times, bench.py with BENCH_ARGS.  Every step has its own time limit;
# the first failure ends the run.  Output under gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05}
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
		if [ "$v" = default ]; then
			step "bench_${v}_$rep" 300 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu} || exit $?
		else
			step "bench_${v}_$rep" 300 env SYZSIG_LIB=exp/libsyzsig_$v.so python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu} || exit $?
		fi
	done
done
exit 0
