#!/bin/bash
# SQ counter pass (scripts/pmc_sq.sh) of the K3 kernels on the headline
# workload, for each library in LIBS ("default" = the in-tree build, else
# exp/libsyzsig_<name>.so).  Output gpurun_out/$TAG/sq_<lib>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--steps 2 --warmup 1 --no-cpu --no-min --no-c5 --no-c4 --no-c1 --no-gw --no-pipe --no-poll"
for l in ${LIBS:-default}; do
	if [ "$l" = default ]; then
		PROF_TAG=${TAG:-r05}/sq_$l PMC_KERNELS="${PMC_KERNELS:-k_agg}" BENCH_ARGS="$A" bash scripts/pmc_sq.sh || exit $?
	else
		SYZSIG_LIB=exp/libsyzsig_$l.so PROF_TAG=${TAG:-r05}/sq_$l PMC_KERNELS="${PMC_KERNELS:-k_agg}" BENCH_ARGS="$A" \
			bash scripts/pmc_sq.sh || exit $?
	fi
done
exit 0
