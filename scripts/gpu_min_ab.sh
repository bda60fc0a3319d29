#!/bin/bash
# Minimize (C3) per build: the Minimize line alone (scripts/min_only.py), the
# default library and the exp builds in VARIANTS, alternating twice; then the
# Minimize GPU tests on the first variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/minab
mkdir -p $O
for rep in 1 2; do
	for v in base ${VARIANTS}; do
		L=syzkaller_amd/libsyzsig.so; [ $v != base ] && L=exp/libsyzsig_$v.so
		SYZSIG_LIB=$L timeout -k 10 300 python -u scripts/min_only.py > $O/${v}_$rep.log 2>&1
		rc=$?; echo "[$v $rep] exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
	done
done
exit 0
