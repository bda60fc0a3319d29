#!/bin/bash
# Minimize line only, per library build in LIBS ("cur" = in-tree; NAME =
# exp/libsyzsig_NAME.so), alternating, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-minab}
mkdir -p gpurun_out/$T
for i in 1 2; do for lib in ${LIBS:-cur}; do
	if [ "$lib" = cur ]; then unset SYZSIG_LIB; else export SYZSIG_LIB=exp/libsyzsig_$lib.so; fi
	timeout -k 10 120 python3 scripts/min_only.py > gpurun_out/$T/$lib$i.log 2>&1 || exit 1
	echo "$lib $i $(tail -1 gpurun_out/$T/$lib$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("min %.3f ms" % d["ms"])')" | tee -a gpurun_out/$T/summary.txt
done; done
