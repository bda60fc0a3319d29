#!/bin/bash
# A/B timing of library builds (LIBS: "cur" = the in-tree library, NAME =
# exp/libsyzsig_NAME.so), alternating, two runs each: ms/step, the scatter
# stage and the Minimize line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/minab
for i in 1 2; do for lib in ${LIBS:-base cur}; do
	if [ "$lib" = cur ]; then unset SYZSIG_LIB; else export SYZSIG_LIB=exp/libsyzsig_$lib.so; fi
	timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/minab/$lib$i.log 2>&1 || exit 1
	echo "$lib $i $(tail -1 gpurun_out/minab/$lib$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/step %.3f part %.3f agg %.3f min %.3f" % (d["ms_per_step"], d["stages"]["part_ms"], d["stages"]["agg_ms"], d["lines"]["minimize"]["ms"]))')" | tee -a gpurun_out/minab/summary.txt
done; done
