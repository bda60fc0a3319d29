#!/bin/bash
# Run bench under several tuning settings (each its own process, own limit);
# one summary line per setting: ms/step and the K3 stage times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}
i=0
while read -r envs; do
	[ -z "$envs" ] && continue
	i=$((i+1))
	extra=""
	case "$envs" in *" -- "*) extra=${envs#* -- }; envs=${envs%% -- *} ;; esac
	env $envs timeout -k 10 300 python3 bench.py $ARGS $extra > gpurun_out/sweep/$i.log 2>&1
	rc=$?
	echo "$i [$envs $extra] exit $rc $(tail -1 gpurun_out/sweep/$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages"]; print("ms/step %.3f part %.3f agg %.3f fin %.3f edge %.2f parts %d ovf %d" % (d["ms_per_step"], s["part_ms"], s["agg_ms"], s["finalize_ms"], s["edge_ms"], d["triage"]["parts"], d["triage"]["overflow_parts"]))' 2>/dev/null)" | tee -a gpurun_out/sweep/summary.txt
	[ $rc -gt 1 ] && exit $rc
done < "${SWEEP_FILE:-scripts/sweep.txt}"
exit 0
