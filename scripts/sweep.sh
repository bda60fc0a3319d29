#!/bin/bash
# Run bench under several tuning settings (each its own process, own limit).
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
	echo "$i [$envs $extra] exit $rc $(tail -1 gpurun_out/sweep/$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/step %.2f probe %.2f part %.2f decide %.2f surv %d cand %d" % (d["ms_per_step"], d["stages"]["probe_ms"], d["triage"]["part_ms"], d["stages"]["decide_ms"], d["triage"]["survivors"], d["triage"]["candidates"]))' 2>/dev/null)" | tee -a gpurun_out/sweep/summary.txt
	[ $rc -gt 1 ] && exit $rc
done < "${SWEEP_FILE:-scripts/sweep.txt}"
exit 0
