#!/bin/bash
# Round 6: the flush-list append of the planned-path scatter (Minimize, short
# calls) against the previous build, on the Minimize and region-walk lines;
# the triage/minimize tests; then the N = 2 gloo rehearsal of the sharded bench
# with its parity object.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06i}
mkdir -p "$O"
step() {
	local name=$1 limit=$2
	shift 2
	timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "[$name] exit $rc" | tee -a "$O/status.log"
	return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_minimize_shard.py \
	tests/test_gpu_triage.py tests/test_gpu_configs.py -k "c3 or minimize or ragged or records or triage" || exit $?
for rep in 1 2; do
	for v in base prev; do
		E=""; [ $v != base ] && E="SYZSIG_LIB=exp/libsyzsig_$v.so"
		step "min_${v}_$rep" 200 env $E python -u scripts/min_only.py || exit $?
		step "rw_${v}_$rep" 200 env $E python -u scripts/line_only.py rw || exit $?
	done
done
step rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
	--master-port 29519 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo || exit $?
exit 0
