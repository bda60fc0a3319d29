#!/bin/bash
# N=2 and N=4 rehearsal of the sharded bench (BASELINE config 4: a 1B-element
# maxSignal hash-sharded over the ranks, each rank building only its own shard)
# on ONE GPU: gloo moves the two equal-split all-to-alls, every rank uses
# cuda:0.  Each N has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for N in ${NS:-2 4}; do
	timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
		--master-port $((29517 + N)) bench.py --gpus $N --steps 3 --warmup 2 --dist-backend gloo > gpurun_out/rehearse$N.log 2>&1
	rc=$?; echo "[rehearse$N] exit $rc" | tee -a gpurun_out/rehearse_status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
