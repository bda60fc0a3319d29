#!/bin/bash
# N=2 rehearsal of the sharded bench on ONE GPU (gloo moves the all-to-alls;
# both ranks share cuda:0), then the C4 shard size (125M-element maxSignal,
# = 1B over 8 GPUs) on one GPU.  Each GPU step has its own limit; a failure
# stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
	--master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/rehearse2.log 2>&1
rc=$?; echo "[rehearse2] exit $rc" | tee -a gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --m0 125000000 > gpurun_out/bench_c4shard.log 2>&1
rc=$?; echo "[c4shard] exit $rc" | tee -a gpurun_out/status.log
exit $rc
