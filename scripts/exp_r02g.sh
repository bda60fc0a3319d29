#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dist.py > gpurun_out/exp_g_tests.log 2>&1
rc=$?; echo "[dist test] exit $rc" | tee -a gpurun_out/status_g.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --no-min > gpurun_out/exp_g_bench2.log 2>&1
rc=$?; echo "[bench n2 gloo] exit $rc" | tee -a gpurun_out/status_g.log
exit $rc
