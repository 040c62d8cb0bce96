#!/bin/bash
# Rehearse the N>1 bench path with 2 ranks on one GPU (gloo collectives on device tensors).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --num-users 8192 > gpurun_out/multirank.log 2>&1
rc=$?; tail -3 gpurun_out/multirank.log; exit $rc
