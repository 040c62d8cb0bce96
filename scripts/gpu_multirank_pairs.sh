#!/bin/bash
# Pairs-path tests, then a 2-rank rehearsal of bench.py (both ranks on the box's one GPU, gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/mr
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 120 --timeout-method thread -k "pairs" > gpurun_out/mr/pytest.log 2>&1 || { tail -30 gpurun_out/mr/pytest.log; exit 1; }
tail -2 gpurun_out/mr/pytest.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/mr/bench_2rank_gloo.json 2> gpurun_out/mr/bench_2rank.err || { tail -20 gpurun_out/mr/bench_2rank.err; exit 1; }
cat gpurun_out/mr/bench_2rank_gloo.json
