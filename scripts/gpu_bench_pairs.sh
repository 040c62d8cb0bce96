#!/bin/bash
# Pairs strategy on the GPU box: parity subset, the default bench line, a 2-rank rehearsal (gloo,
# both ranks on the one GPU) of the column-sharded path.
set -o pipefail
mkdir -p gpurun_out/pairs
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "pairs or column_shards" > gpurun_out/pairs/pytest.log 2>&1 || { tail -30 gpurun_out/pairs/pytest.log; exit 1; }
tail -2 gpurun_out/pairs/pytest.log
timeout -k 10 600 python bench.py > gpurun_out/pairs/bench_n1.json 2> gpurun_out/pairs/bench_n1.err || { tail -20 gpurun_out/pairs/bench_n1.err; exit 1; }
cat gpurun_out/pairs/bench_n1.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/pairs/bench_2rank_gloo.json 2> gpurun_out/pairs/bench_2rank.err || { tail -20 gpurun_out/pairs/bench_2rank.err; exit 1; }
cat gpurun_out/pairs/bench_2rank_gloo.json
