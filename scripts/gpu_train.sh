#!/bin/bash
# Training step on the GPU box: parity tests, config-3 bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out/train
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_train.py -x -q > gpurun_out/train/pytest.log 2>&1 || { tail -40 gpurun_out/train/pytest.log; exit 1; }
tail -3 gpurun_out/train/pytest.log
timeout -k 10 300 python scripts/bench_train.py --cpu > gpurun_out/train/bench.json 2> gpurun_out/train/bench.err && cat gpurun_out/train/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/train/prof -o run -- python3 scripts/bench_train.py --no-torch --steps 20 > gpurun_out/train/prof.log 2>&1 &&
find gpurun_out/train/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -15'
