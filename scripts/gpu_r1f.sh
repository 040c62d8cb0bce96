#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r1f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r1f.log; exit 1; }
tail -1 gpurun_out/bench_r1f.log
scripts/gpu_profile.sh r1f --steps 3 --warmup 1 --no-fp32-leg
