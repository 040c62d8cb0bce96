#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --config 5 > gpurun_out/bench_cfg5.log 2>&1 || { tail -20 gpurun_out/bench_cfg5.log; exit 1; }
tail -1 gpurun_out/bench_cfg5.log
