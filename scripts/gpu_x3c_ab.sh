#!/bin/bash
# x3c pair-table kernel: standalone A/B against x3b (build_ab/x3b.so, -DNAIS_X3C=0), then the
# fp16x6 pair-table / pairs-route parity tests at the x3c default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/x3c
timeout -k 10 300 python -u scripts/bench_table.py --lib x3b=build_ab/x3b.so --blocks 8 --rounds 3 \
  > gpurun_out/x3c/bench_table.txt 2>&1 || { tail -20 gpurun_out/x3c/bench_table.txt; exit 1; }
cat gpurun_out/x3c/bench_table.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -m gpu -x -q -k "pair or fp16x6 or config" --timeout 300 --timeout-method thread \
  > gpurun_out/x3c/pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/x3c/pytest.txt; exit $rc
