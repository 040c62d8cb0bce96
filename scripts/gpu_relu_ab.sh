#!/bin/bash
# v_maximum3_f32 ReLU (default) vs the v_cmp + v_cndmask ReLU (build_ab/x3b.so = the previous
# default build): standalone table A/B, then the NaN / fp16x6 / pairs parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/relu
timeout -k 10 300 python -u scripts/bench_table.py --lib old=build_ab/x3b.so --blocks 8 --rounds 4 \
  > gpurun_out/relu/bench_table.txt 2>&1 || { tail -20 gpurun_out/relu/bench_table.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/relu/bench_table.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/relu/pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/relu/pytest.txt; exit $rc
