#!/bin/bash
# General training kernels (D = H = 128, the reference's default): parity tests + step timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train128
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train_generic.py tests/test_gpu_train.py > gpurun_out/train128/pytest.log 2>&1 || { tail -30 gpurun_out/train128/pytest.log; exit 1; }
tail -2 gpurun_out/train128/pytest.log
timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 > gpurun_out/train128/bench.json 2> gpurun_out/train128/bench.err || { tail -20 gpurun_out/train128/bench.err; exit 1; }
cut -c1-1500 gpurun_out/train128/bench.json
