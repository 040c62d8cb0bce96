#!/bin/bash
# Training parity suites without -x (every failure listed), then the D = H = 128 step timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train_check
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train_generic.py tests/test_gpu_train.py -rf > gpurun_out/train_check/pytest.log 2>&1
rc=$?
tail -8 gpurun_out/train_check/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 > gpurun_out/train_check/bench.json 2> gpurun_out/train_check/bench.err || { tail -20 gpurun_out/train_check/bench.err; exit 1; }
cut -c1-900 gpurun_out/train_check/bench.json
