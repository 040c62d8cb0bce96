#!/bin/bash
# Round-3 probes: heterogeneous fp16x6 error printout, the sharded-prior / merge tests, the prior
# job's phase breakdown, and the general training kernels at D = H = 128 (tests + timing).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3probe
true
true
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_distributed.py tests/test_gpu_prior.py tests/test_gpu_train_generic.py tests/test_gpu_train.py > gpurun_out/r3probe/dist.log 2>&1 || { tail -30 gpurun_out/r3probe/dist.log; exit 1; }
tail -2 gpurun_out/r3probe/dist.log
timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 > gpurun_out/r3probe/train128.json 2> gpurun_out/r3probe/train128.err || { tail -20 gpurun_out/r3probe/train128.err; exit 1; }
cut -c1-1500 gpurun_out/r3probe/train128.json
timeout -k 10 400 python -u scripts/prior_breakdown.py > gpurun_out/r3probe/prior.log 2>&1 || { tail -30 gpurun_out/r3probe/prior.log; exit 1; }
head -4 gpurun_out/r3probe/prior.log
