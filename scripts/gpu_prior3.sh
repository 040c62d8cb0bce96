#!/bin/bash
# Prior route: parity tests (incl. the underflow exit) + the config-4 prior job's phase breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prior3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_prior.py tests/test_gpu_distributed.py > gpurun_out/prior3/pytest.log 2>&1 || { tail -30 gpurun_out/prior3/pytest.log; exit 1; }
tail -2 gpurun_out/prior3/pytest.log
timeout -k 10 400 python -u scripts/prior_breakdown.py > gpurun_out/prior3/prior.log 2>&1 || { tail -30 gpurun_out/prior3/prior.log; exit 1; }
head -4 gpurun_out/prior3/prior.log
