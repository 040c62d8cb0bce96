#!/bin/bash
# Round-4 check after the A/B prune: the prior debug (P = 1002 column shards), then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4check2}
mkdir -p $out
timeout -k 10 300 python scripts/debug_prior_odd.py shared_odd > $out/debug_prior_odd.txt 2>&1
echo "debug rc=$?" >> $out/debug_prior_odd.txt
tail -20 $out/debug_prior_odd.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --durations=30 --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest_gpu.log
tail -8 $out/pytest_gpu.log
