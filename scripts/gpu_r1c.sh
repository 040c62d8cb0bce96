#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_catalog.py --users 128 --rounds 4 > gpurun_out/ab_r1d.json 2> gpurun_out/ab_r1d.err
rc=$?; cat gpurun_out/ab_r1d.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r1d.err; exit $rc; }
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "max \||passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -30
exit $rc
