#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_catalog.py --users 128 --rounds 4 --lib noslp=build/ab/libnais_noslp.so > gpurun_out/ab_r1b.json 2> gpurun_out/ab_r1b.err
rc=$?; cat gpurun_out/ab_r1b.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r1b.err; exit $rc; }
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "max \||passed|failed|Error" gpurun_out/pytest_gpu.log | tail -30
exit $rc
