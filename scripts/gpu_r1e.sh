#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python scripts/ab_catalog.py --users 96 --rounds 3 --only fp16x3 --lib g2=build/ab/lib_g2.so --lib g4=build/ab/lib_g4.so --lib sched=build/ab/lib_sched.so > gpurun_out/ab_r1e.json 2> gpurun_out/ab_r1e.err
rc=$?; grep -E '"lib|median|tflops' gpurun_out/ab_r1e.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r1e.err; exit $rc; }
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -8
exit $rc
