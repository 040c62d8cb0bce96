#!/bin/bash
# Quick GPU iteration: selected tests (args passed to pytest -k) then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SEL="${1:-gpu}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "$SEL" > gpurun_out/pytest_quick.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fp32-leg > gpurun_out/bench_quick.log 2>&1 || { tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log
