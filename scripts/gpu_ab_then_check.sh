#!/bin/bash
# Table-kernel A/B (bench_table.py over the given --lib specs), then the full GPU check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_table.py "$@" > gpurun_out/table_ab.log 2>&1 || { tail -20 gpurun_out/table_ab.log; exit 1; }
grep -v "^{" gpurun_out/table_ab.log
bash scripts/gpu_check.sh
