#!/bin/bash
# Standalone pair-table timings of diagnostic builds (build_ab/<name>.so), one process.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/table_diag
LIBS=()
for name in "$@"; do LIBS+=(--lib "$name=$PWD/build_ab/$name.so"); done
timeout -k 10 300 python scripts/bench_table.py --rounds 4 "${LIBS[@]}" > gpurun_out/table_diag/table.log 2>&1 || { tail -20 gpurun_out/table_diag/table.log; exit 1; }
grep -v "^{" gpurun_out/table_diag/table.log | tail -12
