#!/bin/bash
# Pair-table kernel A/B of library builds: standalone block timings (bench_table.py, one process,
# interleaved rounds), then the whole config-4 job per build (gpu_lib_ab.sh).
# Usage: scripts/gpu_table_ab.sh name1 name2 ...   (build_ab/<name>.so from scripts/build_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lib_ab
LIBS=()
for name in "$@"; do LIBS+=(--lib "$name=$PWD/build_ab/$name.so"); done
timeout -k 10 300 python scripts/bench_table.py "${LIBS[@]}" > gpurun_out/lib_ab/table.log 2>&1 || { tail -20 gpurun_out/lib_ab/table.log; exit 1; }
grep -v "^{" gpurun_out/lib_ab/table.log | tail -12
bash scripts/gpu_lib_ab.sh base "$@"
