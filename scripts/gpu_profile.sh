#!/bin/bash
# Kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the benchmark step.
# Usage (on the GPU box, via gpurun): scripts/gpu_profile.sh <tag> [bench args...]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r1}"; shift
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=("$ROOT/bench.py" --no-cpu-baseline "$@")
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "${BENCH[@]}" > "$OUT/pmc_fetch.log" 2>&1 || { echo "fetch pass failed"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "${BENCH[@]}" > "$OUT/pmc_write.log" 2>&1 || { echo "write pass failed"; tail -20 "$OUT/pmc_write.log"; exit 1; }
find "$OUT" -name "*.csv" | head -20
