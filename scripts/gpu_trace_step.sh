#!/bin/bash
# Kernel trace of a few bench steps (env knobs pass through), for the per-step timeline.
# Usage: scripts/gpu_trace_step.sh <tag> [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/trace_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-fp32-leg "$@" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '"metric"' "$OUT/bench.log" | cut -c1-200
