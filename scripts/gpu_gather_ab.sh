#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gather
for L in "" build/ab/lib_gu1.so build/ab/lib_gu2.so build/ab/lib_gu8.so; do
  ARG=""; [ -n "$L" ] && ARG="--lib $L"
  timeout -k 10 300 python scripts/bench_gather.py $ARG 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', round(d['achieved_GBps']), round(d['measured_copy_GBps']), round(d['frac_of_measured_copy'],3))" || exit 1
done
