#!/bin/bash
# A/B compile variants in one process: scripts/gpu_ab.sh <tag> <ab_catalog args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG="$1"; shift
timeout -k 10 600 python scripts/ab_catalog.py "$@" > gpurun_out/ab_$TAG.json 2> gpurun_out/ab_$TAG.err
rc=$?; cat gpurun_out/ab_$TAG.json; [ $rc -ne 0 ] && tail -20 gpurun_out/ab_$TAG.err
exit $rc
