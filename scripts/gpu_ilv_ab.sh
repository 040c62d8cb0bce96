#!/bin/bash
# A/B: wide x3b with the next group's A_j built between this group's MFMA chains (NAIS_X3B_WIDE_ILV).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
NAIS_HIP_LIB="$PWD/build_ab/ilv.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "128" --timeout 120 --timeout-method thread > gpurun_out/pt_ilv.log 2>&1
rc=$?; tail -2 gpurun_out/pt_ilv.log; [ $rc -eq 0 ] || exit $rc
scripts/gpu_cfg5_ab.sh ilv base
