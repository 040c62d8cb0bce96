#!/bin/bash
# |u| epilogue (NAIS_X3B_ABS) check: split-fp16 parity tests on the in-tree library, then the
# config-4 bench A/B against build_ab/abs0.so, overlapped (default split) and serial tables.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_family.py tests/test_gpu_e2e.py -m gpu -x -q -rf \
  --timeout 120 --timeout-method thread > gpurun_out/pt_abs.log 2>&1
rc=$?; tail -3 gpurun_out/pt_abs.log; [ $rc -eq 0 ] || exit $rc
scripts/gpu_lib_ab.sh base abs0 || exit 1
NAIS_PAIR_TABLE_CUS=0 scripts/gpu_lib_ab.sh base abs0
