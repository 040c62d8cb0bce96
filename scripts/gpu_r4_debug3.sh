#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r4debug3
mkdir -p $out
timeout -k 10 300 python scripts/debug_prior_odd2.py > $out/debug2.txt 2>&1
echo "rc=$?" >> $out/debug2.txt
tail -20 $out/debug2.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_generic.py tests/test_gpu_train.py -q -x -rf --timeout 300 --timeout-method thread -k "trainer_region or config3_full or training_loop" > $out/pytest_train.log 2>&1
echo "pytest rc=$?" >> $out/pytest_train.log
tail -8 $out/pytest_train.log
