#!/bin/bash
# Short-slice split of the general forward + backward (NAIS_GM_TAIL=4, default) vs one launch (build_ab/notail.so), same
# box: D = H = 128 step timing of both, then the training parity tests at the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train_tail
timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 --no-torch > gpurun_out/train_tail/bench_tail.json 2> gpurun_out/train_tail/bench_tail.err || { tail -20 gpurun_out/train_tail/bench_tail.err; exit 1; }
NAIS_HIP_LIB=build_ab/notail.so timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 --no-torch > gpurun_out/train_tail/bench_notail.json 2> gpurun_out/train_tail/bench_notail.err || { tail -20 gpurun_out/train_tail/bench_notail.err; exit 1; }
timeout -k 10 300 python scripts/bench_train.py --D 128 --H 128 --no-torch > gpurun_out/train_tail/bench_tail2.json 2>> gpurun_out/train_tail/bench_tail.err || exit 1
for f in bench_tail bench_notail bench_tail2; do python3 -c "import json,sys; d=json.load(open('gpurun_out/train_tail/$f.json')); print('$f', {k: round(d[k],4) for k in ('hip_ms_per_step','fused_ms_per_step','fused_with_batch_ms_per_step')}, {k: round(v,4) for k,v in d['kernels'].items()})"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train_generic.py tests/test_gpu_train.py > gpurun_out/train_tail/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/train_tail/pytest.log; exit $rc
