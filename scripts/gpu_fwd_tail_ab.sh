#!/bin/bash
# Forward short-slice row tiles (NAIS_GM_FWD_TAIL): training parity tests, then an interleaved A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/fwd_tail
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train_generic.py tests/test_gpu_train.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for r in 1 2; do
  NAIS_GM_FWD_TAIL=0 timeout -k 10 200 python scripts/bench_train.py --D 128 --H 128 > $out/off_$r.json 2>> $out/bench.err || exit 1
  timeout -k 10 200 python scripts/bench_train.py --D 128 --H 128 > $out/on_$r.json 2>> $out/bench.err || exit 1
done
for f in $out/off_1 $out/on_1 $out/off_2 $out/on_2; do
  python -c "import json,sys; d=json.load(open('$f.json')); print('$f', json.dumps(d.get('kernels')), d.get('fused_ms', d.get('fused')))"
done
