#!/bin/bash
# D = H = 128 under fp16x6: the single-slot item-side kernel (default) vs the per-pair split kernel
# (build_ab/ring0.so): parity tests on the default, standalone 512-column table blocks of both,
# and the config-5 direct bench line of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ring1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py -k "128 or config5 or faithful or shapes" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 --lib ring0=$PWD/build_ab/ring0.so > $OUT/table.log 2>&1 || { tail -20 $OUT/table.log; exit 1; }
grep -v "^{" $OUT/table.log | tail -4
for v in default ring0; do
  if [ $v = default ]; then unset NAIS_HIP_LIB; else export NAIS_HIP_LIB=$PWD/build_ab/$v.so; fi
  timeout -k 10 500 python bench.py --config 5 --no-fp32-leg > $OUT/cfg5_$v.json 2> $OUT/cfg5_$v.err || { tail -20 $OUT/cfg5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg5_$v.json').read().strip().splitlines()[-1]); print('$v config5 direct', '%.3g pairs/s' % d['value'], 'frac %.3f' % d['roofline']['frac'], d['roofline']['kernel'])"
done
