#!/bin/bash
# A/B of the 16x16x32 fp16x6 item-side kernel (x6n) against x3b: parity with x6n on, standalone
# table blocks (interleaved, one process, two builds), then the whole config-4 job both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4x6n}
mkdir -p $out
NAIS_X6N=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest_x6n.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest_x6n.log
tail -4 $out/pytest_x6n.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 5 --lib x6n=build_ab/x6n.so > $out/table_ab.txt 2>&1 || { tail -5 $out/table_ab.txt; exit 1; }
tail -3 $out/table_ab.txt | cut -c1-300
for v in 0 1 0 1; do
  NAIS_X6N=$v timeout -k 10 300 python bench.py --no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2 > $out/bench_x6n$v.json 2> $out/bench_x6n$v.err || { tail -5 $out/bench_x6n$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/bench_x6n$v.json').read().splitlines()[-1]); r=d['roofline']; print('x6n=$v', round(d['ms_per_step'],1), 'ms; table', round(r['ms_per_step'] if 'table' in r['kernel'] else r['other_kernel']['ms_per_step'],1), 'frac_cus', r.get('frac_of_its_cus'))" | tee -a $out/bench_ab.txt
done
