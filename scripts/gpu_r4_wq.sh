#!/bin/bash
# work-queue launches of the x6n table kernel and the fused gather (catalog.PAIR_WORK_QUEUE) with
# 8-CU split steps: pairs-route parity, then config 4 and the config-5 shard against the classic
# grids (NAIS_PAIR_WORK_QUEUE=0, engine-sized steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4wq}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_prior.py tests/test_gpu_numerics.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
B="--no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2"
for v in 1 0 1 0; do
  NAIS_PAIR_WORK_QUEUE=$v timeout -k 10 300 python bench.py $B > $out/c4_wq$v.json 2> $out/c4_wq$v.err || { tail -5 $out/c4_wq$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/c4_wq$v.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c4 wq=$v', round(d['ms_per_step'],1), r['kernel'][:10], round(r['ms_per_step'],1), r.get('cus'), o['kernel'][:10], round(o['ms_per_step'],1), o.get('cus'))" | tee -a $out/summary.txt
done
for v in 1 0; do
  NAIS_PAIR_WORK_QUEUE=$v NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/c5_wq$v.json 2> $out/c5_wq$v.err || { tail -5 $out/c5_wq$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/c5_wq$v.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c5 wq=$v', round(d['ms_per_step'],1), round(r['ms_per_step'],1), r.get('cus'), round(o['ms_per_step'],1), o.get('cus'))" | tee -a $out/summary.txt
done
