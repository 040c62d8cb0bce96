#!/bin/bash
# work queues (4 user slots per grab in the gather) for splits off the engine steps: pairs parity
# incl. the forced off-step splits, then config 4 at 160 (classic) vs 152 (work queues) and the
# config-5 shard at the auto split (232, work queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4wq2}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
B="--no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2"
for c in 160 152 160 152; do
  NAIS_PAIR_TABLE_CUS=$c timeout -k 10 300 python bench.py $B > $out/c4_$c.json 2> $out/c4_$c.err || { tail -5 $out/c4_$c.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/c4_$c.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c4 cus=$c', round(d['ms_per_step'],1), r['kernel'][:10], round(r['ms_per_step'],1), o['kernel'][:10], round(o['ms_per_step'],1))" | tee -a $out/summary.txt
done
NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/c5.json 2> $out/c5.err || { tail -5 $out/c5.err; exit 1; }
python -c "import json; d=json.loads(open('$out/c5.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c5 auto', round(d['ms_per_step'],1), round(r['ms_per_step'],1), r.get('cus'), round(o['ms_per_step'],1), o.get('cus'))" | tee -a $out/summary.txt
