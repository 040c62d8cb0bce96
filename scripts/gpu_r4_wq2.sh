#!/bin/bash
# work queues with 4 user slots per grab in the gather: pairs parity (short), config 4 at the
# classic 160 / 96 split with and without work queues, and at 152 / 104 with them
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4wq2}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -rf -k "pairs or config4" --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
B="--no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2"
for cfg in "1 160" "0 160" "1 152" "1 160" "0 160" "1 152"; do
  set -- $cfg
  NAIS_PAIR_WORK_QUEUE=$1 NAIS_PAIR_TABLE_CUS=$2 timeout -k 10 300 python bench.py $B > $out/c4_$1_$2.json 2> $out/c4_$1_$2.err || { tail -5 $out/c4_$1_$2.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/c4_$1_$2.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c4 wq=$1 cus=$2', round(d['ms_per_step'],1), r['kernel'][:10], round(r['ms_per_step'],1), o['kernel'][:10], round(o['ms_per_step'],1))" | tee -a $out/summary.txt
done
