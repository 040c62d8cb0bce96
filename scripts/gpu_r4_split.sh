#!/bin/bash
# config-4 job at table / gather splits around the cost model's 152 / 104 (work queues off the
# 32-CU steps), interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4split}
mkdir -p $out
B="--no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2"
for c in 144 152 160 144 152 160; do
  NAIS_PAIR_TABLE_CUS=$c timeout -k 10 300 python bench.py $B > $out/c4_$c.json 2> $out/c4_$c.err || { tail -5 $out/c4_$c.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/c4_$c.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('c4 cus=$c', round(d['ms_per_step'],1), r['kernel'][:10], round(r['ms_per_step'],1), o['kernel'][:10], round(o['ms_per_step'],1))" | tee -a $out/summary.txt
done
