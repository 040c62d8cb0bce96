#!/bin/bash
# config-4 job vs the share of history entries gathered on the table stream after each block's
# table (NAIS_PAIR_TABLE_GATHER_FRAC): the gather stream is the bound since the x6n tables
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4tgf}
mkdir -p $out
for f in 0 0.03 0.05 0.08 0; do
  NAIS_PAIR_TABLE_GATHER_FRAC=$f timeout -k 10 300 python bench.py --no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2 > $out/b_$f.json 2> $out/b_$f.err || { tail -5 $out/b_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/b_$f.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; g=r if 'gather' in r['kernel'] else o; t=o if g is r else r; print('frac $f', round(d['ms_per_step'],1), 'ms; gather', round(g['ms_per_step'],1), 'table', round(t['ms_per_step'],1))" | tee -a $out/summary.txt
done
