#!/bin/bash
# Table launches on one vs two CU-masked streams (catalog.PAIR_TABLE_STREAMS), same box,
# interleaved runs of the headline job only (no legs, no CPU baseline, no self-check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tstreams
B="--no-fp32-leg --no-cpu-baseline --no-gather-leg --no-self-check --steps 6 --warmup 2"
for r in 1 2; do
  for n in 2 1; do
    NAIS_PAIR_TABLE_STREAMS=$n timeout -k 10 300 python bench.py $B > gpurun_out/tstreams/s${n}_r${r}.json 2> gpurun_out/tstreams/s${n}_r${r}.err || { tail -20 gpurun_out/tstreams/s${n}_r${r}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/tstreams/s${n}_r${r}.json')); r=d['roofline']; print('streams=$n run=$r', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], 'table', round(r['ms_per_step'] if r['kernel'].startswith('catalog') else r['other_kernel']['ms_per_step'],1), 'gather', round(r['other_kernel']['ms_per_step'] if r['kernel'].startswith('catalog') else r['ms_per_step'],1))"
  done
done
