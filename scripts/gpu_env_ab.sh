#!/bin/bash
# A/B of env-var knobs on the default bench. CFGS: ';'-separated lists of VAR=VAL settings
# (space-separated within one config), e.g. CFGS="NAIS_PAIR_BLOCK_COLS=1024;NAIS_PAIR_BLOCK_COLS=2048"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/env_ab
IFS=';' read -r -a LIST <<< "$CFGS"
i=0
for cfg in "${LIST[@]}"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-fp32-leg --no-cpu-baseline \
    > gpurun_out/env_ab/c$i.json 2> gpurun_out/env_ab/c$i.err || { tail -5 gpurun_out/env_ab/c$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '| %.4g pairs/s' % d['value'], '%.1f ms/step' % d['ms_per_step'], 'gather %.1f' % (r['avg_launch_ms']*r['launches_per_step']), 'table %.1f' % r['table_kernel']['ms_per_step'], 'topk %.1f' % r['topk_ms_per_step'])" gpurun_out/env_ab/c$i.json "$cfg"
done
