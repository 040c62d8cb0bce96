#!/bin/bash
# A/B of the pairs strategy's table/gather overlap (CU-masked streams): bench value per setting.
set -o pipefail
mkdir -p gpurun_out/overlap
# CFGS: ';'-separated "table_cus layout block_cols" triples
IFS=';' read -r -a LIST <<< "${CFGS:-0 contiguous 8192;128 contiguous 8192;128 contiguous 4096;112 contiguous 8192}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  NAIS_PAIR_TABLE_CUS=$1 NAIS_PAIR_CU_LAYOUT=$2 NAIS_PAIR_BLOCK_COLS=$3 timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
    --no-fp32-leg --no-cpu-baseline > gpurun_out/overlap/b_$1_$2_$3.json 2> gpurun_out/overlap/b_$1_$2_$3.err \
    || { tail -5 gpurun_out/overlap/b_$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], '%.3g pairs/s' % d['value'], '%.0f ms/step' % d['ms_per_step'], 'gather %.0f ms' % (r['avg_launch_ms']*r['launches_per_step']), 'table %.0f ms' % r['table_kernel']['ms_per_step'])" gpurun_out/overlap/b_$1_$2_$3.json
done
