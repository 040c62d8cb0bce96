#!/bin/bash
# Config 5 (200k users x 1M POIs, d = H = 128) as one whole job through the pairs strategy, timed
# on one rank's column shard of an 8-GPU run (NAIS_EMULATE_WORLD=8), for a few table/gather splits.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cfg5p
for tc in ${TABLE_CUS:-128 192}; do
  NAIS_EMULATE_WORLD=8 NAIS_PAIR_TABLE_CUS=$tc timeout -k 10 500 python -u bench.py --config 5 --strategy pairs --steps 1 --warmup 0 --no-fp32-leg \
    > gpurun_out/cfg5p/tc$tc.json 2> gpurun_out/cfg5p/tc$tc.err || { tail -20 gpurun_out/cfg5p/tc$tc.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.4g pairs/s' % d['value'], '%.0f ms/step' % d['ms_per_step'], 'gather %.0f' % (r['avg_launch_ms']*r['launches_per_step']), 'table %.0f' % r['table_kernel']['ms_per_step'], r['table_kernel']['achieved_tflops'])" gpurun_out/cfg5p/tc$tc.json tc$tc
done
