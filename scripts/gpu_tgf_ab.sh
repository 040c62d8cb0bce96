#!/bin/bash
# Shared gather (PAIR_TABLE_GATHER_FRAC): schedule-invariance tests, then the config-4 bench at
# several fractions of the history entries gathered on the table stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tgf
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "bit_identical or fused_topk" \
  --timeout 120 --timeout-method thread > gpurun_out/tgf/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/tgf/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in "$@"; do
  NAIS_PAIR_TABLE_GATHER_FRAC=$f timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-fp32-leg --no-cpu-baseline \
    > gpurun_out/tgf/f$f.json 2> gpurun_out/tgf/f$f.err || { tail -5 gpurun_out/tgf/f$f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('frac', sys.argv[2], '%.4g pairs/s' % d['value'], '%.1f ms/step' % d['ms_per_step'], 'gather(gs) %.1f ms' % (r['avg_launch_ms']*r['launches_per_step']), 'table %.1f ms' % r['table_kernel']['ms_per_step'], 'achieved %.0f GB/s' % r['achieved'])" gpurun_out/tgf/f$f.json $f
done
