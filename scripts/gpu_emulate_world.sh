#!/bin/bash
# One rank's column shard of an N-GPU config-4 job timed alone on one GPU (NAIS_EMULATE_WORLD=N):
# the per-rank cost behind bench.py --gpus N, before the all-gather + merge.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/emulate
mkdir -p $OUT
for N in 2 4 8; do
  NAIS_EMULATE_WORLD=$N timeout -k 10 300 python bench.py --no-fp32-leg --no-cpu-baseline --no-self-check \
    > $OUT/n$N.json 2> $OUT/n$N.err || { tail -20 $OUT/n$N.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/n$N.json').read().strip().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']
print('N=$N', '%.1f ms/step' % d['ms_per_step'], 'table %.1f ms' % r['ms_per_step'], 'gather %.1f ms' % o['ms_per_step'])"
done
