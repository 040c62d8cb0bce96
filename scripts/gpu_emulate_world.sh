#!/bin/bash
# One rank's column shard of an N-GPU config-4 job timed alone on one GPU (NAIS_EMULATE_WORLD=N):
# the per-rank cost behind bench.py --gpus N, before the all-gather + merge.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/emulate
mkdir -p $OUT
for N in 2 4 8; do
  NAIS_EMULATE_WORLD=$N timeout -k 10 300 python bench.py --no-fp32-leg --no-gather-leg --no-cpu-baseline --no-self-check \
    > $OUT/n$N.json 2> $OUT/n$N.err || { tail -20 $OUT/n$N.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/n$N.json').read().strip().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']
print('N=$N', '%.1f ms/step' % d['ms_per_step'], 'table %.1f ms' % r['ms_per_step'], 'gather %.1f ms' % o['ms_per_step'])"
done
# the real multi-process path, 2 ranks on the box's one GPU over gloo (RCCL needs one GPU per rank)
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-fp32-leg --no-gather-leg --no-cpu-baseline \
  > $OUT/rank2_gloo.json 2> $OUT/rank2_gloo.err || { tail -20 $OUT/rank2_gloo.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/rank2_gloo.json').read().strip().splitlines()[-1])
print('2 ranks (gloo, one GPU):', d['n_gpus'], '%.1f ms/step' % d['ms_per_step'], 'self_check', d['self_check']['topk_ok'])"
