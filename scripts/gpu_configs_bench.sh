#!/bin/bash
# Secondary-config bench lines at the current tree: config 2 (whole job, pairs route) and
# config 5 (direct route on the 4,096-user subset; one rank's 8-GPU column shard of the pairs job).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/configs
mkdir -p $OUT
timeout -k 10 400 python bench.py --config 2 --no-fp32-leg --no-gather-leg --steps 5 --warmup 2 --cpu-users 16 --cpu-seconds 20 > $OUT/config2.json 2> $OUT/config2.err || { tail -20 $OUT/config2.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/config2.json').read().strip().splitlines()[-1]); print('config2', '%.3g pairs/s' % d['value'], '%.1f ms' % d['ms_per_step'], d['self_check']['topk_ok'], d['cpu_baseline']['value'])"
timeout -k 10 500 python bench.py --config 5 --no-fp32-leg > $OUT/config5_direct.json 2> $OUT/config5_direct.err || { tail -20 $OUT/config5_direct.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/config5_direct.json').read().strip().splitlines()[-1]); print('config5 direct', '%.3g pairs/s' % d['value'], '%.1f ms' % d['ms_per_step'], d['roofline']['frac'])"
NAIS_EMULATE_WORLD=8 timeout -k 10 600 python bench.py --config 5 --strategy pairs --no-fp32-leg --no-gather-leg --no-self-check --steps 2 --warmup 1 > $OUT/config5_pairs_shard8.json 2> $OUT/config5_pairs_shard8.err || { tail -20 $OUT/config5_pairs_shard8.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/config5_pairs_shard8.json').read().strip().splitlines()[-1]); print('config5 pairs rank shard of 8', '%.1f ms' % d['ms_per_step'])"
