#!/bin/bash
# the N > 1 path on the final tree: bench.py --gpus 2 over gloo (two ranks share the box's GPU),
# then one rank's column shard of N = 2 / 4 / 8 timed alone (NAIS_EMULATE_WORLD)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4multi}
mkdir -p $out
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 > $out/bench_2rank_gloo.json 2> $out/bench_2rank_gloo.err || { tail -5 $out/bench_2rank_gloo.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_2rank_gloo.json').read().splitlines()[-1]); print('gloo2', d['value'], d['ms_per_step'], d['self_check']['topk_ok'], d['per_rank']['ms_per_step_by_rank'])"
for n in 2 4 8; do
  NAIS_EMULATE_WORLD=$n timeout -k 10 300 python bench.py --no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2 > $out/emulate_$n.json 2> $out/emulate_$n.err || { tail -5 $out/emulate_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/emulate_$n.json').read().splitlines()[-1]); r=d['roofline']; o=r['other_kernel']; print('emulate $n', round(d['ms_per_step'],1), 'ms;', r['kernel'][:12], round(r['ms_per_step'],1), o['kernel'][:12], round(o['ms_per_step'],1))" | tee -a $out/summary.txt
done
