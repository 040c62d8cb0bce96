#!/bin/bash
# Config-4 job A/B over the pairs-route overlap knobs (bench.py --ab), interleaved:
#   scripts/gpu_split_ab.sh TAG "TABLE_CUS:GATHER_FRAC" ...   (empty field = the default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
i=0
for spec in "$@"; do
  i=$((i+1)); cus=${spec%%:*}; frac=${spec##*:}
  env ${cus:+NAIS_PAIR_TABLE_CUS=$cus} ${frac:+NAIS_PAIR_TABLE_GATHER_FRAC=$frac} timeout -k 10 300 python bench.py --ab \
    --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline --no-self-check --steps 3 --warmup 1 \
    > $out/${i}.json 2> $out/${i}.err || { tail -5 $out/${i}.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],1), 'table', round(r['ms_per_step'],1), r['cus'], 'gather', round(r['other_kernel']['ms_per_step'],1))" $out/${i}.json "$spec"
done
