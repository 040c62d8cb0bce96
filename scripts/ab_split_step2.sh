#!/bin/bash
# The 2-CU-step split model's picks against the 4-CU-step ones, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r6s2; mkdir -p $out
run() {   # name, env (or -), bench args...
  local name=$1 envs=$2; shift 2
  [ "$envs" = - ] && envs=""
  env $envs timeout -k 10 300 python bench.py --ab --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline \
    --no-self-check --steps 6 --warmup 2 "$@" > $out/$name.json 2> $out/$name.err || { tail -5 $out/$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],2), d['config']['table_cus'])" $out/$name.json
}
for r in 1 2; do
  run n2_model_r$r - --emulate-world 2
  run n2_188_r$r NAIS_PAIR_TABLE_CUS=188 --emulate-world 2
  run n4_model_r$r - --emulate-world 4
  run n4_184_r$r NAIS_PAIR_TABLE_CUS=184 --emulate-world 4
  run c2_model_r$r - --config 2
  run c2_232_r$r NAIS_PAIR_TABLE_CUS=232 --config 2
done
