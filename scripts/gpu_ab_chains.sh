#!/bin/bash
# A/B of the bounded gather's load chains: default lib, NAIS_PAIR_SHORT_CHAINS=0, and build_ab/<lib>.so
#   scripts/gpu_ab_chains.sh TAG LIBNAME ROUNDS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; lib=$2; rounds=${3:-2}
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $rounds); do
  for v in base nochain $lib; do
    for N in 1 8; do
      envs=""
      [ $v = nochain ] && envs="NAIS_PAIR_SHORT_CHAINS=0"
      [ $v = $lib ] && envs="NAIS_HIP_LIB=build_ab/$lib.so"
      env $envs timeout -k 10 300 python bench.py --emulate-world $N --no-fp32-leg --no-gather-leg --no-train-leg \
        --no-cpu-baseline --no-self-check --steps 6 --warmup 2 > $out/${v}_n${N}_r$r.json 2> $out/${v}_n${N}_r$r.err \
        || { tail -5 $out/${v}_n${N}_r$r.err; exit 1; }
      python - $out/${v}_n${N}_r$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
g, t = (r, r["other_kernel"]) if "bound" in r["kernel"] else (r["other_kernel"], r)
print(sys.argv[1], "ms %.2f" % d["ms_per_step"], "cus", d["config"]["table_cus"], "table %.1f" % t["ms_per_step"],
      "gather %.1f (%.3f/launch)" % (g["ms_per_step"], g["avg_launch_ms"]), "refine %.2f" % (g.get("refine_ms_per_step") or 0), flush=True)
PY
    done
  done
done
