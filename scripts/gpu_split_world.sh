#!/bin/bash
# CU-split sweep of one rank's column shard (bench.py --emulate-world N) on the bounded route:
#   scripts/gpu_split_world.sh TAG "N:cus cus ..." ...   e.g. "8:188 180 172" "4:188 180"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for spec in "$@"; do
  N=${spec%%:*}
  for c in ${spec#*:}; do
    NAIS_PAIR_TABLE_CUS=$c timeout -k 10 300 python bench.py --ab --emulate-world $N --no-fp32-leg --no-gather-leg \
      --no-train-leg --no-cpu-baseline --no-self-check --steps 6 --warmup 2 > $out/n${N}_c$c.json 2> $out/n${N}_c$c.err \
      || { tail -5 $out/n${N}_c$c.err; exit 1; }
    python - $out/n${N}_c$c.json $N $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
g, t = (r, r["other_kernel"]) if "gather" in r["kernel"] or "bound" in r["kernel"] else (r["other_kernel"], r)
print("N", sys.argv[2], "cus", sys.argv[3], "ms %.2f" % d["ms_per_step"], "table %.2f" % t["ms_per_step"],
      "gather %.2f" % g["ms_per_step"], "refine %.2f" % (g.get("refine_ms_per_step") or 0), flush=True)
PY
  done
done
