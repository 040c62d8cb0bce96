#!/bin/bash
# Quick GPU A/B: the pairs-route parity tests, then bench.py (no CPU leg, no secondary legs) under
# each env setting given as an argument ("NAME=V NAME2=V2" per argument; "-" = defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pairs" --timeout 120 --timeout-method thread > gpurun_out/pytest_pairs.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pairs.log; [ $rc -eq 0 ] || exit $rc
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=""; [ "$setting" != "-" ] && envs="$setting"
  echo "== $setting"
  timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --no-fp32-leg --steps 5 --warmup 1 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 1; }
  python - gpurun_out/ab_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; o = r.get("other_kernel", {})
g = o if o.get("unit") == "GB/s" else r
t = r if g is o else o
print("value %.3e ms/step %.1f | gather %s %.1f ms %.0f GB/s on %s CUs | table %.1f ms %.1f TF on %s CUs | check %s"
      % (d["value"], d["ms_per_step"], g["kernel"].split()[0], g["ms_per_step"], g["achieved"] or 0, g["cus"],
         t["ms_per_step"], t["achieved"] or 0, t["cus"], d.get("self_check")))
PY
done
