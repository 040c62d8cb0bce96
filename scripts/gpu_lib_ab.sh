#!/bin/bash
# A/B of library builds (build_ab/<name>.so, "base" = the in-tree library) on the default bench.
# Usage: scripts/gpu_lib_ab.sh base name1 name2 ...   (extra bench args via BENCH_ARGS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lib_ab
for name in "$@"; do
  lib="$PWD/build_ab/$name.so"; [ "$name" = base ] && lib="$PWD/poi_recommendation_models_amd/libnais_hip.so"
  NAIS_HIP_LIB="$lib" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-fp32-leg --no-cpu-baseline $BENCH_ARGS \
    > gpurun_out/lib_ab/$name.json 2> gpurun_out/lib_ab/$name.err || { tail -5 gpurun_out/lib_ab/$name.err; exit 1; }
  python - gpurun_out/lib_ab/$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; o = r.get("other_kernel", {})
g, t = (o, r) if o.get("unit") == "GB/s" else (r, o)
print(sys.argv[2], "%.4g pairs/s %.1f ms/step | gather %.1f ms on %s CUs | table %.1f ms on %s CUs | check %s"
      % (d["value"], d["ms_per_step"], g["ms_per_step"], g["cus"], t["ms_per_step"], t["cus"], d.get("self_check")))
PY
done
