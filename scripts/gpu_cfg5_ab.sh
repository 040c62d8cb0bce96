#!/bin/bash
# Config 5 A/B of library builds: direct (4096-user subset) and the pairs whole job (one rank of 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cfg5ab
for name in "$@"; do
  lib="$PWD/build_ab/$name.so"; [ "$name" = base ] && lib="$PWD/poi_recommendation_models_amd/libnais_hip.so"
  NAIS_HIP_LIB="$lib" timeout -k 10 400 python -u bench.py --config 5 --no-fp32-leg > gpurun_out/cfg5ab/d_$name.json 2> gpurun_out/cfg5ab/d_$name.err || { tail -5 gpurun_out/cfg5ab/d_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'direct %.4g pairs/s' % d['value'], 'frac %.3f' % r['frac'], r.get('achieved'))" gpurun_out/cfg5ab/d_$name.json $name
  NAIS_HIP_LIB="$lib" NAIS_EMULATE_WORLD=8 timeout -k 10 400 python -u bench.py --config 5 --strategy pairs --steps 1 --warmup 0 --no-fp32-leg > gpurun_out/cfg5ab/p_$name.json 2> gpurun_out/cfg5ab/p_$name.err || { tail -5 gpurun_out/cfg5ab/p_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'pairs %.4g pairs/s' % d['value'], '%.0f ms/step' % d['ms_per_step'], 'gather %.0f' % (r['avg_launch_ms']*r['launches_per_step']), 'table %.0f' % r['table_kernel']['ms_per_step'], r['table_kernel']['achieved_tflops'], r['table_kernel']['cus'])" gpurun_out/cfg5ab/p_$name.json $name
done
