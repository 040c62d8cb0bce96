#!/bin/bash
# Training-step A/B at config 3, D = H = 128 (scripts/bench_train.py): the in-tree library ("base")
# and build_ab/<name>.so variants, interleaved: scripts/gpu_diag_bwd.sh TAG base v1 v2 ... base
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/$tag
i=0
for v in "$@"; do
  i=$((i+1))
  if [ $v = base ]; then L=poi_recommendation_models_amd/libnais_hip.so; else L=build_ab/$v.so; fi
  NAIS_HIP_LIB=$L timeout -k 10 200 python scripts/bench_train.py --D 128 --H 128 --no-torch --steps 30 > gpurun_out/$tag/${i}_$v.json 2> gpurun_out/$tag/$v.err || { tail -5 gpurun_out/$tag/$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/$tag/${i}_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['fused_ms_per_step'],4), {k: round(x,4) for k, x in d['kernels'].items()})"
done
