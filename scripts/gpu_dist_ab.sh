#!/bin/bash
# Distance variants on the item-side kernel (in-tree) vs the per-pair split kernel
# (build_ab/nodist.so: python scripts/build_ab.py nodist=-DNAIS_X3B_DIST=0): distance parity tests,
# then the bench legs of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/dist
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "distance" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in base nodist; do
  lib=$PWD/poi_recommendation_models_amd/libnais_hip.so; [ $L = nodist ] && lib=$PWD/build_ab/nodist.so
  NAIS_HIP_LIB=$lib timeout -k 10 500 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench_$L.json 2> $OUT/bench_$L.err \
    || { tail -20 $OUT/bench_$L.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/bench_$L.json').read().strip().splitlines()[-1])
print('$L', '%.4g' % d['value'], '%.1f' % d['ms_per_step'], 'region_distance %.1f ms' % d['region_distance_path']['ms_per_step'], 'prior %.1f' % d['prior_path']['ms_per_step'])"
done
