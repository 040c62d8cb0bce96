#!/bin/bash
# D = H = 128 under fp16x6 on the unit-sliced 16x16x32 kernel (x6n): parity on the D = 128 cases,
# then config 5 A/B (x6n vs the per-pair split kernel it replaces, NAIS_X6N=0): the direct route on
# the 4096-user subset and one rank's column shard of the 8-GPU pairs job.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4d128}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -6 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  NAIS_X6N=$v timeout -k 10 300 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_direct_x6n$v.json 2> $out/cfg5_direct_x6n$v.err || { tail -5 $out/cfg5_direct_x6n$v.err; exit 1; }
  cut -c1-300 $out/cfg5_direct_x6n$v.json
done
for v in 1 0; do
  NAIS_X6N=$v NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_pairs8_x6n$v.json 2> $out/cfg5_pairs8_x6n$v.err || { tail -5 $out/cfg5_pairs8_x6n$v.err; exit 1; }
  cut -c1-300 $out/cfg5_pairs8_x6n$v.json
done
