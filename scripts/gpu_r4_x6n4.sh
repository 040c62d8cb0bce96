#!/bin/bash
# x6n with compile-time hidden slices per step (no W1 selects, NHU > 1 tails without branches):
# parity on the scoring suites, standalone table blocks, config 5 direct and one rank's 8-GPU
# pairs shard, the config-4 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4x6n4}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_e2e.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -6 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 > $out/table64.txt 2>&1 || { tail -5 $out/table64.txt; exit 1; }
grep "ms/block" $out/table64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 300 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_direct.json 2> $out/cfg5_direct.err || { tail -5 $out/cfg5_direct.err; exit 1; }
cut -c1-250 $out/cfg5_direct.json
NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_pairs8.json 2> $out/cfg5_pairs8.err || { tail -5 $out/cfg5_pairs8.err; exit 1; }
cut -c1-250 $out/cfg5_pairs8.json
timeout -k 10 300 python bench.py --no-fp32-leg --no-cpu-baseline --no-gather-leg --no-train-leg --no-self-check --steps 10 --warmup 2 > $out/bench4.json 2> $out/bench4.err || { tail -5 $out/bench4.err; exit 1; }
cut -c1-250 $out/bench4.json
