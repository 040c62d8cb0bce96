#!/bin/bash
# x6n with 64-hidden units at D = 128 (MB = 4): parity on the scoring suites, then same-process
# A/B of the table block against 32-hidden units (mb2), config 5 direct and the 8-GPU pairs
# shard
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4ab5}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_e2e.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
libs=""
for v in mb2; do libs="$libs --lib $v=build_ab/$v.so"; done
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 5 $libs > $out/table64.txt 2>&1 || { tail -5 $out/table64.txt; exit 1; }
grep "ms/block" $out/table64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 5 $libs > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 300 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_direct.json 2> $out/cfg5_direct.err || { tail -5 $out/cfg5_direct.err; exit 1; }
cut -c1-200 $out/cfg5_direct.json
NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_pairs8.json 2> $out/cfg5_pairs8.err || { tail -5 $out/cfg5_pairs8.err; exit 1; }
cut -c1-200 $out/cfg5_pairs8.json
