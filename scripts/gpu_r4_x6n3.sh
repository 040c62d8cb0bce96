#!/bin/bash
# x6n with per-step W1 slice loads at NHU > 1 (no spills at D = H = 128) and branch-free NHU > 1
# tails: parity on the scoring suites, standalone table blocks (lib vs the branchy tail and the
# timing ablations), config 5 direct and one rank's 8-GPU pairs shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4x6n3}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numerics.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_e2e.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -6 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
libs=""
for v in tailbr abl1 abl2 abl4 abl8; do libs="$libs --lib $v=build_ab/$v.so"; done
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 $libs > $out/table64.txt 2>&1 || { tail -5 $out/table64.txt; exit 1; }
grep "ms/block" $out/table64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 $libs > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 300 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_direct.json 2> $out/cfg5_direct.err || { tail -5 $out/cfg5_direct.err; exit 1; }
cut -c1-250 $out/cfg5_direct.json
NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_pairs8.json 2> $out/cfg5_pairs8.err || { tail -5 $out/cfg5_pairs8.err; exit 1; }
cut -c1-250 $out/cfg5_pairs8.json
