#!/bin/bash
# config 5 on the final tree: the direct route (4,096 users x 1M POIs, D = H = 128) and one rank's
# column shard of the 8-GPU pairs job, plus a standalone table block as the box's speed reference
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4cfg5}
mkdir -p $out
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 300 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_direct.json 2> $out/cfg5_direct.err || { tail -5 $out/cfg5_direct.err; exit 1; }
cut -c1-160 $out/cfg5_direct.json
NAIS_EMULATE_WORLD=8 timeout -k 10 400 python bench.py --config 5 --strategy pairs --steps 1 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check > $out/cfg5_pairs8.json 2> $out/cfg5_pairs8.err || { tail -5 $out/cfg5_pairs8.err; exit 1; }
cut -c1-160 $out/cfg5_pairs8.json
