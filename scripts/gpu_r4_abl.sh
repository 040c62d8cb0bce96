#!/bin/bash
# timing ablations of the x6n table kernel (build_ab/abl*.so, NAIS_X6N_ABL bits: 1 no epilogue,
# 2 no build, 4 no A-fragment LDS reads, 8 no tail, 16 no group barriers): standalone table blocks
# at D = H = 64 and D = H = 128, interleaved rounds in one process
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4abl}
mkdir -p $out
libs=""
for v in 1 2 4 8 16 27; do libs="$libs --lib abl$v=build_ab/abl$v.so"; done
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 $libs > $out/abl64.txt 2>&1 || { tail -5 $out/abl64.txt; exit 1; }
grep "ms/block" $out/abl64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 $libs > $out/abl128.txt 2>&1 || { tail -5 $out/abl128.txt; exit 1; }
grep "ms/block" $out/abl128.txt
