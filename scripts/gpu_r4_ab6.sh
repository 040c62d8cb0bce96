#!/bin/bash
# same-process A/B of the x6n table block: lib (block-major) vs sched_group_barrier issue patterns
# (1 or 2 VALU per MFMA slot) vs the next unit's build at the step's middle group
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4ab6}
mkdir -p $out
libs=""
for v in sgb1 sgb2 bpos2; do libs="$libs --lib $v=build_ab/$v.so"; done
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 5 $libs > $out/table64.txt 2>&1 || { tail -5 $out/table64.txt; exit 1; }
grep "ms/block" $out/table64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 5 $libs > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['self_check']['topk_ok'], d['self_check']['max_abs_score_diff'])"
