#!/bin/bash
# Round-4 check: GPU suite, smoke(), the default bench line (with the prior plan and the training
# leg), then a 2-rank gloo rehearsal of the N > 1 line (per-rank phase times) on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4check}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --durations=30 --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest_gpu.log
tail -5 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $out/bench_2rank_gloo.json 2> $out/bench_2rank_gloo.err || { tail -20 $out/bench_2rank_gloo.err; exit 1; }
cut -c1-300 $out/bench_2rank_gloo.json
