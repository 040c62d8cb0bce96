#!/bin/bash
# round-4 final evidence: the whole GPU suite, smoke(), the default bench line; with a second
# argument "profile" also the kernel-trace + FETCH_SIZE / WRITE_SIZE passes of the bench command
# (scripts/gpu_profile.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4final}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --durations=10 --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest_gpu.log
tail -4 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['self_check']['topk_ok'])"
[ "$2" = "profile" ] && scripts/gpu_profile.sh ${1:-r4final} --no-train-leg --steps 5 --warmup 1
true
