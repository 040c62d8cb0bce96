#!/bin/bash
# the auto table-stream gather share (catalog.auto_table_gather_frac): pairs-route parity, then
# the default bench line with every leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4tgf2}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_prior.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['self_check']['topk_ok'], d['config'].get('table_gather_frac'))"
