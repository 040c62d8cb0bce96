set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prior
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_prior.py > gpurun_out/prior/pytest.log 2>&1 || { tail -30 gpurun_out/prior/pytest.log; exit 1; }
tail -2 gpurun_out/prior/pytest.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/prior/bench.json 2> gpurun_out/prior/bench.err || { tail -20 gpurun_out/prior/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/prior/bench.json').read().strip().splitlines()[-1])
print('value %.4g ms %.1f' % (d['value'], d['ms_per_step']))
for k in ('prior_path','region_distance_path','fp32_path','fp16x3_path'): print(k, json.dumps(d.get(k))[:400])
"
