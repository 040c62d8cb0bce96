#!/bin/bash
# Per-user prior_kernel underflow exit: its parity tests, then an interleaved A/B (exit off / on).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prior_exit
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prior.py -q -rf --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for r in 1 2; do
  NAIS_PRIOR_EXIT=0 timeout -k 10 180 python scripts/bench_prior_rows.py >> $out/ab.jsonl 2>> $out/ab.err || exit 1
  timeout -k 10 180 python scripts/bench_prior_rows.py >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
cat $out/ab.jsonl
