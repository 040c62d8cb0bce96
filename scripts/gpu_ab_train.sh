#!/bin/bash
# A/B of training-kernel builds: bench_train.py (D = H = 128) with the default library and each
# build_ab/<name>.so given as arguments, interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab_train
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset NAIS_HIP_LIB; else export NAIS_HIP_LIB="$GRAFT_REPO_ROOT/build_ab/$v.so"; fi
    timeout -k 10 200 python scripts/bench_train.py --D 128 --H 128 --no-torch > gpurun_out/ab_train/$v.$rep.json 2> gpurun_out/ab_train/$v.$rep.err || { tail -5 gpurun_out/ab_train/$v.$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_train/$v.$rep.json')); print('$v', $rep, 'fused %.4f' % d['fused_ms_per_step'], 'fwd %.4f bwd %.4f' % (d['kernels']['forward_ms'], d['kernels']['backward_ms']))"
  done
done
