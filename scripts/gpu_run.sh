#!/bin/bash
# The one GPU-box runner (via gpurun): scripts/gpu_run.sh <mode> <tag> [extra args]
#   check     the GPU suite, smoke(), the default bench line
#   tests     the GPU suite only (extra args replace the selection, e.g. test files, -k EXPR)
#   bench     the default bench line (extra args go to bench.py)
#   profile   rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench command
#   pmc       SQ counter passes of the standalone pair-table block (scripts/bench_table.py; extra
#             args go to bench_table.py, e.g. --dim 128 --hidden 128)
#   configs   config 2 whole job, config 5 direct and one rank's 8-GPU config-5 pairs shard
#   ab        one standalone pair-table A/B (scripts/bench_table.py; extra args go to it, e.g.
#             --variant region_distance --lib pk0=build_ab/pk0.so); output appended to ab.txt
#   abjob     the config-4 pairs job of one variant (scripts/bench_variant.py, all columns on this
#             GPU) per library, interleaved: scripts/gpu_run.sh abjob TAG VARIANT base NAME ...
#             (base = the in-tree library, NAME = build_ab/NAME.so)
#   emulate   one rank's column shard of an N = 2 / 4 / 8 config-4 job, then the real 2-rank
#             process group over gloo on the one GPU
# Every GPU step runs under its own timeout and the steps are chained: the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mode="$1"; tag="${2:-run}"; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.4g pairs/s' % d['value'], '%.1f ms/step' % d['ms_per_step'], 'self_check', (d.get('self_check') or {}).get('topk_ok'))" "$1"; }
tests() {
  local sel=("$@")
  [ ${#sel[@]} -eq 0 ] && sel=(tests)
  timeout -k 10 1100 python -u -m pytest "${sel[@]}" -m gpu --maxfail=10 -q -rf --durations=15 --timeout 300 \
    --timeout-method thread > $out/pytest_gpu.log 2>&1
  local rc=$?
  echo "pytest rc=$rc" >> $out/pytest_gpu.log
  tail -6 $out/pytest_gpu.log
  return $rc
}
case "$mode" in
  check)
    tests || exit $?
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
    timeout -k 10 600 python bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
    line $out/bench.json ;;
  tests)
    tests "$@" ;;
  bench)
    timeout -k 10 900 python bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
    line $out/bench.json ;;
  profile)
    scripts/gpu_profile.sh "$tag" --no-train-leg --steps 5 --warmup 1 "$@" ;;
  pmc)
    timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 "$@" > $out/table.txt 2>&1 || { tail -5 $out/table.txt; exit 1; }
    grep "ms/block" $out/table.txt
    timeout -k 10 600 scripts/gpu_pmc_cmd.sh ${tag}_pmc x6n_kernel scripts/bench_table.py --blocks 8 --rounds 1 "$@" > $out/pmc.txt 2>&1 || { tail -5 $out/pmc.txt; exit 1; }
    tail -20 $out/pmc.txt ;;
  configs)
    timeout -k 10 400 python bench.py --config 2 --no-fp32-leg --no-gather-leg --no-train-leg --steps 5 --warmup 2 --cpu-users 16 --cpu-seconds 20 > $out/config2.json 2> $out/config2.err || { tail -20 $out/config2.err; exit 1; }
    line $out/config2.json
    timeout -k 10 500 python bench.py --config 5 --no-fp32-leg --no-gather-leg --no-train-leg > $out/config5_direct.json 2> $out/config5_direct.err || { tail -20 $out/config5_direct.err; exit 1; }
    line $out/config5_direct.json
    timeout -k 10 600 python bench.py --config 5 --strategy pairs --emulate-world 8 --no-fp32-leg --no-gather-leg --no-train-leg --no-self-check --steps 1 --warmup 1 > $out/config5_pairs_shard8.json 2> $out/config5_pairs_shard8.err || { tail -20 $out/config5_pairs_shard8.err; exit 1; }
    line $out/config5_pairs_shard8.json ;;
  ab)
    timeout -k 10 400 python scripts/bench_table.py "$@" >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
    grep "ms/block" $out/ab.txt | tail -8 ;;
  abjob)
    variant=$1; shift; i=0
    for v in "$@"; do
      i=$((i+1))
      if [ $v = base ]; then L=poi_recommendation_models_amd/libnais_hip.so; else L=build_ab/$v.so; fi
      NAIS_HIP_LIB=$L timeout -k 10 300 python scripts/bench_variant.py --variant $variant --num-users 50000 --num-pois 100000 \
        --dim 64 --hidden 64 --emulate-world 1 --skip direct --steps 2 > $out/${i}_$v.json 2> $out/${i}_$v.err || { tail -5 $out/${i}_$v.err; exit 1; }
      echo $v $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['shard']['seconds_per_rank_step'])" $out/${i}_$v.json)
    done ;;
  emulate)
    for N in 2 4 8; do
      timeout -k 10 300 python bench.py --emulate-world $N --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline --no-self-check \
        > $out/n$N.json 2> $out/n$N.err || { tail -20 $out/n$N.err; exit 1; }
      line $out/n$N.json
    done
    timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline \
      > $out/rank2_gloo.json 2> $out/rank2_gloo.err || { tail -20 $out/rank2_gloo.err; exit 1; }
    line $out/rank2_gloo.json ;;
  *)
    echo "unknown mode $mode"; exit 2 ;;
esac
