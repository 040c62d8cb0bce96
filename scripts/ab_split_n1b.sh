set -o pipefail
mkdir -p gpurun_out/r6n1b
for r in 1 2 3; do for c in 188 190; do
  NAIS_PAIR_TABLE_CUS=$c timeout -k 10 300 python bench.py --ab --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline --no-self-check --steps 8 --warmup 2 > gpurun_out/r6n1b/c${c}_r$r.json 2> gpurun_out/r6n1b/c${c}_r$r.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],2))" gpurun_out/r6n1b/c${c}_r$r.json
done; done
