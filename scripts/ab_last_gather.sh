set -o pipefail
mkdir -p gpurun_out/r6lg
for r in 1 2; do for v in 0 1; do for N in 1 8; do
  NAIS_PAIR_LAST_GATHER_ALL_CUS=$v timeout -k 10 300 python bench.py --emulate-world $N --no-fp32-leg --no-gather-leg --no-train-leg --no-cpu-baseline --no-self-check --steps 6 --warmup 2 > gpurun_out/r6lg/n${N}_v${v}_r$r.json 2> gpurun_out/r6lg/n${N}_v${v}_r$r.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],2))" gpurun_out/r6lg/n${N}_v${v}_r$r.json
done; done; done
