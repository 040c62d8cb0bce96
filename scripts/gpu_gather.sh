#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT" || exit 1
mkdir -p gpurun_out/gather
timeout -k 10 300 python scripts/bench_gather.py --reuse --rows 1000000 > gpurun_out/gather/reuse.json 2>&1 || { cat gpurun_out/gather/reuse.json; exit 1; }
cat gpurun_out/gather/reuse.json
timeout -k 10 300 python scripts/bench_gather.py > gpurun_out/gather/random.json 2>&1 || { cat gpurun_out/gather/random.json; exit 1; }
cat gpurun_out/gather/random.json
timeout -k 10 300 python scripts/bench_gather.py --sorted > gpurun_out/gather/sorted.json 2>&1 || { cat gpurun_out/gather/sorted.json; exit 1; }
cat gpurun_out/gather/sorted.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/gather/trace" -o run -- python3 "$ROOT/scripts/bench_gather.py" --reps 3 > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/gpurun_out/gather/fetch" -o run -- python3 "$ROOT/scripts/bench_gather.py" --reps 3 > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/gpurun_out/gather/write" -o run -- python3 "$ROOT/scripts/bench_gather.py" --reps 3 > /dev/null 2>&1 || exit 1
python3 - "$ROOT/gpurun_out/gather" <<'PY'
import csv, glob, sys
d = sys.argv[1]
for sub in ("fetch", "write"):
    for f in glob.glob(d + "/" + sub + "/run_counter_collection.csv"):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "gather_rows" in r["Kernel_Name"]]
        print(sub, "per-dispatch KB:", vals[:4])
for f in glob.glob(d + "/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "gather" in r["Name"] or "copy" in r["Name"].lower():
            print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
