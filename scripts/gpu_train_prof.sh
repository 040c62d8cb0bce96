#!/bin/bash
# Training kernels: kernel trace + SQ counter passes over scripts/bench_train.py.
#   scripts/gpu_train_prof.sh <tag> [bench_train args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/trainprof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B=("$ROOT/scripts/bench_train.py" --no-torch --steps 10 --warmup 2 --kernel-iters 20 "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${B[@]}" > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
      "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_GDS")
[ -n "$PMC_SETS" ] && IFS='|' read -r -a SETS <<< "$PMC_SETS"
i=0
for SET in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d "$OUT/p$i" -o run -- python3 "${B[@]}" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in glob.glob(out + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for tag in ("train_forward", "train_backward"):
            if tag in k:
                agg[tag][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[tag + r["Counter_Name"]].add(r["Dispatch_Id"])
for tag, d in agg.items():
    print("==", tag)
    for k in sorted(d):
        n = len(cnt[tag + k])
        print(f"  {k:28s} per_dispatch={d[k]/max(n,1):.4g}  (dispatches {n})")
PY
