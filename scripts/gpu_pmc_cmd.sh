#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 --pmc run per set) over any python command, summed over the
# kernels whose name contains FILTER: scripts/gpu_pmc_cmd.sh TAG FILTER script.py [args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; FILTER="$2"; shift 2
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM")
[ -n "$PMC_SETS" ] && IFS='|' read -r -a SETS <<< "$PMC_SETS"
i=0
for SET in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $SET --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" "$FILTER" <<'PY'
import csv, glob, sys, collections
out, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
with open(out + "/summary.txt", "w") as fo:
    for k in sorted(agg):
        line = f"{k:28s} {agg[k]:.6g}  ({n[k]} dispatches)"
        print(line)
        fo.write(line + "\n")
PY
