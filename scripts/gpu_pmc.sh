#!/bin/bash
# SQ counter passes for one catalog-kernel variant: scripts/gpu_pmc.sh <tag> <precision> [ab args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; PREC="$2"; shift 2
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
AB=("$ROOT/scripts/ab_catalog.py" --only "$PREC" --rounds 1 "$@")
i=0
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM")
[ -n "$PMC_SETS" ] && IFS='|' read -r -a SETS <<< "$PMC_SETS"
for SET in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d "$OUT/p$i" -o run -- python3 "${AB[@]}" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "catalog" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.4g}")
PY
