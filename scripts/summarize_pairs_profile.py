#!/usr/bin/env python3
"""Copy a gpu_profile.sh run of the pairs-strategy bench into profiles/<round>/pairs/ and record the
gather kernel's HBM traffic per launch (pmc_by_kernel.csv: per-kernel counter means) in profiles/traffic.json ("pairs_gather").
usage: summarize_pairs_profile.py <prof_dir> <out_dir> <num_users> <num_pois> <world> <block_cols> [precision]"""
import csv
import json
import os
import shutil
import sys

src, dst, users, P, world = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
block_cols = int(sys.argv[6])
precision = sys.argv[7] if len(sys.argv) > 7 else "fp16x6"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
rows = []
for sub in ("pmc_fetch", "pmc_write"):
    for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))):
        n = r["Kernel_Name"]
        if any(t in n for t in ("pair_gather", "pair_bound", "pair_refine", "catalog", "topk", "gather_rows")):  # noqa: E501
            name = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            rows.append({"kernel": name, "dispatch": r["Dispatch_Id"], "counter": r["Counter_Name"],
                         "value_kb": float(r["Counter_Value"]), "grid": r["Grid_Size"],
                         "wg": r["Workgroup_Size"], "lds": r["LDS_Block_Size"], "vgpr": r["VGPR_Count"]})
# one row per (kernel, counter): dispatch count and mean / min / max per dispatch (the per-dispatch
# rows of a full bench run are ~30k lines)
agg = {}
for r in rows:
    agg.setdefault((r["kernel"], r["counter"]), (r, []))[1].append(r["value_kb"])
with open(os.path.join(dst, "pmc_by_kernel.csv"), "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["kernel", "counter", "dispatches", "mean_kb", "min_kb", "max_kb", "wg", "lds", "vgpr"])
    for (kern, ctr), (r0, v) in sorted(agg.items()):
        w.writerow([kern, ctr, len(v), sum(v) / len(v), min(v), max(v), r0["wg"], r0["lds"], r0["vgpr"]])
out = {}
# the headline table kernel: basic variant, D = H = 64, fp16x6 -- the fp32 / fp16x3 /
# region_distance legs' table launches are other instantiations and stay out of the mean
TABLE = {"fp16x6": "catalog_score_x6n_kernel<64, 4, 1, 0>",   # the 16x16x32 form (VAR 0: basic)
         "fp16x3": "catalog_score_x3b_kernel<32, 2, 0, 8, 2>"}
for tag, key in (("pair_gather_topk", "pairs_gather_topk"), ("pair_gather_kernel", "pairs_gather"),
                 ("pair_bound_topk", "pairs_bound_topk"), ("pair_refine_topk", "pairs_refine_topk"),
                 (TABLE.get(precision, "catalog"), "pairs_table_" + precision), ("gather_rows", "gather_rows")):
    sel = [r for r in rows if tag in r["kernel"]]
    f = [r["value_kb"] for r in sel if r["counter"] == "FETCH_SIZE"]
    wr = [r["value_kb"] for r in sel if r["counter"] == "WRITE_SIZE"]
    if not f or not wr:
        continue
    fetch, write = sum(f) / len(f), sum(wr) / len(wr)
    if key == "gather_rows":   # bench.py gather_rows_leg: 4M of 4M rows x d = 128, permutation order
        out[key] = {"kernel": sel[0]["kernel"], "rows": 4_000_000, "dim": 128, "m": 4_000_000,
                    "dispatches": len(f), "fetch_size_kb": fetch, "write_size_kb": write,
                    "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
                    "algorithmic_bytes_per_launch": 4_000_000 * (8 + 8 * 128),
                    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                              "the bench command (its gather_rows leg); bytes = (2*FETCH_SIZE + "
                              "WRITE_SIZE)*1024 per launch (MI355X_MICROARCH.md gfx950 correction)",
                    "source": src}
        continue
    out[key] = {"kernel": sel[0]["kernel"], "num_users": users, "num_pois": P, "world": world,
                "block_cols": block_cols, "precision": precision,
                "dispatches": len(f), "fetch_size_kb": fetch, "write_size_kb": write,
                "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the "
                          "same bench command; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch, averaged "
                          "over the kernel's dispatches (MI355X_MICROARCH.md gfx950 correction)",
                "source": src}
tjp = "profiles/traffic.json"
tj = json.load(open(tjp)) if os.path.exists(tjp) else {}
tj.update(out)
json.dump(tj, open(tjp, "w"), indent=1)
print(json.dumps(out, indent=1))
