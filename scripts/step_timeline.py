#!/usr/bin/env python3
"""Per-step timeline from a rocprofv3 kernel trace of bench.py: splits the trace into steps at
nais mark_kernel launches (one per step; nais_pair_rows) and reports, per step, the span, the busy
time of each kernel family and the idle gaps on the gather and table queues.
usage: step_timeline.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    n = r["Kernel_Name"]
    fam = ("gather" if "pair_gather" in n else "table" if "catalog_score" in n else "topk" if "topk" in n
           else "mark" if "mark_kernel" in n else "scan" if any(t in n for t in ("count_kernel", "scan_blocks", "place_kernel")) else "other")
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam, n[:60]))
ks.sort()
starts = [i for i, k in enumerate(ks) if k[2] == "mark"]
for si, i0 in enumerate(starts):
    i1 = starts[si + 1] if si + 1 < len(starts) else len(ks)
    seg = ks[i0:i1]
    t0 = seg[0][0]
    t1 = max(k[1] for k in seg)
    busy = defaultdict(float)
    for a, b, f, _ in seg:
        busy[f] += (b - a) / 1e6
    g = sorted((a, b) for a, b, f, _ in seg if f == "gather")
    first_g = (g[0][0] - t0) / 1e6 if g else 0
    gaps = sum(max(0, g[i + 1][0] - g[i][1]) for i in range(len(g) - 1)) / 1e6
    tail = (t1 - g[-1][1]) / 1e6 if g else 0
    print(f"step {si}: span {(t1 - t0) / 1e6:.2f} ms | start->first gather {first_g:.2f} | gather gaps {gaps:.2f} "
          f"| after last gather {tail:.2f} | busy " + ", ".join(f"{f} {v:.2f}" for f, v in sorted(busy.items())))
    if si + 1 < len(starts):
        nxt = ks[starts[si + 1]][0]
        print(f"        idle before next step: {(nxt - t1) / 1e6:.2f} ms")
