#!/usr/bin/env python3
"""Per-dispatch durations of the bench's headline job from a rocprofv3 kernel trace (run_kernel_trace.csv):
the first N dispatches of each kernel in start order are the headline's (bench.py runs it before
its legs; N = (warmup + steps) x launches per job), so their mean is the rocprof figure that the
bench line's HIP-event `avg_launch_ms` must agree with. usage:
  headline_dispatches.py <run_kernel_trace.csv> <dispatches> <name substring> [...]"""
import csv
import sys

import numpy as np

path, n = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
for tag in sys.argv[3:]:
    sel = sorted((r for r in rows if tag in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel[:n]])
    print("%-45s dispatches %5d (of %5d)  mean %.3f ms  median %.3f ms" % (tag, len(d), len(sel), d.mean(), np.median(d)))
