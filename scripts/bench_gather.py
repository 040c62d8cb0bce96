#!/usr/bin/env python3
"""HBM roofline of the standalone embedding gather (nais_gather_rows, model.py:64):
out[i] = table[idx[i]] with a table well past the 256 MB Infinity Cache.
Algorithmic bytes per call = m * (8 B index + 4d B row read + 4d B row write).
The reference ceiling is measured in the same process: a device-to-device copy of the same
byte volume (read + write), i.e. the achievable HBM bandwidth on this box."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--m", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="alternative libnais_hip.so to time")
    ap.add_argument("--sorted", action="store_true", help="ascending indices (CSR-history order)")
    ap.add_argument("--reuse", action="store_true",
                    help="i.i.d. random rows (re-reads may hit the Infinity Cache) instead of a "
                         "random permutation (every row read exactly once from HBM)")
    a = ap.parse_args()
    from poi_recommendation_models_amd import _capi
    lib = _capi.load(a.lib) if a.lib else _capi.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(a.rows, a.dim, device=dev, generator=g)
    if a.reuse:
        idx = torch.randint(0, a.rows, (a.m,), device=dev, generator=g)
    else:
        idx = torch.randperm(a.rows, device=dev, generator=g)[:a.m].contiguous()
    if a.sorted:
        idx, _ = torch.sort(idx)
    out = torch.empty(a.m, a.dim, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream

    def gather():
        _capi.check(lib.nais_gather_rows(table.data_ptr(), a.rows, a.dim, idx.data_ptr(), a.m,
                                         out.data_ptr(), sh), "gather")
    t_g = timed(gather, a.reps)
    assert torch.equal(out[:1000], table[idx[:1000]])
    algo = a.m * (8 + 8 * a.dim)
    src = torch.empty(a.m * a.dim, device=dev)
    dst = torch.empty_like(src)
    t_c = timed(lambda: dst.copy_(src), a.reps * 2)
    copy_bw = 2 * src.numel() * 4 / t_c
    print(json.dumps({
        "kernel": "gather_rows_kernel (nais_gather_rows)", "table_bytes": a.rows * a.dim * 4,
        "rows_gathered": a.m, "dim": a.dim, "sorted_indices": a.sorted,
        "index_pattern": "iid random (re-reads)" if a.reuse else "random permutation (each row once)",
        "algorithmic_bytes": algo, "time_ms": t_g * 1e3, "achieved_GBps": algo / t_g / 1e9,
        "measured_copy_GBps": copy_bw / 1e9, "frac_of_measured_copy": algo / t_g / copy_bw,
        "frac_of_8TBps_spec": algo / t_g / 8e12}, indent=1))


if __name__ == "__main__":
    main()
