#!/usr/bin/env python3
"""A/B the catalog scorer variants in ONE process (cdna_hip_programming.md rule 24):
interleaved rounds of nais_score_catalog per variant on the config-4 geometry, HIP-event
timing on the launch stream, plus max |dscore| between variants.
Variants: 'fp32', 'fp16x3', and optionally extra .so builds given as --lib NAME=PATH
(each runs in both precisions)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--num-pois", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--variant", default="basic")
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--only", default=None, help="comma list of precisions to run")
    a = ap.parse_args()
    from poi_recommendation_models_amd import _capi
    from poi_recommendation_models_amd.catalog import DeviceCSR
    from poi_recommendation_models_amd.model import NAIS_basic, NAIS_regionEmbedding, NAIS_region_distance_Embedding
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    dev = torch.device("cuda", 0)
    P, D, H = a.num_pois, a.dim, a.hidden
    data = make_checkins(a.users, P, a.h_max, seed=5, num_regions=1024)
    p = init_nais_params(P, D, H, seed=6, emb_std=0.3, bias_std=0.1, variant=a.variant, num_regions=1024)
    if a.variant == "basic":
        m = NAIS_basic(P, D, H, 0.5)
    elif a.variant == "region":
        m = NAIS_regionEmbedding(P, D, H, 0.5, 1024)
    else:
        m = NAIS_region_distance_Embedding(P, D, H, 0.5, 1024, 1)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(dev).eval()
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    hl = data.hist_len()
    order = np.argsort(-(P - hl) * hl, kind="stable").astype(np.int32)
    users = torch.from_numpy(order).to(dev)
    reg = torch.from_numpy(data.region_of).to(dev) if a.variant != "basic" else None
    cor = torch.from_numpy(data.place_coords).to(dev) if a.variant == "region_distance" else None
    libs = {"lib": _capi.load()}
    for spec in a.lib:
        name, path = spec.split("=", 1)
        libs[name] = _capi.load(path)
    precs = a.only.split(",") if a.only else ["fp32", "fp16x3", "fp16x3_pairsplit"]
    variants = [(ln, prec) for ln in libs for prec in precs]
    out = {v: torch.empty(a.users, P, device=dev) for v in variants}
    times = {v: [] for v in variants}
    stream = torch.cuda.current_stream(dev)
    work = float(((P - hl) * hl).sum()) * (2 * D * H + 3 * H + 4 * D)
    for r in range(a.rounds + 1):
        for v in variants:
            ln, prec = v
            m.precision = prec
            prm = m.nais_params()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = libs[ln].nais_score_catalog(prm, csr.indptr.data_ptr(), csr.indices.data_ptr(),
                                             users.data_ptr(), a.users, _capi.ptr(reg), _capi.ptr(cor),
                                             None, out[v].data_ptr(), P, None, stream.cuda_stream)
            e1.record(stream)
            assert rc == 0, libs[ln].nais_last_error()
            torch.cuda.synchronize()
            if r > 0:
                times[v].append(e0.elapsed_time(e1))
    base = out[variants[0]]
    res = {}
    for v in variants:
        t = np.array(times[v])
        res["/".join(v)] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                            "tflops": work / (np.median(t) / 1e3) / 1e12,
                            "max_abs_diff_vs_first": float((out[v] - base).abs().max().item())}
    print(json.dumps({"users": a.users, "P": P, "D": D, "H": H, "variant": a.variant, "results": res}, indent=1))


if __name__ == "__main__":
    main()
