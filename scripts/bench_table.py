#!/usr/bin/env python3
"""A/B of the pair-table kernel (nais_pair_table) in ONE process: config-4 geometry (J = P =
100k distinct history POIs, d = H = 64), `--blocks` 512-column blocks per round, interleaved rounds
over (library, precision) variants, HIP events on the launch stream. Reports ms per block and
algorithmic TFLOP/s (2dH + 3H + 4d FLOP per pair), plus max |de| between variants.
Extra builds: --lib NAME=PATH (scripts/build_ab.py output)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-pois", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--cols", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--only", default="fp16x6")
    ap.add_argument("--variant", default="basic", choices=["basic", "region", "region_distance", "distance"])
    a = ap.parse_args()
    from poi_recommendation_models_amd import _capi
    from poi_recommendation_models_amd import model as M
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    dev = torch.device("cuda", 0)
    P, D, H, W = a.num_pois, a.dim, a.hidden, a.cols
    R = 1024
    p = init_nais_params(P, D, H, seed=6, emb_std=0.3, bias_std=0.1, variant=a.variant, num_regions=R)
    m = {"basic": lambda: M.NAIS_basic(P, D, H, 0.5),
         "region": lambda: M.NAIS_regionEmbedding(P, D, H, 0.5, R),
         "region_distance": lambda: M.NAIS_region_distance_Embedding(P, D, H, 0.5, R, 1),
         "distance": lambda: M.NAIS_distance_Embedding(P, D, H, 0.5, R, 1)}[a.variant]()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(dev).eval()
    side = make_checkins(2, P, 2, seed=1, num_regions=R)
    reg = torch.as_tensor(side.region_of, dtype=torch.int64, device=dev)
    cor = torch.as_tensor(np.ascontiguousarray(side.place_coords, dtype=np.float64), device=dev)
    reg_p = reg.data_ptr() if a.variant in ("region", "region_distance") else None
    cor_p = cor.data_ptr() if a.variant in ("region_distance", "distance") else None
    items = torch.arange(P, dtype=torch.int64, device=dev)
    J = P
    libs = {"lib": _capi.load()}
    for spec in a.lib:
        name, path = spec.split("=", 1)
        libs[name] = _capi.load(path)
    variants = [(ln, prec) for ln in libs for prec in a.only.split(",")]
    tabs = {v: torch.empty(2, J, W, device=dev) for v in variants}   # e rows then e*s rows, ld = W
    st = torch.cuda.current_stream(dev)
    times = {v: [] for v in variants}
    for r in range(a.rounds + 1):
        for v in variants:
            lib = libs[v[0]]
            m.precision = v[1]
            prm = m.nais_params()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for b in range(a.blocks):
                c0 = (b * W) % (P - W)
                _capi.check(lib.nais_pair_table(prm, items.data_ptr(), J, c0, W, reg_p, cor_p, None,
                                                tabs[v][0].data_ptr(), tabs[v][1].data_ptr(), W,
                                                None, st.cuda_stream), "nais_pair_table")
            e1.record(st)
            torch.cuda.synchronize(dev)
            if r > 0:
                times[v].append(e0.elapsed_time(e1) / a.blocks)
    din = D + (2 if "distance" in a.variant else 0)
    flop = J * W * (2 * din * H + 3 * H + 4 * D)
    base = tabs[variants[0]]
    out = {}
    for v in variants:
        ms = float(np.median(times[v]))
        d = float((tabs[v] - base).abs().max().item())
        rel = float(((tabs[v] - base).abs() / base.abs().clamp_min(1e-30)).max().item())
        out.setdefault("max_rel_diff_vs_first", {})["%s/%s" % v] = rel
        out["%s/%s" % v] = {"ms_per_block": ms, "tflops": flop / ms / 1e9, "max_abs_diff_vs_first": d}
        print("%-24s %8.3f ms/block  %6.1f TF/s  max|d| %.3g" % ("%s/%s" % v, ms, flop / ms / 1e9, d),
              flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
