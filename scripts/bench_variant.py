#!/usr/bin/env python3
"""A secondary NAIS variant at a BASELINE.json configuration's geometry (the
region_distance variant at config 5: 200k users x 1M POIs, d = H = 128, h <= 200, top-50).

Two timings, each one warm-up + `--steps` timed runs (HIP-synchronised wall clock):
  direct  the per-user route (nais_score_topk, x6n kernel with the distance K-step) over the
          first `--users` users, as bench.py --config 5 times NAIS_basic;
  shard   one rank's POI-column shard of an `--emulate-world`-GPU pairs job over ALL users
          (nais_pair_table + the fused gather), as bench.py --config 5 --strategy pairs
          --emulate-world 8 does for NAIS_basic.
Self-check (test infrastructure): 2 users of the direct run against the numpy oracle on their
top-50 plus 500 sampled candidates (scores within 1e-4, no sampled candidate above the weakest
winner beyond 4 ulps). One JSON line on stdout."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="region_distance", choices=["region_distance", "distance", "region", "basic"])
    ap.add_argument("--num-users", type=int, default=200_000)
    ap.add_argument("--num-pois", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--users", type=int, default=4096, help="users of the direct timing")
    ap.add_argument("--emulate-world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--skip", default="", help="comma list of legs to skip: direct, shard")
    a = ap.parse_args()
    from oracle import nais_oracle
    from poi_recommendation_models_amd import model as M
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs, score_topk
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    dev = torch.device("cuda", 0)
    U, P, D, H, K, R = a.num_users, a.num_pois, a.dim, a.hidden, 50, 1024
    t0 = time.perf_counter()
    data = make_checkins(U, P, a.h_max, seed=2024, num_regions=R)
    p = init_nais_params(P, D, H, seed=11, emb_std=0.3, bias_std=0.1, variant=a.variant, num_regions=R)
    m = {"basic": lambda: M.NAIS_basic(P, D, H, 0.5),
         "region": lambda: M.NAIS_regionEmbedding(P, D, H, 0.5, R),
         "region_distance": lambda: M.NAIS_region_distance_Embedding(P, D, H, 0.5, R, 1),
         "distance": lambda: M.NAIS_distance_Embedding(P, D, H, 0.5, R, 1)}[a.variant]()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(dev).eval()
    m.report_nan = False
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    coords = data.place_coords
    if a.variant == "distance":      # a 100x tighter box keeps the x1000 feature off saturation
        coords = coords.mean(0) + (coords - coords.mean(0)) * 0.01
    kw = {}
    if a.variant in ("region", "region_distance"):
        kw["region_of"] = data.region_of
    if a.variant in ("region_distance", "distance"):
        kw["coords"] = coords
    hl = data.hist_len()
    out = {"variant": a.variant, "num_users": U, "num_pois": P, "embed_dim": D, "hidden": H,
           "h_max": a.h_max, "precision": m.precision, "setup_s": round(time.perf_counter() - t0, 1)}
    din = D + (2 if "distance" in a.variant else 0)
    flop_item = 2 * din * H + 3 * H + 4 * D            # SURVEY.md 8(d), distance columns included

    def timed(fn, steps):
        fn()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            r = fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / steps, r

    if "direct" not in a.skip:
        users = np.arange(a.users)
        warm = users[:64]
        score_topk(m, csr, warm, K, strategy="direct", **kw)
        sec, (ids, sc) = timed(lambda: score_topk(m, csr, users, K, strategy="direct", **kw), a.steps)
        pairs = float((P - hl[users]).sum())
        work = float(((P - hl[users]) * hl[users]).sum())
        tf = work * flop_item / sec / 1e12
        out["direct"] = {"users": int(len(users)), "seconds": sec, "pairs_per_s": pairs / sec,
                         "kernel": "catalog_score_x6n_kernel (nais_score_topk)",
                         "achieved_tflops": tf, "peak_tflops": 2500.0 / 6, "frac": tf / (2500.0 / 6)}
        ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
        rng = np.random.default_rng(3)
        worst, ok = 0.0, True
        for u in (int(np.argmin(hl[users])), int(np.argmax(hl[users]))):
            hist = data.history(u)
            cand = nais_oracle.complement_candidates(hist, P)
            extra = rng.choice(cand, 500, replace=False)
            probe = np.concatenate([ids[u], extra[~np.isin(extra, ids[u])]])
            uh = np.broadcast_to(hist, (len(probe), len(hist)))
            if a.variant == "region_distance":
                ll = nais_oracle.latlon_pairs(coords, np.broadcast_to(probe[:, None], uh.shape), uh).astype(np.float32)
                ref = nais_oracle._sigmoid(nais_oracle.attention_region_distance(
                    p, uh, probe, data.region_of[uh], data.region_of[probe], ll))
            elif a.variant == "distance":
                ll = nais_oracle.latlon_pairs(coords, np.broadcast_to(probe[:, None], uh.shape), uh).astype(np.float32)
                ref = nais_oracle._sigmoid(nais_oracle.attention_distance(p, uh, probe, ll))
            elif a.variant == "region":
                ref = nais_oracle._sigmoid(nais_oracle.attention_region(p, uh, probe, data.region_of[uh],
                                                                       data.region_of[probe]))
            else:
                ref = nais_oracle.forward_basic(p, uh, probe)[0]
            worst = max(worst, float(np.max(np.abs(ref[:K] - sc[u]))))
            weakest = float(ref[:K].min())
            ok = ok and bool(np.all(ref[K:] - weakest <= 4 * np.spacing(np.float32(weakest))))
        out["direct"]["self_check"] = {"users": "shortest and longest history of the timed users",
                                       "oracle": "oracle/nais_oracle.py (numpy), top-50 + 500 sampled",
                                       "max_abs_score_diff": worst, "ok": ok and worst <= 1e-4}
    if "shard" not in a.skip:
        S = (P + a.emulate_world - 1) // a.emulate_world
        ev = []
        users = np.arange(U)
        sec, _ = timed(lambda: _score_topk_pairs(m, csr, users, K, kw.get("region_of"), kw.get("coords"),
                                                 None, None, force=True, cols=(0, S)), a.steps)
        pairs = float(S) * U - float(np.count_nonzero(data.indices < S))
        out["shard"] = {"emulated_world": a.emulate_world, "columns": S, "seconds_per_rank_step": sec,
                        "pairs_per_s_per_gpu": pairs / sec,
                        "note": "one rank's POI-column shard of the whole job, timed alone on one GPU"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
