"""Time nais_powerlaw_prior (the per-user prior_kernel, powerLaw.py:90-92) on a config-4-shaped
slice: U users x 100k POIs, h ~ U{1..200}, (a, b) = bench.py's prior. Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1024)
    ap.add_argument("--pois", type=int, default=100_000)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from bench import PRIOR_A, PRIOR_B
    from poi_recommendation_models_amd.catalog import DeviceCSR, prior_rows
    from poi_recommendation_models_amd.synthetic import make_checkins
    dev = torch.device("cuda:0")
    data = make_checkins(a.users, a.pois, a.h_max, seed=2024)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, a.pois, dev)
    G, mx = prior_rows(csr, range(a.users), PRIOR_A, PRIOR_B, data.place_coords, dev)   # warm-up
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        G, mx = prior_rows(csr, range(a.users), PRIOR_A, PRIOR_B, data.place_coords, dev)
        t1.record()
        torch.cuda.synchronize()
        ms.append(t0.elapsed_time(t1))
    zero = float(((G == 0) | (G == -1)).double().mean())
    print(json.dumps({"kernel": "prior_kernel", "users": a.users, "pois": a.pois, "h_max": a.h_max,
                      "ms": ms, "best_ms": min(ms),
                      "pairs_per_s": a.users * a.pois / (min(ms) / 1e3), "frac_zero_or_hist": zero,
                      "checksum_bits": int(G.view(torch.int64).sum().item())}))


if __name__ == "__main__":
    main()
