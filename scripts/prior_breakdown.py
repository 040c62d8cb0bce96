"""Config-4 job with the power-law prior (bench.py's prior_path), phase by phase: per-kind HIP-event
totals of one job (table stream: e / es + pr_d tables; gather stream: score + prior gathers; the
blend top-k), next to the plain job. Usage: python scripts/prior_breakdown.py [--reps 2]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poi_recommendation_models_amd import catalog  # noqa: E402
from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_basic  # noqa: E402
from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cols", type=int, default=0, help="score only POIs [0, cols) (0: all)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    U, P, D, K = 50_000, 100_000, 64, 50
    data = make_checkins(U, P, 200, seed=2024)
    p = init_nais_params(P, D, D, seed=7, emb_std=0.3, bias_std=0.1)
    m = NAIS_basic(P, D, D, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(dev).eval()
    m.report_nan = False
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    users = np.arange(U)
    prior = (0.052, -1.37, 0.2, data.place_coords)
    cols = (0, a.cols) if a.cols else None
    out = {}
    for name, pr in (("plain", None), ("prior", prior)):
        _score_topk_pairs(m, csr, users, K, None, None, None, None, force=True, prior=pr, cols=cols)
        torch.cuda.synchronize()
        for r in range(a.reps):
            ev = []
            t0 = time.perf_counter()
            _score_topk_pairs(m, csr, users, K, None, None, None, None, force=True, prior=pr,
                              events=ev, cols=cols)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            per = {}
            for kind, e0, e1, n in ev:
                if e0 is None:
                    per[kind] = n
                else:
                    per[kind] = per.get(kind, 0.0) + e0.elapsed_time(e1)
            per["wall_ms"] = wall
            out[f"{name}_{r}"] = per
            print(name, json.dumps(per), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
