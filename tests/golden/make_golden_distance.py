"""Golden fixtures for NAIS_distance_Embedding (model.py:306-408), produced by
the REFERENCE's own code. Run here only (needs /root/reference):

    python tests/golden/make_golden_distance.py [/root/reference]

forward_distance.npz   NAIS_distance_Embedding.forward (model.py:339-395) on [b, n] batches with
                       target_lat_long built as run.py:47-54 / validation.py:108-118, for a
                       city-sized coordinate box (x1000 saturates the sigmoid) and a 100x tighter
                       one (it does not); init and trained-like parameters
catalog_distance.npz   validation.NAIS_region_distance_validation (validation.py:62-131) run with
                       NAIS_distance_Embedding, as run.py:431 does
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import (Args, capture_validation, data_arrays, load_params, load_reference,  # noqa: E402
                         pack_catalog, params_arrays, split_by_user)
from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins  # noqa: E402


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    rng = np.random.default_rng(4321)
    k_list = [5, 10, 15, 20, 25, 30]

    # ------------------------------------------------------------ forward_distance
    P, E, H = 800, 16, 32
    base = make_checkins(4, P, 5, seed=98).place_coords
    out = {}
    for box, coords in (("city", base), ("tight", base.mean(0) + (base - base.mean(0)) * 0.01)):
        out[f"{box}/coords"] = coords
        for tag, std, bstd, seed in (("init", 0.01, 0.0, 61), ("trained", 0.3, 0.1, 62)):
            p = init_nais_params(P, E, H, seed=seed, emb_std=std, variant="distance", bias_std=bstd)
            m = model.NAIS_distance_Embedding(P, E, H, 0.5, 10, 1)
            load_params(torch, m, p)
            m.eval()
            out.update(params_arrays(f"{box}/{tag}/", p))
            for n in (1, 7):
                b = 48
                hist = np.stack([rng.choice(P, n, replace=False) for _ in range(b)]).astype(np.int64)
                tgt = rng.integers(0, P, b).astype(np.int64)
                tgt[0] = hist[0, 0]
                ll = np.abs(coords[tgt][:, None, :] - coords[hist])           # run.py:51-52
                zeros = torch.zeros_like(torch.from_numpy(hist))
                with torch.no_grad():
                    pred = m(torch.from_numpy(hist), torch.from_numpy(tgt), zeros, zeros[:, 0],
                             torch.tensor(ll, dtype=torch.float32)).numpy()  # validation.py:118
                out[f"{box}/{tag}/n{n}/hist"] = hist
                out[f"{box}/{tag}/n{n}/target"] = tgt
                out[f"{box}/{tag}/n{n}/pred"] = pred.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "forward_distance.npz"), **out)

    # ------------------------------------------------------------ catalog_distance
    P = 1200
    data = make_checkins(12, P, 20, seed=8, num_regions=64)
    data.place_coords = data.place_coords.mean(0) + (data.place_coords - data.place_coords.mean(0)) * 0.01
    X = data.to_scipy()
    coords_list = [tuple(c) for c in data.place_coords.tolist()]
    latlon_mat = run.lat_lon_mat(P, coords_list)                  # run.py:47-54, reference code
    out = data_arrays(data)
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 71), ("trained", 0.3, 0.1, 72)):
        p = init_nais_params(P, 16, 32, seed=seed, emb_std=std, variant="distance", bias_std=bstd)
        m = model.NAIS_distance_Embedding(P, 16, 32, 0.5, 64, 1)
        load_params(torch, m, p)
        chunks, recs, metrics = capture_validation(
            torch, validation, validation.NAIS_region_distance_validation, m, Args(),
            data.num_users, data.test_positive, data.val_positive, X, data.region_of,
            latlon_mat, k_list)
        out.update(params_arrays(f"{tag}/", p))
        out.update(pack_catalog(f"{tag}/", split_by_user(chunks, data), recs, data, keep_full=4))
        out[f"{tag}/metrics"] = np.array(metrics, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "catalog_distance.npz"), **out)
    print("golden distance fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
