"""Golden training-step fixtures beyond NAIS_basic at small dims, produced by
the REFERENCE's own autograd. Run here only:

    python tests/golden/make_golden_train_region.py [/root/reference]

train_step_region.npz  one get_NAIS_batch_region-shaped batch (batches.py:67-108: shared
    history, 1 positive + 4 negatives per history item, regions of every POI) through
    forward + BCELoss + backward, dropout off (eval()), for
      region/           NAIS_regionEmbedding(P, 32, 24, 0.5, R)             (model.py:99-187)
      region_distance/  NAIS_region_distance_Embedding(P, 32, 24, 0.5, R, 1) with
                        target_lat_long = latlon_mat[target, history] (run.py:240-245)
      basic128/         NAIS_basic(P, 128, 128, 0.5): run.py's default factor_num = hidden_dim
      distance/         NAIS_distance_Embedding(P, 32, 24, 0.5, R, 1) (model.py:306-408), latlon
                        from a 20x tighter box (x1000 would saturate the sigmoid)
    <case>/p/<param>, <case>/grad/<param>, hist, data, labels, hist_region, data_region, latlon,
    pred, loss.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_params, load_reference  # noqa: E402
from make_golden_disent import random_state  # noqa: E402
from poi_recommendation_models_amd.synthetic import make_checkins  # noqa: E402


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    rng = np.random.default_rng(97)
    P, R = 400, 30
    coords = make_checkins(2, P, 3, seed=8).place_coords
    region_of = rng.integers(0, R, P).astype(np.int64)
    out = {"coords": coords, "region_of": region_of}
    cases = (("region", lambda: model.NAIS_regionEmbedding(P, 32, 24, 0.5, R)),
             ("region_distance", lambda: model.NAIS_region_distance_Embedding(P, 32, 24, 0.5, R, 1)),
             ("basic128", lambda: model.NAIS_basic(P, 128, 128, 0.5)),
             ("distance", lambda: model.NAIS_distance_Embedding(P, 32, 24, 0.5, R, 1)))
    for ci, (case, make) in enumerate(cases):
        m = make()
        p = random_state(m, 300 + ci, 0.3, 0.1)
        load_params(torch, m, p)
        m.eval()                                   # dropout off for parity
        n = 9
        positives = np.sort(rng.choice(P, n, replace=False))
        negs = rng.choice(np.setdiff1d(np.arange(P), positives), 4 * n, replace=False).reshape(n, 4)
        data_ = np.concatenate([positives.reshape(-1, 1), negs], 1).reshape(-1)
        labels = np.concatenate([np.ones((n, 1)), np.zeros((n, 4))], 1).reshape(-1)
        hist = np.repeat(positives.reshape(1, -1), len(data_), 0)
        hreg, dreg = region_of[hist], region_of[data_]
        latlon = np.abs(coords[data_][:, None, :] - coords[hist]).astype(np.float32)   # run.py:47-54
        if case == "distance":    # x1000 saturates the sigmoid at city scale: a tighter box
            latlon = (latlon * 0.05).astype(np.float32)
        args = [torch.from_numpy(hist), torch.from_numpy(data_)]
        if case != "basic128":
            args += [torch.from_numpy(hreg), torch.from_numpy(dreg)]
        if case in ("region_distance", "distance"):
            args.append(torch.from_numpy(latlon))
        pred = m(*args)
        loss = m.loss_func(pred, torch.tensor(labels, dtype=torch.float32))
        loss.backward()
        pre = case + "/"
        out.update({pre + "p/" + k: v for k, v in p.items()})
        out.update({pre + "hist": hist, pre + "data": data_, pre + "labels": labels.astype(np.float32),
                    pre + "hist_region": hreg, pre + "data_region": dreg, pre + "latlon": latlon,
                    pre + "pred": pred.detach().numpy(), pre + "loss": np.float32(loss.item())})
        for k, v in m.named_parameters():
            if v.grad is not None:
                out[pre + "grad/" + k] = v.grad.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "train_step_region.npz"), **out)
    print("golden training fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
