"""Golden fixtures for New4 (model.py:1169-1306) and new4_validation
(validation.py:254-280), produced by the REFERENCE's own code. Run here only:

    python tests/golden/make_golden_new4.py [/root/reference]

New4.forward hard-codes `.cuda()` on the near-POI index tensor (model.py:1215); this container
has no GPU, so the run replaces torch.Tensor.cuda with the identity for its duration (device
placement only -- every op then runs on the CPU as it would on the GPU). nearPOI is a random
[P, K] id array with each POI first in its own list (as argpartition of a distance matrix with a
zero diagonal usually gives); New4 consumes it as given.

new4_forward.npz   New4.forward on [b, n] batches, init and trained-like parameters
new4_catalog.npz   new4_validation (P = 1500 > 1024 + h: the reference's chunk loop needs >= 2
                   chunks per user, validation.py:264-270)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import (Args, capture_validation, data_arrays, load_params, load_reference,  # noqa: E402
                         pack_catalog, params_arrays, split_by_user)
from poi_recommendation_models_amd.synthetic import make_checkins  # noqa: E402


def new4_params(P, E, H, R, seed, std, bias_std):
    r = np.random.default_rng(seed)
    f = np.float32
    p = {"embed_ingoing.weight": r.normal(0, std, (P, E // 4)).astype(f),
         "embed_outgoing.weight": r.normal(0, std, (P, E // 4)).astype(f),
         "embed_history.weight": r.normal(0, std, (P, E // 2)).astype(f),
         "embed_target.weight": r.normal(0, std, (P, E // 2)).astype(f),
         "embed_region.weight": r.normal(0, std, (R, E // 2)).astype(f),
         "attn_layer1.weight": r.uniform(-E ** -0.5, E ** -0.5, (H, E)).astype(f),
         "attn_layer1.bias": (r.normal(0, bias_std, H) if bias_std else np.zeros(H)).astype(f),
         "attn_layer2.weight": r.uniform(-H ** -0.5, H ** -0.5, (1, H)).astype(f)}
    for n in ("query", "key", "value"):
        p[n + ".weight"] = r.uniform(-(E // 2) ** -0.5, (E // 2) ** -0.5, (E // 2, E // 2)).astype(f)
        p[n + ".bias"] = np.zeros(E // 2, f)
    return p


def near_pois(P, K, seed):
    r = np.random.default_rng(seed)
    out = np.empty((P, K), np.int64)
    for p in range(P):
        others = r.choice(np.setdiff1d(np.arange(P), [p]), K - 1, replace=False)
        out[p] = np.r_[p, others]
    return out


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    orig_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        rng = np.random.default_rng(2468)
        # ------------------------------------------------------------ new4_forward
        P, E, H, R, K = 700, 32, 32, 20, 10
        out = {"near": near_pois(P, K, 1)}
        for tag, std, bstd, seed in (("init", 0.01, 0.0, 81), ("trained", 0.3, 0.1, 82)):
            p = new4_params(P, E, H, R, seed, std, bstd)
            m = model.New4(P, E, H, 0.5, R)
            load_params(torch, m, p)
            m.eval()
            out.update(params_arrays(f"{tag}/", p))
            for n in (1, 7):
                b = 48
                hist = np.stack([rng.choice(P, n, replace=False) for _ in range(b)]).astype(np.int64)
                tgt = rng.integers(0, P, b).astype(np.int64)
                tgt[0] = hist[0, 0]
                with torch.no_grad():
                    pred = m(torch.from_numpy(hist), torch.from_numpy(tgt), out["near"],
                             torch.zeros(b, dtype=torch.int64)).numpy()
                out[f"{tag}/n{n}/hist"] = hist
                out[f"{tag}/n{n}/target"] = tgt
                out[f"{tag}/n{n}/pred"] = pred.astype(np.float32)
        np.savez_compressed(os.path.join(HERE, "new4_forward.npz"), **out)

        # ------------------------------------------------------------ new4_catalog
        P, K = 1500, 12
        data = make_checkins(10, P, 20, seed=9, num_regions=30)
        X = data.to_scipy()
        out = data_arrays(data)
        out["near"] = near_pois(P, K, 2)
        for tag, std, bstd, seed in (("init", 0.01, 0.0, 91), ("trained", 0.3, 0.1, 92)):
            p = new4_params(P, 32, 32, 30, seed, std, bstd)
            m = model.New4(P, 32, 32, 0.5, 30)
            load_params(torch, m, p)
            chunks, recs, metrics = capture_validation(
                torch, validation, validation.new4_validation, m, Args(), data.num_users,
                data.test_positive, data.val_positive, X, data.region_of, [5, 10, 15, 20, 25, 30],
                out["near"])
            out.update(params_arrays(f"{tag}/", p))
            out.update(pack_catalog(f"{tag}/", split_by_user(chunks, data), recs, data, keep_full=4))
            out[f"{tag}/metrics"] = np.array(metrics, dtype=np.float64)
        np.savez_compressed(os.path.join(HERE, "new4_catalog.npz"), **out)
    finally:
        torch.Tensor.cuda = orig_cuda
    print("golden New4 fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
