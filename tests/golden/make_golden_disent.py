"""Golden fixtures for NAIS_region_distance_disentangled_Embedding (model.py:409-541; SURVEY.md
8(f4)), produced by the REFERENCE's own class. Run here only:

    python tests/golden/make_golden_disent.py [/root/reference]

forward_disent.npz  forward (model.py:446-455) on [b, n] batches whose target_distance is built
                    as run.py:326-333 does, with the reference's powerLaw.dist (km) over seeded
                    city-sized coordinates; init-like and trained-like parameters (every
                    state_dict entry overwritten with seeded values), H = D as run.py:315.
                    dist/<case>: the same distances alone, for nais_pair_distances.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_params, load_reference  # noqa: E402
from poi_recommendation_models_amd.synthetic import make_checkins  # noqa: E402


def random_state(module, seed, std, bias_std):
    r = np.random.default_rng(seed)
    p = {}
    for k, v in module.state_dict().items():
        shape = tuple(v.shape)
        if k.endswith(".bias"):
            a = r.normal(0, bias_std, shape) if bias_std else np.zeros(shape)
        elif k.startswith("embed_"):
            a = r.normal(0, std, shape)
        else:
            a = r.uniform(-shape[1] ** -0.5, shape[1] ** -0.5, shape)
        p[k] = a.astype(np.float32)
    return p


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    rng = np.random.default_rng(2718)
    P, E, R = 600, 32, 25
    coords = make_checkins(2, P, 3, seed=5).place_coords
    region_of = rng.integers(0, R, P).astype(np.int64)
    out = {"coords": coords, "region_of": region_of}
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 71), ("trained", 0.3, 0.1, 72)):
        m = model.NAIS_region_distance_disentangled_Embedding(P, E, E, 0.5, R, 1)
        p = random_state(m, seed, std, bstd)
        if tag == "trained":     # a distance weight large enough to matter at km scale
            p["embed_distance.weight"] *= 0.2
        load_params(torch, m, p)
        m.eval()
        out.update({f"{tag}/{k}": v for k, v in p.items()})
        for n in (1, 9):
            b = 40
            hist = rng.choice(P, n, replace=False).astype(np.int64)      # one shared history (run.py)
            tgt = rng.integers(0, P, b).astype(np.int64)
            tgt[0] = hist[0]
            hp = [(coords[i][0], coords[i][1]) for i in hist]
            tp = [(coords[i][0], coords[i][1]) for i in tgt]
            td = torch.tensor([[powerLaw.dist(a, c) for c in hp] for a in tp], dtype=torch.float32)
            H2 = torch.from_numpy(np.tile(hist, (b, 1)))
            with torch.no_grad():
                pred = m(H2, torch.from_numpy(tgt), torch.from_numpy(region_of[H2.numpy()]),
                         torch.from_numpy(region_of[tgt]), td).numpy()
            key = f"{tag}/n{n}"
            out[key + "/hist"] = hist
            out[key + "/target"] = tgt
            out[key + "/dist"] = td.numpy()
            out[key + "/pred"] = pred.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "forward_disent.npz"), **out)
    print("golden disentangled fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
