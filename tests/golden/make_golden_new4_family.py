"""Golden fixtures for the rest of the New4 family, produced by the REFERENCE's
own classes: New4_padding (model.py:1308), all_in_out (:1447), nearPOI_embedding (:1578),
no_POI_emb (:1707), transform_ingoing_outgoing (:1822), transform_attn (:1959) and
only_area_not_inout (:2100). Run here only:

    python tests/golden/make_golden_new4_family.py [/root/reference]

As in make_golden_new4.py, torch.Tensor.cuda is the identity for the run (the forwards hard-code
`.cuda()` on the near-POI indices). Parameters: every state_dict entry of the reference module is
overwritten with seeded values of its shape (embeddings N(0, 0.3), Linear weights U(+-1/sqrt(in)),
biases N(0, 0.1)), so the projections of transform_* have non-zero biases.

new4_family.npz   per member M: M/<param>, M/n{1,7}/{hist,target,pred} (forward on [48, n]
                  batches), and new4_validation on a 10-user catalog: M/cat/... (make_golden
                  pack_catalog layout) + M/cat/metrics; shared near / near_cat and the dataset;
                  transform_attn/cat1/...: the same with 1-3 item histories (its own data/ keys).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import (Args, capture_validation, data_arrays, load_params, load_reference,  # noqa: E402
                         pack_catalog, split_by_user)
from make_golden_new4 import near_pois  # noqa: E402
from poi_recommendation_models_amd.synthetic import make_checkins  # noqa: E402

MEMBERS = ("New4_padding", "all_in_out", "nearPOI_embedding", "no_POI_emb",
           "transform_ingoing_outgoing", "transform_attn", "only_area_not_inout")


def random_state(module, seed):
    r = np.random.default_rng(seed)
    p = {}
    for k, v in module.state_dict().items():
        shape = tuple(v.shape)
        if k.endswith(".bias"):
            a = r.normal(0, 0.1, shape)
        elif k.startswith("embed_"):
            a = r.normal(0, 0.3, shape)
        else:
            a = r.uniform(-shape[1] ** -0.5, shape[1] ** -0.5, shape)
        p[k] = a.astype(np.float32)
    return p


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    orig_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        rng = np.random.default_rng(1357)
        P, E, H, R, K = 700, 32, 32, 20, 10
        Pc, Kc = 1500, 12
        data = make_checkins(10, Pc, 20, seed=9, num_regions=30)
        X = data.to_scipy()
        out = {"near": near_pois(P, K, 1), "near_cat": near_pois(Pc, Kc, 2)}
        out.update(data_arrays(data))
        for mi, name in enumerate(MEMBERS):
            m = getattr(model, name)(P, E, H, 0.5, R)
            p = random_state(m, 500 + mi)
            load_params(torch, m, p)
            m.eval()
            out.update({f"{name}/{k}": v for k, v in p.items()})
            for n in (1, 7):
                b = 48
                hist = np.stack([rng.choice(P, n, replace=False) for _ in range(b)]).astype(np.int64)
                tgt = rng.integers(0, P, b).astype(np.int64)
                tgt[0] = hist[0, 0]
                with torch.no_grad():
                    pred = m(torch.from_numpy(hist), torch.from_numpy(tgt), out["near"],
                             torch.zeros(b, dtype=torch.int64)).numpy()
                out[f"{name}/n{n}/hist"] = hist
                out[f"{name}/n{n}/target"] = tgt
                out[f"{name}/n{n}/pred"] = pred.astype(np.float32)
            # new4_validation (validation.py:254-280) on the catalog data
            mc = getattr(model, name)(Pc, E, H, 0.5, 30)
            pc = random_state(mc, 600 + mi)
            load_params(torch, mc, pc)
            chunks, recs, metrics = capture_validation(
                torch, validation, validation.new4_validation, mc, Args(), data.num_users,
                data.test_positive, data.val_positive, X, data.region_of, [5, 10, 15, 20, 25, 30],
                out["near_cat"])
            out.update({f"{name}/cat/{k}": v for k, v in pc.items()})
            out.update(pack_catalog(f"{name}/cat/", split_by_user(chunks, data), recs, data, keep_full=3))
            out[f"{name}/cat/metrics"] = np.array(metrics, dtype=np.float64)
            if name == "transform_attn":
                # one-item histories couple the rows of each 1024-candidate chunk (model.py:2042)
                d1 = make_checkins(4, Pc, 3, seed=17, num_regions=30)
                assert (np.diff(d1.indptr) == 1).any()
                chunks, recs, metrics = capture_validation(
                    torch, validation, validation.new4_validation, mc, Args(), d1.num_users,
                    d1.test_positive, d1.val_positive, d1.to_scipy(), d1.region_of,
                    [5, 10, 15, 20, 25, 30], out["near_cat"])
                out.update({f"{name}/cat1/data/{k}": v for k, v in data_arrays(d1).items()})
                out.update(pack_catalog(f"{name}/cat1/", split_by_user(chunks, d1), recs, d1, keep_full=4))
            print(name, "done", flush=True)
        np.savez_compressed(os.path.join(HERE, "new4_family.npz"), **out)
    finally:
        torch.Tensor.cuda = orig_cuda
    print("golden New4-family fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
