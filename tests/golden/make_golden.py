"""Capture golden vectors from the reference itself (run HERE only; never on the GPU box).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

The reference (muyeon-jo/POI_recommendation_models) is pure Python + PyTorch and has no tests
or fixtures of its own, so parity is pinned by running its NAIS path on
seeded synthetic inputs and committing inputs + outputs as small .npz fixtures.

`model.py:4-6` imports torch_geometric / torchmetrics / haversine, which are not installed and
are not used by any NAIS symbol (GCNConv only in GGLR/GPR model.py:630-705; the torchmetrics
function is never called; haversine is unused in model.py). They are replaced by empty
placeholder modules in sys.modules before import, as recorded in SURVEY.md 8(c). No
placeholder symbol is ever called on the paths captured here.

Fixtures written to tests/golden/:
  forward_basic.npz            NAIS_basic.forward (model.py:40-95) incl. mask and NaN rows
  forward_region.npz           NAIS_regionEmbedding.forward (model.py:132-185)
  forward_region_distance.npz  NAIS_region_distance_Embedding.forward (model.py:231-302)
  catalog_basic.npz            validation.NAIS_validation (validation.py:7-31), 2 weight sets
  catalog_region.npz           validation.NAIS_region_validation (validation.py:34-59)
  catalog_region_distance.npz  validation.NAIS_region_distance_validation (validation.py:62-131)
  powerlaw.npz                 powerLaw.dist / pr_d / predict / fit_distance_distribution, run.normalize
  train_step.npz               NAIS_basic forward + BCELoss backward, dropout off (model.py:21,40-97)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from poi_recommendation_models_amd.synthetic import make_checkins, init_nais_params  # noqa: E402


def load_reference(path):
    for name in ["torch_geometric", "torch_geometric.nn", "torchmetrics", "torchmetrics.functional",
                 "torchmetrics.functional.pairwise", "haversine"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["torch_geometric.nn"].GCNConv = None
    sys.modules["torchmetrics.functional.pairwise"].pairwise_manhattan_distance = None
    sys.modules["haversine"].haversine = None
    sys.modules["haversine"].haversine_vector = None
    sys.path.insert(0, path)
    import model, validation, powerLaw, eval_metrics, run  # noqa: E401
    return model, validation, powerLaw, eval_metrics, run


class Args:
    topk = 50
    powerlaw_weight = 0.2


def load_params(torch, module, p):
    sd = module.state_dict()
    for k in sd:
        if k in p:
            sd[k] = torch.from_numpy(np.ascontiguousarray(p[k]))
    module.load_state_dict(sd)


def capture_validation(torch, validation, fn, model, *args):
    """Run a reference validation function, capturing per-chunk (targets, scores) through a
    forward hook and the recommended lists through eval_metrics.evaluate_mp."""
    chunks, recs = [], {}
    h = model.register_forward_hook(
        lambda m, inp, out: chunks.append((inp[1].detach().numpy().copy(), out.detach().numpy().copy())))
    orig = validation.eval_metrics.evaluate_mp

    def spy(positive, rec, k_list):
        recs.setdefault("rec", [list(map(int, r)) for r in rec])
        return orig(positive, rec, k_list)

    validation.eval_metrics.evaluate_mp = spy
    try:
        metrics = fn(model, *args)
    finally:
        validation.eval_metrics.evaluate_mp = orig
        h.remove()
    return chunks, recs["rec"], metrics


def split_by_user(chunks, data):
    """Reassemble per-user full-catalog score vectors from the hook's chunk stream."""
    out, i = [], 0
    for u in range(data.num_users):
        need = data.num_pois - (data.indptr[u + 1] - data.indptr[u])
        tg, sc = [], []
        got = 0
        while got < need:
            t, s = chunks[i]
            tg.append(t)
            sc.append(s)
            got += len(t)
            i += 1
        out.append((np.concatenate(tg), np.concatenate(sc)))
    return out


def pack_catalog(prefix, per_user, recs, data, keep_full):
    d = {}
    topk_scores = []
    for u, (tg, sc) in enumerate(per_user):
        lut = dict(zip(tg.tolist(), sc.tolist()))
        topk_scores.append([lut[c] for c in recs[u]])
        if u < keep_full:
            d[f"{prefix}full_scores_u{u}"] = sc.astype(np.float32)
    d[f"{prefix}topk_ids"] = np.array(recs, dtype=np.int64)
    d[f"{prefix}topk_scores"] = np.array(topk_scores, dtype=np.float32)
    return d


def data_arrays(data):
    lens = [len(x) for x in data.test_positive]
    vlens = [len(x) for x in data.val_positive]
    return dict(indptr=data.indptr, indices=data.indices, coords=data.place_coords,
                region_of=data.region_of, num_pois=np.int64(data.num_pois),
                num_users=np.int64(data.num_users), num_regions=np.int64(data.num_regions),
                test_flat=np.array(sum(data.test_positive, []), dtype=np.int64),
                test_len=np.array(lens, dtype=np.int64),
                val_flat=np.array(sum(data.val_positive, []), dtype=np.int64),
                val_len=np.array(vlens, dtype=np.int64))


def params_arrays(prefix, p):
    return {prefix + k: v for k, v in p.items()}


def main(ref_path="/root/reference"):
    import torch
    torch.set_num_threads(8)
    model, validation, powerLaw, eval_metrics, run = load_reference(ref_path)
    k_list = [5, 10, 15, 20, 25, 30]
    rng = np.random.default_rng(1234)

    # ---------------------------------------------------------------- forward_basic
    P, D, H = 1000, 16, 16
    out = {}
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 11), ("trained", 0.3, 0.1, 12)):
        p = init_nais_params(P, D, H, seed=seed, emb_std=std, bias_std=bstd)
        m = model.NAIS_basic(P, D, H, 0.5)
        load_params(torch, m, p)
        m.eval()
        out.update(params_arrays(f"{tag}/", p))
        for n in (1, 5, 20):
            b = 64
            hist = np.stack([rng.choice(P, n, replace=False) for _ in range(b)]).astype(np.int64)
            tgt = rng.integers(0, P, b).astype(np.int64)
            tgt[0] = hist[0, n // 2]          # target inside history -> masked term (model.py:77-78)
            if n == 1:
                tgt[1:8] = hist[1:8, 0]       # single-item history equal to target -> 0/0 = NaN
            with torch.no_grad():
                pred = m(torch.from_numpy(hist), torch.from_numpy(tgt)).numpy()
            out[f"{tag}/n{n}/hist"] = hist
            out[f"{tag}/n{n}/target"] = tgt
            out[f"{tag}/n{n}/pred"] = pred.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "forward_basic.npz"), **out)

    # ------------------------------------------------------- forward_region(_distance)
    P, E, H, R = 800, 16, 32, 40
    coords = make_checkins(4, P, 5, seed=99).place_coords
    for variant, fname in (("region", "forward_region.npz"),
                           ("region_distance", "forward_region_distance.npz")):
        out = {"coords": coords}
        for tag, std, bstd, seed in (("init", 0.01, 0.0, 21), ("trained", 0.3, 0.1, 22)):
            p = init_nais_params(P, E, H, seed=seed, emb_std=std, variant=variant,
                                 num_regions=R, bias_std=bstd)
            if variant == "region":
                m = model.NAIS_regionEmbedding(P, E, H, 0.5, R)
            else:
                m = model.NAIS_region_distance_Embedding(P, E, H, 0.5, R, 1)
            load_params(torch, m, p)
            m.eval()
            out.update(params_arrays(f"{tag}/", p))
            region_of = rng.integers(0, R, P).astype(np.int64)
            out[f"{tag}/region_of"] = region_of
            for n in (1, 7):
                b = 48
                hist = np.stack([rng.choice(P, n, replace=False) for _ in range(b)]).astype(np.int64)
                tgt = rng.integers(0, P, b).astype(np.int64)
                tgt[0] = hist[0, 0]
                hr, tr = region_of[hist], region_of[tgt]
                args = [torch.from_numpy(hist), torch.from_numpy(tgt),
                        torch.from_numpy(hr), torch.from_numpy(tr)]
                if variant == "region_distance":
                    ll = np.abs(coords[tgt][:, None, :] - coords[hist])   # run.py:51-52
                    args.append(torch.tensor(ll, dtype=torch.float32))     # validation.py:118
                with torch.no_grad():
                    pred = m(*args).numpy()
                out[f"{tag}/n{n}/hist"] = hist
                out[f"{tag}/n{n}/target"] = tgt
                out[f"{tag}/n{n}/pred"] = pred.astype(np.float32)
        np.savez_compressed(os.path.join(HERE, fname), **out)

    # ---------------------------------------------------------------- catalog_basic
    data = make_checkins(24, 2000, 20, seed=5, empty_positive_every=7)
    X = data.to_scipy()
    out = data_arrays(data)
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 31), ("trained", 0.3, 0.1, 32)):
        p = init_nais_params(2000, 16, 16, seed=seed, emb_std=std, bias_std=bstd)
        m = model.NAIS_basic(2000, 16, 16, 0.5)
        load_params(torch, m, p)
        chunks, recs, metrics = capture_validation(
            torch, validation, validation.NAIS_validation, m, Args(), data.num_users,
            data.test_positive, data.val_positive, X, k_list)
        out.update(params_arrays(f"{tag}/", p))
        out.update(pack_catalog(f"{tag}/", split_by_user(chunks, data), recs, data, keep_full=6))
        out[f"{tag}/metrics"] = np.array(metrics, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "catalog_basic.npz"), **out)

    # --------------------------------------------------------------- catalog_region
    data = make_checkins(16, 2000, 20, seed=6, num_regions=64)
    X = data.to_scipy()
    out = data_arrays(data)
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 41), ("trained", 0.3, 0.1, 42)):
        p = init_nais_params(2000, 16, 32, seed=seed, emb_std=std, variant="region",
                             num_regions=64, bias_std=bstd)
        m = model.NAIS_regionEmbedding(2000, 16, 32, 0.5, 64)
        load_params(torch, m, p)
        chunks, recs, metrics = capture_validation(
            torch, validation, validation.NAIS_region_validation, m, Args(), data.num_users,
            data.test_positive, data.val_positive, X, data.region_of, k_list)
        out.update(params_arrays(f"{tag}/", p))
        out.update(pack_catalog(f"{tag}/", split_by_user(chunks, data), recs, data, keep_full=4))
        out[f"{tag}/metrics"] = np.array(metrics, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "catalog_region.npz"), **out)

    # ------------------------------------------------------ catalog_region_distance
    P = 1200
    data = make_checkins(12, P, 20, seed=7, num_regions=64)
    X = data.to_scipy()
    coords_list = [tuple(c) for c in data.place_coords.tolist()]
    latlon_mat = run.lat_lon_mat(P, coords_list)                  # run.py:47-54, reference code
    out = data_arrays(data)
    for tag, std, bstd, seed in (("init", 0.01, 0.0, 51), ("trained", 0.3, 0.1, 52)):
        p = init_nais_params(P, 16, 32, seed=seed, emb_std=std, variant="region_distance",
                             num_regions=64, bias_std=bstd)
        m = model.NAIS_region_distance_Embedding(P, 16, 32, 0.5, 64, 1)
        load_params(torch, m, p)
        chunks, recs, metrics = capture_validation(
            torch, validation, validation.NAIS_region_distance_validation, m, Args(),
            data.num_users, data.test_positive, data.val_positive, X, data.region_of,
            latlon_mat, k_list)
        out.update(params_arrays(f"{tag}/", p))
        out.update(pack_catalog(f"{tag}/", split_by_user(chunks, data), recs, data, keep_full=4))
        out[f"{tag}/metrics"] = np.array(metrics, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "catalog_region_distance.npz"), **out)

    # -------------------------------------------------------------------- powerlaw
    out = {}
    pr = np.random.default_rng(77)
    a_pts = np.stack([35.5 + 0.4 * pr.random(600), 139.4 + 0.5 * pr.random(600)], 1)
    b_pts = np.stack([35.5 + 0.4 * pr.random(600), 139.4 + 0.5 * pr.random(600)], 1)
    b_pts[:40] = a_pts[:40]                                   # identical -> 0.0 branch
    b_pts[40:80] = a_pts[40:80] + pr.uniform(-9e-7, 9e-7, (40, 2))   # < 1e-6 branch
    b_pts[80:120] = a_pts[80:120] + pr.uniform(-3e-6, 3e-6, (40, 2))  # tiny but > 1e-6
    out["dist_a"], out["dist_b"] = a_pts, b_pts
    out["dist"] = np.array([powerLaw.dist(tuple(x), tuple(y)) for x, y in zip(a_pts, b_pts)])
    G = powerLaw.PowerLaw(a=0.052, b=-1.37)
    ds = np.concatenate([[0.0, 0.001, 0.01, 0.02], pr.uniform(0, 40, 200)])
    out["pr_d_in"], out["pr_d_ab"] = ds, np.array([0.052, -1.37])
    out["pr_d"] = np.array([G.pr_d(x) for x in ds])
    pdata = make_checkins(30, 400, 25, seed=8)
    # one long history to exercise product underflow
    long_hist = np.sort(pr.choice(400, 300, replace=False))
    indptr = np.concatenate([pdata.indptr, [pdata.indptr[-1] + len(long_hist)]])
    indices = np.concatenate([pdata.indices, long_hist])
    import scipy.sparse as sp
    Xp = sp.csr_matrix((np.ones(len(indices)), indices, indptr), shape=(31, 400))
    coords = pdata.place_coords
    np.random.seed(0)
    Gf = powerLaw.PowerLaw()
    Gf.fit_distance_distribution(Xp, coords)
    np.random.seed(0)
    w0, w1 = np.random.random(), np.random.random()
    out["fit_w_init"] = np.array([w0, w1])
    out["fit_ab"] = np.array([Gf.a, Gf.b])
    out["pl_indptr"], out["pl_indices"], out["pl_coords"] = indptr, indices, coords
    cands = pr.choice(400, 50, replace=False)
    out["predict_cands"] = cands
    out["predict"] = np.array([[Gf.predict(u, int(c)) for c in cands] for u in range(31)])
    out["normalize_in"] = out["predict"][:3]
    out["normalize"] = np.array([run.normalize(list(r)) for r in out["predict"][:3]])
    out["normalize_zero"] = np.array(run.normalize([0.0, 0.0, 0.0]))
    np.savez_compressed(os.path.join(HERE, "powerlaw.npz"), **out)

    # ------------------------------------------------------------------ train_step
    P, D, H = 500, 16, 16
    p = init_nais_params(P, D, H, seed=61, emb_std=0.3, bias_std=0.1)
    m = model.NAIS_basic(P, D, H, 0.5)
    load_params(torch, m, p)
    m.eval()                                 # dropout off for parity (hard part 7)
    positives = np.sort(rng.choice(P, 12, replace=False))
    negs = rng.choice(np.setdiff1d(np.arange(P), positives), 48, replace=False).reshape(12, 4)
    data_ = np.concatenate([positives.reshape(-1, 1), negs], 1).reshape(-1)        # batches.py:38-40
    labels = np.concatenate([np.ones((12, 1)), np.zeros((12, 4))], 1).reshape(-1)  # batches.py:42-44
    hist = np.repeat(positives.reshape(1, -1), len(data_), 0)                     # batches.py:30
    pred = m(torch.from_numpy(hist), torch.from_numpy(data_))
    loss = m.loss_func(pred, torch.tensor(labels, dtype=torch.float32))
    loss.backward()
    out = params_arrays("p/", p)
    out.update(hist=hist, data=data_, labels=labels.astype(np.float32),
               pred=pred.detach().numpy(), loss=np.float32(loss.item()))
    for k, v in m.named_parameters():
        out["grad/" + k] = v.grad.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "train_step.npz"), **out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
