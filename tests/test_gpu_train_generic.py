"""GPU parity of the general training kernels: NAIS_regionEmbedding and
NAIS_region_distance_Embedding (run.py:153-200, 222-262) and NAIS_basic at the dims the fused
MFMA kernels do not take (run.py's defaults factor_num = hidden_dim = 128; odd sizes), through the
drop-in modules' train-mode forward + BCELoss + backward (nais_train_forward_ex / _backward_ex).

* golden: the reference's own autograd (tests/golden/train_step_region.npz, dropout off)
* oracle: float64 restatement (oracle/train_oracle.train_step) with dropout p = 0.5 injected as
  the device's own mask (nais_dropout_mask) for the same seed
Tolerances as tests/test_gpu_train.py: predictions within SCORE_ATOL (1e-4), every gradient within
GRAD_RTOL x max|reference gradient| of that tensor.
"""
import numpy as np
import pytest
import torch

from _helpers import SCORE_ATOL, adagrad_slack, assert_params_close, load_golden
from oracle import train_oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GRAD_RTOL = 1e-4


def _load(m, p):
    sd = m.state_dict()
    assert set(p) <= set(sd), set(p) - set(sd)    # unused sub-modules (embed_distance) keep their init
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(p[k])) if k in p else v for k, v in sd.items()})
    m.report_nan = False
    return m.to(DEV).train()


def _make(case, p, drop_p=0.0):
    from poi_recommendation_models_amd import model as M
    P, I = p["embed_history.weight"].shape
    H, din = p["attn_layer1.weight"].shape
    if case == "basic":
        m = M.NAIS_basic(P, I, H, 0.5)
    elif case == "distance":
        m = M.NAIS_distance_Embedding(P, I, H, 0.5, 10, 1)
    elif case == "region":
        m = M.NAIS_regionEmbedding(P, din, H, 0.5, p["embed_region.weight"].shape[0])
    else:
        m = M.NAIS_region_distance_Embedding(P, din - 2, H, 0.5, p["embed_region.weight"].shape[0], 1)
    m = _load(m, p)
    if hasattr(m, "drop"):
        m.drop.p = drop_p
    return m


def _t(x):
    return torch.as_tensor(np.ascontiguousarray(x)).to(DEV)


def _step(m, case, hist, data, labels, hreg=None, dreg=None, latlon=None):
    for q in m.parameters():
        q.grad = None
    args = [_t(hist), _t(data)]
    if case != "basic":
        args += [_t(hreg), _t(dreg)]
    if case in ("region_distance", "distance"):
        args.append(_t(latlon))
    pred = m(*args)
    loss = m.loss_func(pred, _t(labels))
    loss.backward()
    grads = {k: q.grad.detach().cpu().numpy() for k, q in m.named_parameters() if q.grad is not None}
    return pred.detach().cpu().numpy(), float(loss.item()), grads


def _assert_grads(got, ref, rtol=GRAD_RTOL):
    assert set(got) == set(ref), set(got) ^ set(ref)
    for k in ref:
        r = np.asarray(ref[k], np.float64).reshape(got[k].shape)
        scale = max(np.abs(r).max(), 1e-30)
        assert np.abs(got[k] - r).max() / scale <= rtol, (k, np.abs(got[k] - r).max() / scale)


@pytest.mark.parametrize("case", ["region", "region_distance", "basic128", "distance"])
def test_train_generic_golden(case):
    z = load_golden("train_step_region.npz")
    pre = case + "/"
    p = {k[len(pre) + 2:]: z[k] for k in z.files if k.startswith(pre + "p/")}
    kind = "basic" if case == "basic128" else case
    m = _make(kind, p)
    pred, loss, grads = _step(m, kind, z[pre + "hist"], z[pre + "data"], z[pre + "labels"],
                              z[pre + "hist_region"], z[pre + "data_region"], z[pre + "latlon"])
    assert np.max(np.abs(pred - z[pre + "pred"])) <= SCORE_ATOL
    assert abs(loss - float(z[pre + "loss"])) <= 1e-5
    _assert_grads(grads, {k[len(pre) + 5:]: z[k] for k in z.files if k.startswith(pre + "grad/")})


def _mask(seed, b, n, H, p):
    from poi_recommendation_models_amd import _capi
    out = torch.empty(b * n * H, dtype=torch.uint8, device=DEV)
    _capi.check(_capi.load().nais_dropout_mask(seed, b, n, H, p, out.data_ptr(),
                                               _capi.stream_handle(torch.device(DEV))),
                "nais_dropout_mask")
    return out.view(b, n, H).cpu().numpy()


def _params(case, P, R, D, H, seed):
    r = np.random.default_rng(seed)
    f = np.float32
    I = D if case in ("basic", "distance") else D // 2
    din = D + 2 if case in ("region_distance", "distance") else D
    p = {"embed_history.weight": r.normal(0, 0.3, (P, I)).astype(f),
         "embed_target.weight": r.normal(0, 0.3, (P, I)).astype(f),
         "attn_layer1.weight": r.uniform(-din ** -0.5, din ** -0.5, (H, din)).astype(f),
         "attn_layer1.bias": r.normal(0, 0.1, H).astype(f),
         "attn_layer2.weight": r.uniform(-H ** -0.5, H ** -0.5, (1, H)).astype(f)}
    if case in ("region", "region_distance"):
        p["embed_region.weight"] = r.normal(0, 0.3, (R, D // 2)).astype(f)
    if case in ("region_distance", "distance"):
        p["dist_layer.weight"] = r.uniform(-0.7, 0.7, (2, 2)).astype(f)
        p["dist_layer.bias"] = r.normal(0, 0.1, 2).astype(f)
    return p


@pytest.mark.parametrize("case,D,H,n,drop", [
    ("basic", 128, 128, 40, 0.5),     # run.py's defaults
    ("basic", 96, 100, 17, 0.5),      # odd sizes: lanes past H / D idle
    ("basic", 64, 128, 9, 0.5),       # hidden > 64 leaves the fused kernels
    ("region", 64, 64, 30, 0.5),
    ("region", 128, 128, 12, 0.5),
    ("region_distance", 64, 48, 25, 0.0),   # no dropout in this model (model.py:268)
    ("region_distance", 128, 128, 8, 0.0),
    ("distance", 64, 64, 20, 0.0),          # NAIS_distance_Embedding (x1000, no dropout)
    ("distance", 128, 100, 11, 0.0),
    # past the general kernels (embed_dim > 128 or hidden > 128): the generic-shape training
    # kernels (nais_train.hip gxt_*, one W1 hidden block at a time in LDS) -- VERDICT r5 Next 7
    ("basic", 192, 192, 40, 0.5),
    ("basic", 256, 64, 33, 0.5),
    ("basic", 64, 320, 21, 0.5),
    ("basic", 150, 130, 37, 0.5),
    ("region", 256, 48, 35, 0.5),
    ("region_distance", 192, 160, 19, 0.0),
    ("distance", 200, 96, 9, 0.0),
])
def test_train_generic_oracle(case, D, H, n, drop, monkeypatch):
    P, R = 3000, 40
    p = _params(case, P, R, D, H, seed=D + H + n)
    r = np.random.default_rng(n)
    pos = r.choice(P, n, replace=False)
    neg = r.choice(np.setdiff1d(np.arange(P), pos), n * 4, replace=False).reshape(n, 4)
    data = np.concatenate([pos.reshape(-1, 1), neg], 1).reshape(-1)
    labels = np.concatenate([np.ones((n, 1)), np.zeros((n, 4))], 1).reshape(-1).astype(np.float32)
    hist = np.repeat(pos.reshape(1, -1), len(data), 0)
    region_of = r.integers(0, R, P)
    hreg, dreg = region_of[hist], region_of[data]
    latlon = r.uniform(0, 0.05 if case != "distance" else 0.003, (len(data), n, 2)).astype(np.float32)
    m = _make(case, p, drop)
    seed = 123456789 + n
    monkeypatch.setattr(torch, "randint", lambda *a, **k: torch.tensor([seed]))
    pred, loss, grads = _step(m, case, hist, data, labels, hreg, dreg, latlon)
    keep = _mask(seed, len(data), n, H, drop) if drop > 0 else None
    kw = {}
    if case in ("region", "region_distance"):
        kw.update(hist_region=hreg, data_region=dreg)
    if case in ("region_distance", "distance"):
        kw["latlon"] = latlon
    if case == "distance":
        kw["dist_scale"] = 1000.0
    ref = train_oracle.train_step(p, hist, data, labels, keep=keep, drop_p=drop, **kw)
    assert np.max(np.abs(pred - ref["pred"])) <= SCORE_ATOL
    assert abs(loss - ref["loss"]) <= 1e-5
    _assert_grads(grads, ref["grads"])


def test_train_generic_loop_with_adagrad_reduces_loss():
    """run.py:153-200's loop shape for NAIS_regionEmbedding at D = H = 128: a few epochs of
    forward / BCELoss / backward / the package's Adagrad over one fixed batch."""
    from poi_recommendation_models_amd.optim import Adagrad
    P, R, n = 2000, 30, 20
    p = _params("region", P, R, 128, 128, seed=5)
    m = _make("region", p, 0.5)
    opt = Adagrad(m.parameters(), lr=0.05)
    r = np.random.default_rng(1)
    pos = r.choice(P, n, replace=False)
    neg = r.choice(np.setdiff1d(np.arange(P), pos), n * 4, replace=False).reshape(n, 4)
    data = np.concatenate([pos.reshape(-1, 1), neg], 1).reshape(-1)
    labels = np.concatenate([np.ones((n, 1)), np.zeros((n, 4))], 1).reshape(-1).astype(np.float32)
    hist = np.repeat(pos.reshape(1, -1), len(data), 0)
    region_of = r.integers(0, R, P)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        pred = m(_t(hist), _t(data), _t(region_of[hist]), _t(region_of[data]))
        loss = m.loss_func(pred, _t(labels))
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    assert losses[-1] < 0.7 * losses[0], losses


def test_train_generic_errors():
    from poi_recommendation_models_amd import model as M
    m = M.NAIS_regionEmbedding(100, 32, 16, 0.5, 5).to(DEV).train()
    with pytest.raises(ValueError):
        m(_t(np.zeros((3, 2), np.int64)), _t(np.arange(3)), None, None)
    m = M.NAIS_basic(100, 264, 16, 0.5).to(DEV).train()   # embed_dim > 256
    with pytest.raises(RuntimeError, match="256"):
        m(_t(np.zeros((3, 2), np.int64)), _t(np.arange(3)))


# ------------------------------------------------ device-side region / distance training (f1 + f2)
def _csr_region(U, P, h_max, seed, h_min=2):
    import scipy.sparse as sp
    r = np.random.default_rng(seed)
    rows, cols = [], []
    for u in range(U):
        h = int(r.integers(h_min, h_max + 1))
        rows += [u] * h
        cols += sorted(r.choice(P, h, replace=False).tolist())
    return sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(U, P))


@pytest.mark.parametrize("case,D,H,drop,wd", [
    ("region", 64, 64, 0.5, 0.0),
    ("region", 128, 128, 0.5, 0.01),
    ("region_distance", 64, 48, 0.0, 0.0),
    ("region_distance", 128, 128, 0.0, 0.01),
    ("distance", 64, 64, 0.0, 0.0),
    ("region", 192, 192, 0.5, 0.01),          # the generic-shape kernels in the fused step
    ("region_distance", 192, 160, 0.0, 0.0),
])
def test_trainer_region_step_oracle(case, D, H, drop, wd):
    """NAISTrainer drives the region / distance variants on the device --
    get_NAIS_batch_region's region ids (batches.py:67-108) and run.py:240-245's target_lat_long built
    from the CSR, region_of and the POI coordinates by nais_make_train_batch + device gathers, one
    nais_train_step_ex per step (forward, BCELoss, backward, torch.optim.Adagrad over every
    parameter, embed_region / dist_layer densely). Two steps against oracle/train_oracle.py carried
    over both: the batch the device drew is read back and fed to the oracle, dropout with the
    device's mask injected; loss within 1e-5, every updated parameter within rtol 1e-4."""
    from poi_recommendation_models_amd.trainer import NAISTrainer
    P, R = 3000, 40
    p = _params(case, P, R, D, H, seed=D + H + 7)
    X = _csr_region(6, P, 40, seed=D + H)
    r = np.random.default_rng(3)
    region_of = r.integers(0, R, P)
    coords = np.stack([40.7 + r.random(P) * 0.05, -74.0 + r.random(P) * 0.05], 1)
    if case == "distance":          # a 10x tighter box keeps the x1000 feature off saturation
        coords = coords.mean(0) + (coords - coords.mean(0)) * 0.1
    m = _make(case, p, drop)
    tr = NAISTrainer(m, X, lr=0.02, weight_decay=wd, region_of=region_of, poi_coords=coords)
    ref = {k: v.copy() for k, v in p.items()}
    st = {k: np.zeros_like(v) for k, v in p.items()}
    slack = {k: np.zeros(v.shape) for k, v in p.items()}
    total = 0.0
    for step, uid in ((1, 2), (2, 5)):
        batch = tr.batch(uid, seed=100 + step)
        hist, data, labels = (t.cpu().numpy() for t in batch[:3])
        b, n = len(data), len(hist)
        kw = {}
        if case != "distance":
            hreg, dreg = batch[3].cpu().numpy(), batch[4].cpu().numpy()
            np.testing.assert_array_equal(hreg, region_of[hist])           # batches.py:96-101
            np.testing.assert_array_equal(dreg, region_of[data])
            kw.update(hist_region=np.repeat(hreg[None], b, 0), data_region=dreg)
        if case != "region":
            ll = batch[-1].cpu().numpy()
            want = np.abs(coords[data][:, None, :] - coords[hist][None, :, :]).astype(np.float32)
            np.testing.assert_array_equal(ll, want)                        # run.py:47-54, 240-245
            kw["latlon"] = ll
        if case == "distance":
            kw["dist_scale"] = 1000.0
        seed = 424242 + step
        tr.step(*batch, dropout_seed=seed)
        loss = tr.finish() - total
        total += loss
        keep = _mask(seed, b, n, H, drop) if drop > 0 else None
        o = train_oracle.train_step(ref, np.repeat(hist[None], b, 0), data, labels, keep=keep,
                                    drop_p=drop, **kw)
        assert abs(loss - o["loss"]) <= 1e-5, (step, loss, o["loss"])
        for k in ref:
            g = o["grads"][k].reshape(ref[k].shape)
            slack[k] += adagrad_slack(g + wd * ref[k], 0.02)
            ref[k], st[k] = train_oracle.adagrad(ref[k], st[k], g, 0.02, step, weight_decay=wd)
    got = dict(m.named_parameters())
    for k in ref:
        assert_params_close(k, got[k].detach().cpu().numpy(), ref[k], slack[k])
    for k, s in tr.optimizer_state().items():
        np.testing.assert_allclose(s["sum"].cpu().numpy(), st[k], rtol=1e-3, atol=1e-9)
    assert not tr._g_small.any() and (tr._g_er is None or not tr._g_er.any())
    assert tr._g_dist is None or not tr._g_dist.any()


@pytest.mark.parametrize("case", ["region", "region_distance"])
def test_trainer_region_epochs_reduce_loss(case):
    """run.py:139-200 / 206-262 as NAISTrainer.epoch: every user's device batch and fused step,
    one host sync per epoch; the summed loss falls."""
    from poi_recommendation_models_amd.trainer import NAISTrainer
    P, R, D, H = 2000, 30, 64, 64
    p = _params(case, P, R, D, H, seed=9)
    for k in ("embed_history.weight", "embed_target.weight", "embed_region.weight"):
        if k in p:
            p[k] = (p[k] * 0.03).astype(np.float32)      # the reference's N(0, 0.01)-like init scale
    X = _csr_region(40, P, 30, seed=4)
    r = np.random.default_rng(5)
    region_of = r.integers(0, R, P)
    coords = np.stack([40.7 + r.random(P) * 0.05, -74.0 + r.random(P) * 0.05], 1)
    m = _make(case, p, 0.5 if case == "region" else 0.0)
    tr = NAISTrainer(m, X, lr=0.05, region_of=region_of, poi_coords=coords)
    losses = [tr.epoch() for _ in range(6)]
    assert all(np.isfinite(losses))
    assert losses[-1] < 0.8 * losses[0], losses
    assert not tr._g_eh.any() and not tr._g_et.any() and not tr._g_small.any() and not tr._g_er.any()


def test_trainer_region_errors():
    from poi_recommendation_models_amd import model as M
    from poi_recommendation_models_amd.trainer import NAISTrainer
    X = _csr_region(3, 100, 5, seed=1)
    m = M.NAIS_regionEmbedding(100, 32, 16, 0.5, 5).to(DEV).train()
    with pytest.raises(ValueError, match="region_of"):
        NAISTrainer(m, X)
    tr = NAISTrainer(m, X, region_of=np.zeros(100, np.int64))
    hist, tgt, lab, hreg, treg = tr.batch(0, seed=1)
    with pytest.raises(TypeError):
        tr.step(hist, tgt, lab)                      # the region ids are required
    tr.step(hist, tgt, lab, hreg, treg)
    assert np.isfinite(tr.finish())
