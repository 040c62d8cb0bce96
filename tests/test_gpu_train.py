"""GPU parity of the NAIS_basic training step through the C-ABI.

* golden: the reference's own autograd gradients (tests/golden/train_step.npz, dropout off)
* oracle: float64 restatement of forward + backward (oracle/train_oracle.py) on seeded
  get_NAIS_batch-shaped batches (batches.py:24-50), with dropout p = 0.5 injected as the device's
  own mask (nais_dropout_mask) so both sides drop the same units
* Adagrad: nais_adagrad / nais_adagrad_rows against torch.optim.Adagrad's update (run.py:89)

Tolerance: predictions within 1e-4 (SCORE_ATOL, the north star's fp32 bar); every gradient within
GRAD_RTOL x max|reference gradient| of that tensor (fp32 MFMA + atomic summation order against a
float64 / CPU-fp32 reference; observed ~1e-6).
"""
import numpy as np
import pytest
import torch

from _helpers import SCORE_ATOL, adagrad_slack, assert_params_close, load_golden
from oracle import train_oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GRAD_RTOL = 1e-4
NAMES = ["embed_history.weight", "embed_target.weight", "attn_layer1.weight", "attn_layer1.bias",
         "attn_layer2.weight"]


def _model(p, beta=0.5, drop_p=0.0):
    from poi_recommendation_models_amd import model as M
    P, D = p["embed_history.weight"].shape
    H = p["attn_layer1.weight"].shape[0]
    m = M.NAIS_basic(P, D, H, beta)
    sd = m.state_dict()
    for k in sd:
        sd[k] = torch.from_numpy(np.ascontiguousarray(p[k]))
    m.load_state_dict(sd)
    m.report_nan = False
    m.drop.p = drop_p
    return m.to(DEV).train()


def _params(P, D, H, seed, emb_std=0.3):
    r = np.random.default_rng(seed)
    f = np.float32
    bound = 1 / np.sqrt(D)
    return {"embed_history.weight": r.normal(0, emb_std, (P, D)).astype(f),
            "embed_target.weight": r.normal(0, emb_std, (P, D)).astype(f),
            "attn_layer1.weight": r.uniform(-bound, bound, (H, D)).astype(f),
            "attn_layer1.bias": r.normal(0, 0.1, H).astype(f),
            "attn_layer2.weight": r.uniform(-1 / np.sqrt(H), 1 / np.sqrt(H), (1, H)).astype(f)}


def _batch(P, n, num_ng, seed):
    """get_NAIS_batch (batches.py:24-50): n positives (shuffled) shared as history by
    n * (1 + num_ng) rows [pos, neg x num_ng] per positive, labels 1 / 0."""
    r = np.random.default_rng(seed)
    pos = r.choice(P, n, replace=False)
    neg = r.choice(np.setdiff1d(np.arange(P), pos), n * num_ng, replace=False).reshape(n, num_ng)
    data = np.concatenate([pos.reshape(-1, 1), neg], 1).reshape(-1)
    labels = np.concatenate([np.ones((n, 1)), np.zeros((n, num_ng))], 1).reshape(-1).astype(np.float32)
    hist = np.repeat(pos.reshape(1, -1), len(data), 0)
    return hist, data, labels


def _step(m, hist, data, labels):
    for q in m.parameters():
        q.grad = None
    pred = m(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV))
    loss = m.loss_func(pred, torch.as_tensor(labels).to(DEV))
    loss.backward()
    grads = {k: q.grad.detach().cpu().numpy() for k, q in m.named_parameters()}
    return pred.detach().cpu().numpy(), float(loss.item()), grads


def _assert_grads(got, ref, rtol=GRAD_RTOL):
    worst = 0.0
    for k in NAMES:
        r = np.asarray(ref[k], np.float64).reshape(got[k].shape)
        scale = max(np.abs(r).max(), 1e-30)
        err = np.abs(got[k] - r).max() / scale
        worst = max(worst, err)
        assert err <= rtol, (k, err)
    return worst


def test_train_step_golden():
    z = load_golden("train_step.npz")
    p = {k[2:]: z[k] for k in z.files if k.startswith("p/")}
    m = _model(p)
    pred, loss, grads = _step(m, z["hist"], z["data"], z["labels"])
    assert np.max(np.abs(pred - z["pred"])) <= SCORE_ATOL
    assert abs(loss - float(z["loss"])) <= 1e-5
    _assert_grads(grads, {k: z["grad/" + k] for k in NAMES})


@pytest.mark.parametrize("D,H", [(8, 8), (16, 16), (32, 20), (32, 48), (64, 64)])
@pytest.mark.parametrize("n", [1, 3, 37, 204])
def test_train_step_oracle_shapes(D, H, n):
    P = 3000
    p = _params(P, D, H, seed=D * 1000 + H + n)
    hist, data, labels = _batch(P, n, 4, seed=n)
    m = _model(p)
    ref = train_oracle.train_step_basic(p, hist, data, labels)
    if n == 1:
        # row 0's target is the whole history: S = 0 -> NaN (model.py:92-95), as the reference;
        # BCELoss then raises (as the reference's CPU BCELoss does) instead of a device assert
        pred = m(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV))
        got = pred.detach().cpu().numpy()
        assert np.isnan(got[0]) and np.isnan(ref["pred"][0])
        assert np.array_equal(np.isnan(got), np.isnan(ref["pred"]))
        assert np.max(np.abs(got[1:] - ref["pred"][1:])) <= SCORE_ATOL
        with pytest.raises(RuntimeError, match="between 0 and 1"):
            m.loss_func(pred, torch.as_tensor(labels).to(DEV))
        return
    pred, loss, grads = _step(m, hist, data, labels)
    assert np.max(np.abs(pred - ref["pred"])) <= SCORE_ATOL
    assert abs(loss - ref["loss"]) <= 1e-5
    _assert_grads(grads, ref["grads"])


def _mask(seed, b, n, H, p):
    from poi_recommendation_models_amd import _capi
    out = torch.empty(b * n * H, dtype=torch.uint8, device=DEV)
    _capi.check(_capi.load().nais_dropout_mask(seed, b, n, H, p, out.data_ptr(),
                                               _capi.stream_handle(torch.device(DEV))),
                "nais_dropout_mask")
    return out.view(b, n, H).cpu().numpy()


def test_dropout_mask_statistics():
    m = _mask(1234, 1020, 204, 64, 0.5)
    assert abs(m.mean() - 0.5) < 2e-3
    assert np.array_equal(m, _mask(1234, 1020, 204, 64, 0.5))           # deterministic per seed
    assert (m != _mask(1235, 1020, 204, 64, 0.5)).mean() > 0.45         # new seed, new mask
    assert _mask(7, 4, 3, 16, 0.0).all() and not _mask(7, 4, 3, 16, 1.0).any()
    assert abs(_mask(9, 256, 64, 64, 0.2).mean() - 0.8) < 3e-3


@pytest.mark.parametrize("D,H,n", [(16, 16, 12), (64, 64, 204)])
def test_train_step_dropout_injected(D, H, n, monkeypatch):
    """Dropout on: the oracle applies the device's mask for the same seed."""
    P = 5000
    p = _params(P, D, H, seed=n)
    hist, data, labels = _batch(P, n, 4, seed=n + 1)
    m = _model(p, drop_p=0.5)
    seed = 987654321
    monkeypatch.setattr(torch, "randint", lambda *a, **k: torch.tensor([seed]))
    pred, loss, grads = _step(m, hist, data, labels)
    keep = _mask(seed, len(data), n, H, 0.5)
    ref = train_oracle.train_step_basic(p, hist, data, labels, keep=keep, drop_p=0.5)
    assert np.max(np.abs(pred - ref["pred"])) <= SCORE_ATOL
    assert abs(loss - ref["loss"]) <= 1e-5
    _assert_grads(grads, ref["grads"])


def test_train_empty_history():
    P, D, H = 100, 16, 16
    m = _model(_params(P, D, H, 3))
    pred, loss, grads = _step(m, np.zeros((5, 0), np.int64), np.arange(5), np.ones(5, np.float32))
    assert np.all(pred == 0.5)
    for k in NAMES:
        assert not np.any(grads[k])


def test_train_per_row_history_raises():
    m = _model(_params(100, 16, 16, 4))
    hist = np.array([[1, 2], [3, 4]])
    with pytest.raises(NotImplementedError):
        m(torch.as_tensor(hist).to(DEV), torch.as_tensor([5, 6]).to(DEV))


@pytest.mark.parametrize("wd,lr_decay", [(0.0, 0.0), (0.01, 0.0), (0.0, 0.1)])
def test_adagrad_matches_torch(wd, lr_decay):
    from poi_recommendation_models_amd import optim
    torch.manual_seed(0)
    shapes = [(3000, 64), (64, 64), (64,), (1, 64)]
    ps = [torch.randn(s) for s in shapes]
    ours = [torch.nn.Parameter(x.clone().to(DEV)) for x in ps]
    ref = [torch.nn.Parameter(x.clone()) for x in ps]
    o = optim.Adagrad(ours, lr=0.05, lr_decay=lr_decay, weight_decay=wd)
    r = torch.optim.Adagrad(ref, lr=0.05, lr_decay=lr_decay, weight_decay=wd, foreach=False)
    for step in range(3):
        gs = [torch.randn(s) for s in shapes]
        for q, g in zip(ours, gs):
            q.grad = g.to(DEV)
        for q, g in zip(ref, gs):
            q.grad = g.clone()
        o.step()
        r.step()
    for a, b in zip(ours, ref):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().numpy(), rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(o.state[a]["sum"].cpu().numpy(), r.state[b]["sum"].numpy(),
                                   rtol=1e-6, atol=1e-7)


def test_adagrad_rows_bit_identical_to_dense():
    """Row update == dense update bit for bit when the gradient is zero outside the rows (the
    embedding grads of a training backward: rows = the batch's history / targets)."""
    from poi_recommendation_models_amd import optim
    P, D, H, n = 4000, 64, 64, 50
    p = _params(P, D, H, 11)
    hist, data, labels = _batch(P, n, 4, seed=5)
    m = _model(p)
    _, _, grads = _step(m, hist, data, labels)      # one set of gradients for both optimizers
    pa = [torch.nn.Parameter(q.detach().clone()) for q in m.parameters()]
    pb = [torch.nn.Parameter(q.detach().clone()) for q in m.parameters()]
    oa = optim.Adagrad(pa, lr=0.01)
    ob = optim.Adagrad(pb, lr=0.01, row_update=False)
    rows = {0: torch.as_tensor(hist[0]).to(DEV), 1: torch.as_tensor(data).to(DEV)}
    for _ in range(3):
        for i, (qa, qb, k) in enumerate(zip(pa, pb, NAMES)):
            g = torch.as_tensor(grads[k]).to(DEV)
            qa.grad, qb.grad = g.clone(), g.clone()
            if i in rows:
                qa._nais_rows = [rows[i], rows[i][:7]]     # repeats: each row updated once
        oa.step()
        ob.step()
    for qa, qb, k in zip(pa, pb, NAMES):
        assert torch.equal(qa, qb), k
        assert torch.equal(oa.state[qa]["sum"], ob.state[qb]["sum"]), k


@pytest.mark.parametrize("D,H,drop", [(32, 32, 0.0), (64, 64, 0.5), (128, 128, 0.5)])
def test_training_loop_matches_oracle(D, H, drop, monkeypatch):
    """Three run.py-style steps of the autograd drop-in (forward, BCELoss, backward with the u
    cache, optim.Adagrad with the sorted-row update) against the float64 oracle carried over the
    same three steps -- drift across drop-in steps is covered, not only one step from equal state.
    Dropout: the oracle applies the device's mask of each step's seed."""
    from poi_recommendation_models_amd import optim
    P, n = 2000, 40
    p = _params(P, D, H, 21)
    m = _model(p, drop_p=drop)
    o = optim.Adagrad(m.parameters(), lr=0.01)
    ref = {k: v.copy() for k, v in p.items()}
    st = {k: np.zeros_like(v) for k, v in p.items()}
    slack = {k: np.zeros(v.shape) for k, v in p.items()}
    first_g = {}
    for step in range(1, 4):
        hist, data, labels = _batch(P, n, 4, seed=100 + step)
        seed = 4242 + step
        monkeypatch.setattr(torch, "randint", lambda *a, **k: torch.tensor([seed]))
        o.zero_grad()
        pred, loss, _ = _step(m, hist, data, labels)
        o.step()
        keep = _mask(seed, len(data), n, H, drop) if drop else None
        r = train_oracle.train_step_basic(ref, hist, data, labels, keep=keep, drop_p=drop)
        assert abs(loss - r["loss"]) <= 1e-5
        for k in NAMES:
            g = r["grads"][k].reshape(ref[k].shape)
            slack[k] += adagrad_slack(g, 0.01)
            first_g.setdefault(k, g)
            ref[k], st[k] = train_oracle.adagrad(ref[k], st[k], g, 0.01, step)
    # Adagrad divides by sqrt(sum g^2): an element whose gradient is small against the tensor's
    # largest amplifies the gradient's fp32 rounding (a sign flip at the first step moves it 2 lr);
    # each element may differ by its own accumulated slack only (assert_params_close prints them).
    for k, q in m.named_parameters():
        assert_params_close(k, q.detach().cpu().numpy(), ref[k], slack[k], g=first_g[k])


# ------------------------------------------------------------------ fused step + device batches
def _csr(U, P, h_max, seed, h_min=1):
    import scipy.sparse as sp
    r = np.random.default_rng(seed)
    rows, cols = [], []
    for u in range(U):
        h = int(r.integers(h_min, h_max + 1))
        rows += [u] * h
        cols += sorted(r.choice(P, h, replace=False).tolist())
    return sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(U, P))


def _trainer(m, X, **kw):
    from poi_recommendation_models_amd.trainer import NAISTrainer
    return NAISTrainer(m, X, **kw)


def test_make_batch_properties():
    P, D, H = 3000, 16, 16
    X = _csr(20, P, 60, seed=3)
    tr = _trainer(_model(_params(P, D, H, 1)), X)
    seen = set()
    for u in range(20):
        pos = X.getrow(u).indices
        n = len(pos)
        hist, tgt, lab = [t.cpu().numpy() for t in tr.batch(u, seed=100 + u)]
        assert sorted(hist.tolist()) == sorted(pos.tolist())               # a permutation
        rows = tgt.reshape(n, 5)
        assert np.array_equal(rows[:, 0], hist)                              # batches.py:38-40
        neg = rows[:, 1:].reshape(-1)
        assert len(set(neg.tolist())) == 4 * n and not set(neg.tolist()) & set(pos.tolist())
        assert neg.min() >= 0 and neg.max() < P
        assert np.array_equal(lab.reshape(n, 5), np.repeat([[1, 0, 0, 0, 0]], n, 0))
        seen.add(tuple(tr.batch(u, seed=7)[1].cpu().numpy()[:10].tolist()))
    h1 = tr.batch(0, seed=1)[1].cpu().numpy().copy()
    h2 = tr.batch(0, seed=2)[1].cpu().numpy()
    assert not np.array_equal(h1, h2)


def test_make_batch_negatives_uniform():
    """Every non-positive POI is drawn with probability n*ng/(P-n) (shuffle-and-slice)."""
    P, n, trials = 64, 6, 3000
    import scipy.sparse as sp
    pos = np.array([3, 10, 11, 40, 41, 63])
    X = sp.csr_matrix((np.ones(n), (np.zeros(n, int), pos)), shape=(1, P))
    tr = _trainer(_model(_params(P, 8, 8, 1)), X)
    cnt = np.zeros(P)
    first = np.zeros(n)
    for s in range(trials):
        hist, tgt, _ = tr.batch(0, seed=s)
        t = tgt.cpu().numpy().reshape(n, 5)
        np.add.at(cnt, t[:, 1:].reshape(-1), 1)
        first[np.searchsorted(pos, hist.cpu().numpy()[0])] += 1
    assert cnt[pos].sum() == 0
    expect = trials * n * 4 / (P - n)
    free = np.setdiff1d(np.arange(P), pos)
    assert np.abs(cnt[free] / expect - 1).max() < 0.12, cnt[free] / expect
    assert np.abs(first / (trials / n) - 1).max() < 0.15, first      # shuffled history order


@pytest.mark.parametrize("D,H", [(64, 64), (128, 128)])   # fused MFMA kernels / general kernels
def test_fused_step_matches_dropin(D, H):
    """NAISTrainer.step == forward + BCELoss + backward + optim.Adagrad (same batch, same dropout).

    Each step starts both sides from identical parameters and Adagrad sums (copied from the fused
    side), so summation-order noise of one step cannot compound over the next. Adagrad's update is
    ill-conditioned where the gradient is ~0 (the first step moves by lr * sign(g)), so elements
    whose gradient is below 1e-4 of the tensor's largest are left out of the parameter check; the
    sums (g^2) are checked everywhere."""
    from poi_recommendation_models_amd import optim
    P, n = 3000, 60
    p = _params(P, D, H, 5)
    X = _csr(4, P, 80, seed=9)
    ma, mb = _model(p, drop_p=0.5), _model(p, drop_p=0.5)
    tr = _trainer(ma, X, lr=0.01)
    ob = optim.Adagrad(mb.parameters(), lr=0.01)
    names = [k for k, _ in ma.named_parameters()]
    for step in range(3):
        with torch.no_grad():
            for (k, a), b in zip(ma.named_parameters(), mb.parameters()):
                b.copy_(a)
                ob.state[b]["sum"].copy_(tr.sums[k])
        hist, data, labels = _batch(P, n, 4, seed=step)
        tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV),
                torch.as_tensor(labels).to(DEV), dropout_seed=1000 + step)
        ob.zero_grad()
        torch_randint = torch.randint
        torch.randint = lambda *a, **k: torch.tensor([1000 + step])
        try:
            pred = mb(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV))
        finally:
            torch.randint = torch_randint
        mb.loss_func(pred, torch.as_tensor(labels).to(DEV)).backward()
        grads = {k: (b.grad.detach().cpu().numpy().copy() if b.grad is not None else None)
                 for k, b in zip(names, mb.parameters())}
        ob.step()
        for (k, a), b in zip(ma.named_parameters(), mb.parameters()):
            g = grads[k]
            sl = 0.0 if g is None else adagrad_slack(g, 0.01)
            assert_params_close(f"step {step} {k}", a.detach().cpu().numpy(), b.detach().cpu().numpy(),
                                sl, rtol=1e-5, atol=1e-6, g=g)
            np.testing.assert_allclose(tr.sums[k].cpu().numpy(), ob.state[b]["sum"].cpu().numpy(),
                                       rtol=1e-3, atol=1e-9)
    assert tr.finish() > 0


@pytest.mark.parametrize("split", ["1", "0"])
def test_general_kernels_short_slice_split_config3(split, monkeypatch):
    """Config-3 shape at the reference's D = H = 128 (1,020 rows x 204 history items, run.py:86,
    837-838): the general kernels run the six full 32-item slices with 12-row workgroups and the
    12-item last slice as a second launch of 4-row workgroups (g_split_slices, nais_train.hip:
    85 x 7 = 595 units would take 3 rounds over 256 CUs, 510 take 2). Gradients and loss equal the
    float64 oracle's with the split on and off (NAIS_GM_TAIL=0), dropout off."""
    monkeypatch.setenv("NAIS_GM_TAIL", split)
    P, D, H, n = 3000, 128, 128, 204
    p = _params(P, D, H, 12)
    hist, data, labels = _batch(P, n, 4, seed=3)
    assert hist.shape == (1020, 204)
    pred, loss, grads = _step(_model(p), hist, data, labels)
    r = train_oracle.train_step_basic(p, hist, data, labels)
    assert np.abs(pred - r["pred"]).max() <= SCORE_ATOL
    assert abs(loss - r["loss"]) <= 1e-5
    _assert_grads(grads, r["grads"])


@pytest.mark.parametrize("wd", [0.0, 0.01])
@pytest.mark.parametrize("D,H", [(32, 48), (128, 128), (80, 72)])
def test_fused_step_oracle(wd, D, H):
    P, n = 2000, 40
    p = _params(P, D, H, 6)
    X = _csr(2, P, 10, seed=1)
    m = _model(p)
    tr = _trainer(m, X, lr=0.02, weight_decay=wd)
    hist, data, labels = _batch(P, n, 4, seed=11)
    tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV), torch.as_tensor(labels).to(DEV))
    loss = tr.finish()
    r = train_oracle.train_step_basic(p, hist, data, labels)
    assert abs(loss - r["loss"]) <= 1e-5
    for k, q in m.named_parameters():
        g = r["grads"][k].reshape(p[k].shape)
        want, _ = train_oracle.adagrad(p[k], np.zeros_like(p[k]), g, 0.02, 1, weight_decay=wd)
        assert_params_close(k, q.detach().cpu().numpy(), want, adagrad_slack(g + wd * p[k], 0.02),
                            g=g + wd * p[k])


def test_fused_step_config3_split_vs_oracle():
    """NAISTrainer.step at the config-3 shape, D = H = 128 (the fused step's u cache and the split
    general kernels together): loss and the Adagrad-updated parameters against the oracle."""
    P, D, H, n = 3000, 128, 128, 204
    p = _params(P, D, H, 13)
    X = _csr(2, P, 10, seed=4)
    m = _model(p)
    tr = _trainer(m, X, lr=0.02)
    hist, data, labels = _batch(P, n, 4, seed=5)
    tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV), torch.as_tensor(labels).to(DEV))
    loss = tr.finish()
    r = train_oracle.train_step_basic(p, hist, data, labels)
    assert abs(loss - r["loss"]) <= 1e-5
    for k, q in m.named_parameters():
        g = r["grads"][k].reshape(p[k].shape)
        want, _ = train_oracle.adagrad(p[k], np.zeros_like(p[k]), g, 0.02, 1)
        assert_params_close(k, q.detach().cpu().numpy(), want, adagrad_slack(g, 0.02), g=g)


@pytest.mark.parametrize("D,H", [(16, 16), (128, 128)])
def test_fused_nan_batch_skips_update(D, H):
    P = 500
    p = _params(P, D, H, 8)
    X = _csr(2, P, 5, seed=2)
    m = _model(p)
    tr = _trainer(m, X)
    before = {k: q.detach().clone() for k, q in m.named_parameters()}
    hist = torch.tensor([7], device=DEV)
    data = torch.tensor([7, 1, 2, 3, 4], device=DEV)    # row 0: target == the whole history
    labels = torch.tensor([1., 0, 0, 0, 0], device=DEV)
    tr.step(hist, data, labels)
    with pytest.raises(RuntimeError, match="between 0 and 1"):
        tr.finish()
    for k, q in m.named_parameters():
        assert torch.equal(q, before[k]), k
    assert not tr._g_eh.any() and not tr._g_et.any() and not tr._g_small.any()


def test_trainer_epochs_reduce_loss():
    P, D, H = 2000, 32, 32
    X = _csr(40, P, 30, seed=4, h_min=2)   # a 1-item history is the reference's NaN batch
    m = _model(_params(P, D, H, 12, emb_std=0.01), drop_p=0.5)
    tr = _trainer(m, X, lr=0.05)
    losses = [tr.epoch() for _ in range(6)]
    assert all(np.isfinite(losses))
    assert losses[-1] < 0.8 * losses[0], losses
    assert not tr._g_eh.any() and not tr._g_et.any() and not tr._g_small.any()  # scratch stays zero


@pytest.mark.parametrize("wd", [0.0, 0.01])
@pytest.mark.parametrize("D,H", [(64, 64), (128, 128)])
def test_fused_step_config3_full_catalog(D, H, wd):
    """config 3 at its own size -- P = 100k POIs, one get_NAIS_batch batch of
    1,020 rows x 204 history items (batches.py:24-50), dropout 0.5 with the device's mask injected
    into the oracle. weight_decay != 0 runs the dense Adagrad pass over both 100k-row tables
    (every row moves); weight_decay = 0 the row-stamped update of the touched rows only. Loss and
    every updated parameter (all 100k rows) against oracle/train_oracle.py, two steps."""
    P, n = 100_000, 204
    p = _params(P, D, H, 31)
    X = _csr(2, P, 10, seed=6)
    m = _model(p, drop_p=0.5)
    tr = _trainer(m, X, lr=0.02, weight_decay=wd)
    ref = {k: v.copy() for k, v in p.items()}
    st = {k: np.zeros_like(v) for k, v in ref.items()}
    slack = {k: np.zeros(v.shape) for k, v in ref.items()}
    first_g = {}
    total = 0.0
    for step in (1, 2):
        hist, data, labels = _batch(P, n, 4, seed=40 + step)
        assert hist.shape == (1020, 204)
        seed = 777 + step
        tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV),
                torch.as_tensor(labels).to(DEV), dropout_seed=seed)
        loss = tr.finish() - total      # finish() returns the running sum of run.py:107
        total += loss
        keep = _mask(seed, len(data), n, H, 0.5)
        r = train_oracle.train_step_basic(ref, hist, data, labels, keep=keep, drop_p=0.5)
        assert abs(loss - r["loss"]) <= 1e-5, (step, loss, r["loss"])
        for k in NAMES:
            g = r["grads"][k].reshape(ref[k].shape)
            slack[k] += adagrad_slack(g + wd * ref[k], 0.02)      # the gradient Adagrad sees
            first_g.setdefault(k, g + wd * ref[k])
            ref[k], st[k] = train_oracle.adagrad(ref[k], st[k], g, 0.02, step, weight_decay=wd)
    touched = np.zeros(P, bool)
    for k, q in m.named_parameters():
        got = q.detach().cpu().numpy()
        assert_params_close(k, got, ref[k], slack[k], g=first_g[k])
        if k.startswith("embed") and wd == 0.0:   # untouched rows: bit-identical to the start
            touched[:] = False
            for step in (1, 2):
                hist, data, _ = _batch(P, n, 4, seed=40 + step)
                touched[hist[0]] = True
                touched[data] = True
            assert np.array_equal(got[~touched], p[k][~touched]), k
