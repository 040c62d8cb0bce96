"""Any embed_size / hidden_size at the drop-in (the reference builds
Linear(embed_size, hidden_size) for any sizes, /root/reference/model.py:9-38, 100-229, 306-329).

The scoring / forward kernels are compiled for embedding widths 8, 16, 32, 64, 128; other widths
run from zero-padded copies (model._NAISDevice._score_params: each half of the region variants'
[history | region] rows padded separately, attn_layer1's columns moved to the padded positions,
the distance columns after them) -- exact, a padded dimension adds 0 * x = 0. Training takes the
parameters as they are (its kernels are runtime-shaped up to 128). Checked against the numpy
oracle (oracle/nais_oracle.py) at the north star's tolerance (scores within 1e-4, tie-aware
top-50) on both catalog routes, the forward, and one training step at (100, 100)."""
import numpy as np
import pytest
import torch

from _helpers import SCORE_ATOL, assert_topk_equivalent
from oracle import nais_oracle, train_oracle
from test_gpu_parity import TIE_ULPS, _catalog_vs_oracle, _model, _t

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SHAPES = [("basic", 12, 20), ("basic", 100, 100), ("basic", 40, 72), ("region", 12, 20),
          ("region", 100, 100), ("region_distance", 100, 100), ("region_distance", 12, 20),
          ("distance", 100, 100), ("distance", 12, 20)]


@pytest.mark.parametrize("strategy", ["direct", "pairs"])
@pytest.mark.parametrize("precision", ["fp16x6", "fp32", "fp16x3"])
@pytest.mark.parametrize("variant,D,H", SHAPES)
def test_catalog_any_width_vs_oracle(variant, D, H, precision, strategy):
    _catalog_vs_oracle(variant, D, H, precision, strategy)


@pytest.mark.parametrize("variant,D,H", SHAPES)
def test_forward_any_width_vs_oracle(variant, D, H):
    from poi_recommendation_models_amd.synthetic import init_nais_params
    P, R, b, n = 700, 30, 45, 13
    p = init_nais_params(P, D, H, seed=D + 7 * H, emb_std=0.3, variant=variant, num_regions=R,
                         bias_std=0.1)
    m = _model(variant, p)
    rng = np.random.default_rng(D * H)
    hist = rng.integers(0, P, (b, n)).astype(np.int64)
    tgt = rng.integers(0, P, b).astype(np.int64)
    tgt[4] = hist[4, 2]                                  # a masked term
    hreg, treg = rng.integers(0, R, (b, n)), rng.integers(0, R, b)
    ll = rng.uniform(0, 0.02, (b, n, 2)).astype(np.float32)
    if variant == "basic":
        got = m(_t(hist), _t(tgt))
        ref = nais_oracle.attention_basic(p, hist, tgt)
    elif variant == "region":
        got = m(_t(hist), _t(tgt), _t(hreg), _t(treg))
        ref = nais_oracle.attention_region(p, hist, tgt, hreg, treg)
    elif variant == "region_distance":
        got = m(_t(hist), _t(tgt), _t(hreg), _t(treg), _t(ll))
        ref = nais_oracle.attention_region_distance(p, hist, tgt, hreg, treg, ll)
    else:
        got = m(_t(hist), _t(tgt), None, None, _t(ll))
        ref = nais_oracle.attention_distance(p, hist, tgt, ll)
    ref = nais_oracle._sigmoid(ref)
    got = got.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.max(np.abs(got[ok] - ref[ok])) <= SCORE_ATOL, np.max(np.abs(got[ok] - ref[ok]))


# hidden_size > 128 (up to 256): the x6n kernel in four 64-hidden units per item (fp16x6, the
# drop-in default) and the forward kernel in hidden passes of 128
WIDE_H = [("basic", 64, 200), ("basic", 128, 200), ("basic", 32, 256), ("region", 64, 160),
          ("region_distance", 64, 200), ("distance", 128, 144)]


@pytest.mark.parametrize("strategy", ["direct", "pairs"])
@pytest.mark.parametrize("variant,D,H", WIDE_H)
def test_catalog_hidden_above_128_vs_oracle(variant, D, H, strategy):
    _catalog_vs_oracle(variant, D, H, "fp16x6", strategy)


@pytest.mark.parametrize("variant,D,H", WIDE_H + [("basic", 100, 200)])
def test_forward_hidden_above_128_vs_oracle(variant, D, H):
    test_forward_any_width_vs_oracle(variant, D, H)


@pytest.mark.parametrize("strategy", ["direct", "pairs"])
@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
def test_hidden_above_128_other_precisions_vs_oracle(precision, strategy):
    """fp32 / fp16x3 catalog kernels stop at hidden 128; above it those precisions take the
    generic-shape kernels (exact fp32, nais_generic.hip) instead of raising (round 5)."""
    _catalog_vs_oracle("basic", 64, 200, precision, strategy)


def test_padded_copies_follow_parameter_updates():
    """The padded copies are rebuilt when a parameter changes in place (an optimizer step)."""
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_catalog
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    P, D, H = 900, 100, 36
    data = make_checkins(3, P, 40, seed=5)
    p = init_nais_params(P, D, H, seed=3, emb_std=0.3, bias_std=0.1)
    m = _model("basic", p, precision="fp16x6")
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, torch.device(DEV))
    a = score_catalog(m, csr, range(3)).cpu().numpy()
    with torch.no_grad():
        m.embed_target.weight.mul_(0.5)
        m.attn_layer1.weight[:, 7] += 0.25
    b = score_catalog(m, csr, range(3)).cpu().numpy()
    q = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    for u in range(3):
        cand, ref = nais_oracle.catalog_scores_basic(q, data.history(u), P)
        assert np.max(np.abs(b[u][cand] - ref)) <= SCORE_ATOL
        assert np.max(np.abs(a[u][cand] - ref)) > 1e-3          # the old copies would fail


def test_width_above_256_raises():
    from poi_recommendation_models_amd.synthetic import init_nais_params
    p = init_nais_params(50, 264, 16, seed=1)
    m = _model("basic", p)
    with pytest.raises(RuntimeError, match="256"):
        m(_t(np.zeros((2, 3), np.int64)), _t(np.zeros(2, np.int64)))


# Shapes past the tuned kernels' tiles (VERDICT r5 Next 7; model.py:9-38 builds Linear(embed_size,
# hidden_size) for any sizes): embed_size above 128 (up to 256), hidden above 256, odd widths --
# the generic-shape kernels (nais_generic.hip: exact fp32, one W1 hidden block at a time in LDS)
BIG = [("basic", 192, 192), ("basic", 256, 64), ("basic", 64, 320), ("basic", 129, 40),
       ("basic", 100, 300), ("region", 192, 192), ("region_distance", 192, 160),
       ("distance", 200, 96), ("region", 256, 48)]


@pytest.mark.parametrize("strategy", ["direct", "pairs"])
@pytest.mark.parametrize("variant,D,H", BIG)
def test_catalog_big_shapes_vs_oracle(variant, D, H, strategy):
    _catalog_vs_oracle(variant, D, H, "fp16x6", strategy)


@pytest.mark.parametrize("variant,D,H", BIG)
def test_forward_big_shapes_vs_oracle(variant, D, H):
    test_forward_any_width_vs_oracle(variant, D, H)


@pytest.mark.parametrize("variant,D,H", [("basic", 192, 192), ("region_distance", 192, 160),
                                         ("basic", 64, 320)])
def test_forward_big_shapes_shared_history(variant, D, H):
    """A history shared by every row (stride-0 rows, as the eval chunks of validation.py:14-22
    build them with repeat): the generic forward's shared-chunk mode."""
    from poi_recommendation_models_amd.synthetic import init_nais_params
    P, R, b, n = 900, 30, 70, 45
    p = init_nais_params(P, D, H, seed=D + 3 * H, emb_std=0.3, variant=variant, num_regions=R,
                         bias_std=0.1)
    m = _model(variant, p)
    rng = np.random.default_rng(D + H)
    h1 = rng.choice(P, n, replace=False).astype(np.int64)
    tgt = rng.integers(0, P, b).astype(np.int64)
    tgt[3] = h1[5]                                        # a masked term
    r1 = rng.integers(0, R, n)
    hist = np.broadcast_to(h1, (b, n))
    hreg = np.broadcast_to(r1, (b, n))
    treg = rng.integers(0, R, b)
    ll = rng.uniform(0, 0.02, (b, n, 2)).astype(np.float32)
    th = torch.as_tensor(h1, device=DEV).expand(b, n)
    assert th.stride(0) == 0
    if variant == "basic":
        got = m(th, _t(tgt))
        ref = nais_oracle.attention_basic(p, hist, tgt)
    else:
        thr = torch.as_tensor(r1, device=DEV).expand(b, n)
        got = m(th, _t(tgt), thr, _t(treg), _t(ll))
        ref = nais_oracle.attention_region_distance(p, hist, tgt, hreg, treg, ll)
    ref = nais_oracle._sigmoid(ref)
    got = got.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.max(np.abs(got[ok] - ref[ok])) <= SCORE_ATOL, np.max(np.abs(got[ok] - ref[ok]))


def test_training_step_100x100_vs_oracle():
    """run.py:101-109 at embed_size = hidden_size = 100: forward (dropout off), BCELoss, backward
    and one optim.Adagrad step against the float64 oracle (oracle/train_oracle.py)."""
    from poi_recommendation_models_amd import optim
    from test_gpu_train import _assert_grads, _batch, _params, _step
    from test_gpu_train import _model as _train_model
    from _helpers import adagrad_slack, assert_params_close
    P, D, H, n = 2000, 100, 100, 37
    p = _params(P, D, H, seed=100)
    m = _train_model(p)
    hist, data, labels = _batch(P, n, 4, seed=9)
    pred, loss, grads = _step(m, hist, data, labels)
    r = train_oracle.train_step_basic(p, hist, data, labels)
    assert np.max(np.abs(pred - r["pred"])) <= SCORE_ATOL
    assert abs(loss - r["loss"]) <= 1e-5
    _assert_grads(grads, r["grads"])
    o = optim.Adagrad(m.parameters(), lr=0.01)
    o.step()
    for k, q in m.named_parameters():
        g = r["grads"][k].reshape(p[k].shape)
        want, _ = train_oracle.adagrad(p[k], np.zeros_like(p[k]), g, 0.01, 1)
        assert_params_close(k, q.detach().cpu().numpy(), want, adagrad_slack(g, 0.01), g=g)
    # eval-mode scoring of the trained module runs from the padded copies of the new parameters
    m.eval()
    h0 = hist[0][:5]
    got = m(_t(np.tile(h0, (6, 1))), _t(np.arange(6))).cpu().numpy()
    q = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    ref, _ = nais_oracle.forward_basic(q, np.tile(h0, (6, 1)), np.arange(6))
    assert np.max(np.abs(got - ref)) <= SCORE_ATOL


@pytest.mark.parametrize("writer", ["adagrad", "trainer"])
def test_padded_copies_follow_native_optimizer_writes(writer):
    """the padded copies for an embed width off the native set (D = 100) are
    keyed on the parameters' version counters; optim.Adagrad and NAISTrainer write the parameters
    through raw device pointers and must bump those counters. The run.py flow -- score, train,
    score again (validation inside the epoch loop, run.py:112-116) -- must score the NEW
    parameters: checked against the numpy oracle after each writer."""
    from poi_recommendation_models_amd import optim
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_catalog
    from poi_recommendation_models_amd.synthetic import make_checkins
    from test_gpu_train import _batch, _csr, _params, _trainer
    from test_gpu_train import _model as _train_model
    P, D, H = 1500, 100, 48
    data = make_checkins(3, P, 30, seed=8)
    m = _train_model(_params(P, D, H, seed=21))
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, torch.device(DEV))

    def check(tag):
        m.eval()
        got = score_catalog(m, csr, range(3)).cpu().numpy()
        q = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
        worst = 0.0
        for u in range(3):
            cand, ref = nais_oracle.catalog_scores_basic(q, data.history(u), P)
            worst = max(worst, float(np.max(np.abs(got[u][cand] - ref))))
        assert worst <= SCORE_ATOL, (tag, worst)
        return q

    before = check("before")
    hist, tgt, labels = _batch(P, 40, 4, seed=3)
    m.train()
    if writer == "adagrad":
        o = optim.Adagrad(m.parameters(), lr=0.05)
        for q in m.parameters():
            q.grad = None
        pred = m(torch.as_tensor(hist).to(DEV), torch.as_tensor(tgt).to(DEV))
        m.loss_func(pred, torch.as_tensor(labels).to(DEV)).backward()
        o.step()
    else:
        tr = _trainer(m, _csr(3, P, 30, seed=4), lr=0.05)
        tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(tgt).to(DEV),
                torch.as_tensor(labels).to(DEV))
        tr.finish()
    after = check("after " + writer)
    moved = max(float(np.max(np.abs(after[k] - before[k]))) for k in before)
    assert moved > 1e-3                       # the parameters did change


@pytest.mark.parametrize("D,H,drop", [(192, 192, 0.5), (64, 320, 0.0), (256, 96, 0.5)])
def test_fused_step_big_shapes_vs_oracle(D, H, drop):
    """run.py:91-109 (the fused NAISTrainer step: forward, BCELoss, backward, Adagrad) at embed /
    hidden sizes past the general kernels (the generic-shape training kernels), two steps of a
    config-3-like batch (204 positives x 5) against the float64 oracle, dropout mask injected."""
    from test_gpu_train import _batch, _csr, _mask, _params, _trainer
    from test_gpu_train import _model as _train_model
    from _helpers import adagrad_slack, assert_params_close
    P, n = 3000, 204
    p = _params(P, D, H, seed=D + H)
    m = _train_model(p, drop_p=drop)
    tr = _trainer(m, _csr(2, P, 10, seed=4), lr=0.02)
    ref = {k: v.copy() for k, v in p.items()}
    st = {k: np.zeros_like(v) for k, v in p.items()}
    slack = {k: np.zeros(v.shape) for k, v in p.items()}
    first_g, total = {}, 0.0
    for step in (1, 2):
        hist, data, labels = _batch(P, n, 4, seed=60 + step)
        seed = 5150 + step
        tr.step(torch.as_tensor(hist).to(DEV), torch.as_tensor(data).to(DEV),
                torch.as_tensor(labels).to(DEV), dropout_seed=seed)
        loss = tr.finish() - total
        total += loss
        keep = _mask(seed, len(data), n, H, drop) if drop else None
        r = train_oracle.train_step_basic(ref, hist, data, labels, keep=keep, drop_p=drop)
        assert abs(loss - r["loss"]) <= 1e-5, (step, loss, r["loss"])
        for k in ref:
            g = r["grads"][k].reshape(ref[k].shape)
            slack[k] += adagrad_slack(g, 0.02)
            first_g.setdefault(k, g)
            ref[k], st[k] = train_oracle.adagrad(ref[k], st[k], g, 0.02, step)
    for k, q in m.named_parameters():
        assert_params_close(k, q.detach().cpu().numpy(), ref[k], slack[k], g=first_g[k])
