"""GPU: nais_topk_rows (the torch.topk of validation.py:26-27) on crafted score rows, against a
numpy restatement of the build's total order: candidates are entries >= 0 (history POIs are
scored -1), ranked by (score desc, POI id asc) with NaN above +inf; rows with fewer than k
candidates are padded with id -1 / NaN and counted. Exact (bit-equal ids and scores).

Covers the select's early exit (the keys at or above the selected digit prefix must fit the
4096-key collect buffer), rows that force all eight digits (long runs of equal scores), clustered
rows (one dominant histogram bin), NaN, -1 entries, unaligned rows (scalar load path), k = 1 / 50
/ 1024 and short rows."""
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_topk(row, k):
    c = np.nonzero(~(row < 0))[0]           # NaN is a candidate (NaN < 0 is False)
    v = row[c].astype(np.float32)
    nan = np.isnan(v)
    # order: NaN first (by id), then score desc, then id asc
    o = np.lexsort((c, -np.where(nan, 0, v).astype(np.float64), ~nan))
    o = o[:k]
    ids = np.full(k, -1, np.int64)
    sc = np.full(k, np.nan, np.float32)
    ids[:len(o)] = c[o]
    sc[:len(o)] = v[o]
    return ids, sc, len(c) < k


def _run(rows, k, ld=None):
    from poi_recommendation_models_amd import _capi
    n, P = rows.shape
    ld = ld or P
    buf = np.full((n, ld), -1.0, np.float32)
    buf[:, :P] = rows
    t = torch.from_numpy(buf).to(DEV)
    ids = torch.empty(n, k, dtype=torch.int32, device=DEV)
    sc = torch.empty(n, k, dtype=torch.float32, device=DEV)
    short = torch.zeros(1, dtype=torch.int32, device=DEV)
    _capi.check(_capi.load().nais_topk_rows(t.data_ptr(), ld, P, n, k, ids.data_ptr(), sc.data_ptr(),
                                            short.data_ptr(), _capi.stream_handle(torch.device(DEV))),
                "nais_topk_rows")
    torch.cuda.synchronize()
    return ids.cpu().numpy(), sc.cpu().numpy(), int(short.item())


def _check(rows, k, ld=None):
    ids, sc, short = _run(rows, k, ld)
    nshort = 0
    for r in range(rows.shape[0]):
        rid, rsc, s = _ref_topk(rows[r], k)
        nshort += s
        np.testing.assert_array_equal(ids[r], rid, err_msg=f"row {r}")
        np.testing.assert_array_equal(sc[r].view(np.int32)[~np.isnan(rsc)], rsc.view(np.int32)[~np.isnan(rsc)])
        assert np.all(np.isnan(sc[r][np.isnan(rsc)]))
    assert short == nshort


def _rows(kind, n, P, rng):
    if kind == "uniform":
        x = rng.random((n, P), dtype=np.float32)
    elif kind == "sigmoid":                       # spread like real scores
        x = (1 / (1 + np.exp(-rng.normal(0, 3, (n, P))))).astype(np.float32)
    elif kind == "quantized":                     # ties straddling rank k
        x = (np.round(rng.random((n, P)) * 200) / 200).astype(np.float32)
    elif kind == "equal":                         # one score: only the id digits separate
        x = np.full((n, P), 0.73, np.float32)
    elif kind == "clustered":                     # one dominant bin + a few high outliers
        x = np.full((n, P), 0.5, np.float32) + rng.random((n, P), dtype=np.float32) * 1e-6
        x[:, rng.choice(P, 20, replace=False)] = 0.9
    elif kind == "narrow":                        # 10k distinct ids at one score in the top bin
        x = rng.random((n, P), dtype=np.float32) * 0.5
        x[:, rng.choice(P, 10000, replace=False)] = 0.99
    else:
        raise ValueError(kind)
    hist = rng.random((n, P)) < 0.002
    x[hist] = -1.0
    return x


@pytest.mark.parametrize("kind", ["uniform", "sigmoid", "quantized", "equal", "clustered", "narrow"])
@pytest.mark.parametrize("k", [1, 50, 1024])
def test_topk_rows_kinds(kind, k):
    rng = np.random.default_rng(zlib.crc32(f"{kind}/{k}".encode()))
    _check(_rows(kind, 6, 100003, rng), k)


@pytest.mark.parametrize("ld_pad", [1, 3])
def test_topk_rows_unaligned(ld_pad):
    """Rows start off a 16-byte boundary (score_ld not a multiple of 4): the scalar path."""
    rng = np.random.default_rng(ld_pad)
    rows = _rows("quantized", 5, 20001, rng)
    _check(rows, 50, ld=20001 + ld_pad)


def test_topk_rows_nan_and_short():
    rng = np.random.default_rng(7)
    rows = _rows("uniform", 4, 3000, rng)
    rows[0, [5, 17, 2999]] = np.nan
    rows[1, :] = -1.0
    rows[1, [3, 9]] = [0.2, 0.2]                   # 2 candidates < k
    rows[2, :2990] = -1.0                          # 10 candidates
    _check(rows, 50)


def test_topk_rows_small_p():
    rng = np.random.default_rng(11)
    for P in (1, 2, 5, 63, 64, 65, 4097):
        _check(_rows("uniform", 3, P, rng), min(50, P))


# ---- nais_topk_blend_rows (run.py:537-539 with normalize run.py:55-59): the f64 blended key ----
def _ref_blend_topk(s, g, gm, alpha, k):
    """The kernel's total order on f64(f32((1 - alpha) * s)) + alpha * (g / gm): candidates s >= 0
    (or NaN), NaN first, then blended desc, then id asc; scores reported as f32."""
    c = np.nonzero(~(s < 0))[0]
    t = (s[c] * np.float32(1.0 - alpha)).astype(np.float64)
    gn = g[c] / gm if gm != 0.0 else g[c]
    v = t + alpha * gn
    nan = np.isnan(v)
    o = np.lexsort((c, -np.where(nan, 0, v), ~nan))[:k]
    ids = np.full(k, -1, np.int64)
    sc = np.full(k, np.nan, np.float32)
    ids[:len(o)] = c[o]
    sc[:len(o)] = v[o].astype(np.float32)
    return ids, sc, len(c) < k


def _check_blend(s, g, k, alpha=0.2):
    from poi_recommendation_models_amd import _capi
    n, P = s.shape
    gmv = np.array([max([x for x in g[r][~(s[r] < 0)]] + [0.0]) for r in range(n)], np.float64)
    ts, tg = torch.from_numpy(s).to(DEV), torch.from_numpy(g).to(DEV)
    tm = torch.from_numpy(gmv.view(np.int64)).to(DEV)
    ids = torch.empty(n, k, dtype=torch.int32, device=DEV)
    sc = torch.empty(n, k, dtype=torch.float32, device=DEV)
    short = torch.zeros(1, dtype=torch.int32, device=DEV)
    _capi.check(_capi.load().nais_topk_blend_rows(
        ts.data_ptr(), P, tg.data_ptr(), P, tm.data_ptr(), P, n, k, alpha, ids.data_ptr(),
        sc.data_ptr(), short.data_ptr(), _capi.stream_handle(torch.device(DEV))), "nais_topk_blend_rows")
    torch.cuda.synchronize()
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    nshort = 0
    for r in range(n):
        rid, rsc, sh = _ref_blend_topk(s[r], g[r], gmv[r], alpha, k)
        nshort += sh
        np.testing.assert_array_equal(ids[r], rid, err_msg=f"row {r}")
        ok = ~np.isnan(rsc)
        np.testing.assert_array_equal(sc[r].view(np.int32)[ok], rsc.view(np.int32)[ok])
        assert np.all(np.isnan(sc[r][~ok]))
    assert int(short.item()) == nshort


@pytest.mark.parametrize("kind", ["sigmoid", "quantized", "equal", "narrow"])
@pytest.mark.parametrize("k", [1, 50, 1024])
def test_topk_blend_rows_kinds(kind, k):
    """Early exit after a few score digits (sigmoid), ties straddling rank k (quantized), one
    blended value for every candidate (equal: > 4,096 equal keys force the ~id digits), a wide
    top bin (narrow)."""
    rng = np.random.default_rng(zlib.crc32(f"blend/{kind}/{k}".encode()))
    s = _rows(kind, 4, 30011, rng)
    if kind == "equal":
        g = np.full(s.shape, 0.25, np.float64)
    elif kind == "quantized":
        g = np.round(rng.random(s.shape) * 50) / 50
    else:
        g = rng.random(s.shape) ** 8          # a power-law-like spread of products
    g[s < 0] = -1.0
    _check_blend(s, g, k)


def test_topk_blend_rows_nan_zero_max_and_short():
    rng = np.random.default_rng(19)
    s = _rows("uniform", 4, 5000, rng)
    g = rng.random(s.shape)
    s[0, [7, 123]] = np.nan                   # NaN scores rank first
    g[1, :] = 0.0                             # every product underflowed: gmax 0, no normalisation
    s[2, :] = -1.0
    s[2, [4, 40, 400]] = [0.3, 0.3, 0.1]      # 3 candidates < k
    s[3, 4100:] = -1.0
    g[s < 0] = -1.0
    _check_blend(s, g, 50)
