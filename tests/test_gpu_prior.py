"""GPU parity of the power-law prior path (powerLaw.py, run.py:55-59, 537-539) through the C-ABI,
against the reference golden vectors (tests/golden/powerlaw.npz) and the pure-Python oracle."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from _helpers import assert_topk_equivalent, load_golden, params_from
from oracle import nais_oracle, powerlaw_oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _csr(ip, ix, P):
    return sp.csr_matrix((np.ones(len(ix)), ix, ip), shape=(len(ip) - 1, P))


def test_prior_rows_match_reference_predict():
    from poi_recommendation_models_amd.catalog import prior_rows
    z = load_golden("powerlaw.npz")
    ip, ix, co = z["pl_indptr"], z["pl_indices"], z["pl_coords"]
    a, b = z["fit_ab"]
    X = _csr(ip, ix, len(co))
    G, mx = prior_rows(X, range(len(ip) - 1), a, b, co, DEV)
    G, mx = G.cpu().numpy(), mx.cpu().numpy()
    ref = z["predict"]                                  # reference PowerLaw.predict values
    worst = 0.0
    for u in range(len(ip) - 1):
        hist = set(ix[ip[u]:ip[u + 1]].tolist())
        for ci, c in enumerate(z["predict_cands"]):
            if int(c) in hist:
                assert G[u, c] == -1.0
                continue
            r = ref[u, ci]
            if r == 0.0:
                assert G[u, c] < 1e-300
            else:
                worst = max(worst, abs(G[u, c] - r) / abs(r))
        # normalize() divisor: max over the user's complement candidates
        cand = np.array([c for c in range(len(co)) if c not in hist])
        assert mx[u] == np.max(G[u, cand])
    # powerLaw.dist is acos(sin*sin*cos + cos*cos): for POIs tens of metres apart cos ~ 1 - 1e-11
    # and a 1-ulp difference between the device's and glibc's sin/cos/acos moves d by ~1e-6
    # relative. The prior is normalised and weighted by alpha = 0.2 before it meets scores in
    # [0, 1], so 1e-6 relative here is < 2e-7 absolute in the blended score (bar: 1e-4).
    assert worst < 1e-6, worst
    print("prior max relative error vs reference predict:", worst)


def test_distance_histogram_and_fit():
    from poi_recommendation_models_amd.powerlaw import PowerLaw, distance_histogram
    z = load_golden("powerlaw.npz")
    ip, ix, co = z["pl_indptr"], z["pl_indices"], z["pl_coords"]
    X = _csr(ip, ix, len(co))
    got = distance_histogram(X, co, DEV)
    ref = {}
    for u in range(len(ip) - 1):
        lids = ix[ip[u]:ip[u + 1]]
        for i in range(len(lids)):
            for j in range(i + 1, len(lids)):
                k = int(powerlaw_oracle.dist(co[lids[i]], co[lids[j]]))
                ref[k] = ref.get(k, 0) + 1
    assert got == ref
    np.random.seed(0)
    G = PowerLaw()
    G.fit_distance_distribution(X, co, DEV)
    np.testing.assert_allclose([G.a, G.b], z["fit_ab"], rtol=1e-12)


@pytest.mark.parametrize("strategy", ["direct", "pairs"])
def test_score_topk_with_prior_blend(strategy):
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    from poi_recommendation_models_amd.model import NAIS_basic
    z = load_golden("catalog_basic.npz")
    p = params_from(z, "trained")
    P, U = int(z["num_pois"]), int(z["num_users"])
    m = NAIS_basic(P, 16, 16, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(DEV).eval()
    m.report_nan = False
    csr = DeviceCSR.from_arrays(z["indptr"], z["indices"], P, torch.device(DEV))
    co = z["coords"]
    a, b, alpha = 0.052, -1.37, 0.2
    for prec in ("fp32", "fp16x6", "fp16x3"):
        m.precision = prec
        ids, sc = score_topk(m, csr, range(8), 50, prior=(a, b, alpha, co), strategy=strategy)
        ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
        for u in range(8):
            hist = z["indices"][z["indptr"][u]:z["indptr"][u + 1]]
            cand, s = nais_oracle.catalog_scores_basic(p, hist, P)
            g = [powerlaw_oracle.predict(a, b, co, hist, int(c)) for c in cand]
            gn = np.array(powerlaw_oracle.normalize(g))
            blended = powerlaw_oracle.blend(s, gn, alpha)
            rid, rsc = nais_oracle.topk_ids(cand, blended, 50)
            assert_topk_equivalent(rid, rsc, ids[u], sc[u], tie_ulps=8,   # blended f64 prior: ill-conditioned dist(), 8 ulps
                                  
                                   lookup=dict(zip(cand.tolist(), blended.tolist())))


@pytest.mark.parametrize("h_max,flags,a", [(60, 0, 0.052), (60, 1, 0.052), (240, 0, 0.052),
                                           (240, 1, 0.052), (240, 0, -0.052)])
def test_pair_prior_gather_equals_prior_rows_bits(h_max, flags, a):
    """The pairs route's G (nais_pair_prior_table + nais_pair_prior_gather, several column blocks)
    is bit-identical to nais_powerlaw_prior's rows (the direct route), and so is the per-user max --
    also with the underflow exit (flags = NAIS_PRIOR_FINITE) on histories long enough (h up to 240)
    that whole stripes of G underflow to 0.0 (np.prod's own result, powerLaw.py:92). flags = 0
    computes every factor, so the (240, 0) case also pins prior_kernel's own underflow exit
    (prior_zero_exit) bit for bit; a < 0 (signed zeros: the exit must be off) pins its guard."""
    from poi_recommendation_models_amd import _capi
    from poi_recommendation_models_amd.catalog import DeviceCSR, prior_rows
    from poi_recommendation_models_amd.synthetic import make_checkins
    data = make_checkins(40, 1500, h_max, seed=8)
    P, U = data.num_pois, data.num_users
    b = -1.37
    dev = torch.device(DEV)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    ref, ref_max = prior_rows(csr, range(U), a, b, data.place_coords, dev)
    lib = _capi.load()
    users = torch.arange(U, dtype=torch.int32, device=dev)
    rowmap = torch.empty(P, dtype=torch.int32, device=dev)
    items = torch.empty(P, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(lib.nais_pair_rows_workspace_size(P), dtype=torch.uint8, device=dev)
    st = _capi.stream_handle(dev)
    _capi.check(lib.nais_pair_rows(csr.indptr.data_ptr(), csr.indices.data_ptr(), users.data_ptr(), U, P,
                                   rowmap.data_ptr(), items.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
                                   ws.numel(), st), "nais_pair_rows")
    J = int(cnt.item())
    co = torch.as_tensor(data.place_coords, dtype=torch.float64, device=dev)
    W = 384                                             # blocks of 384 columns, the last one partial
    pr = torch.empty(J, W, dtype=torch.float64, device=dev)
    G = torch.empty(U, P, dtype=torch.float64, device=dev)
    gmax = torch.zeros(U, dtype=torch.int64, device=dev)
    for c0 in range(0, P, W):
        w = min(W, P - c0)
        _capi.check(lib.nais_pair_prior_table(co.data_ptr(), P, items.data_ptr(), J, c0, w, a, b,
                                              pr.data_ptr(), W, st), "nais_pair_prior_table")
        _capi.check(lib.nais_pair_prior_gather(pr.data_ptr(), W, rowmap.data_ptr(), csr.indptr.data_ptr(),
                                               csr.indices.data_ptr(), users.data_ptr(), U, c0, w,
                                               G.data_ptr(), P, 0, gmax.data_ptr(), flags, st),
                    "nais_pair_prior_gather")
    torch.cuda.synchronize()
    assert torch.equal(G.view(torch.int64), ref.view(torch.int64))
    assert torch.equal(gmax, ref_max.view(torch.int64))
    if h_max > 200 and a > 0:   # the case the exit is for: some users' whole rows underflowed
        assert bool(((G == 0) | (G == -1)).all(dim=1).any())


def test_prior_pairs_route_vs_direct_route():
    """score_topk(prior=...) through the pairs route (score rows + pr_d tables + G products +
    nais_topk_blend_rows) against the per-user route on 400 users x 6,000 POIs sharing POIs: the
    G rows are bit-identical by construction (previous test), the scores agree within the tie rule."""
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    from poi_recommendation_models_amd.model import NAIS_basic
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    data = make_checkins(400, 6000, 120, seed=31)
    P, U = data.num_pois, data.num_users
    p = init_nais_params(P, 64, 64, seed=32, emb_std=0.3, bias_std=0.1)
    m = NAIS_basic(P, 64, 64, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(DEV).eval()
    m.report_nan = False
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, torch.device(DEV))
    prior = (0.052, -1.37, 0.2, data.place_coords)
    ia, sa = score_topk(m, csr, range(U), 50, prior=prior, strategy="direct")
    ib, sb = score_topk(m, csr, range(U), 50, prior=prior, strategy="pairs")
    ia, sa, ib, sb = ia.cpu().numpy(), sa.cpu().numpy(), ib.cpu().numpy(), sb.cpu().numpy()
    same = np.all(ia == ib, axis=1)
    for u in np.nonzero(~same)[0]:
        assert_topk_equivalent(ia[u], sa[u], ib[u], sb[u], tie_ulps=8)
    assert np.max(np.abs(sa - sb)) < 1e-6
    print(f"prior pairs vs direct: {int((~same).sum())} of {U} lists differ inside tie runs")
