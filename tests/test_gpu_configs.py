"""GPU parity at the BASELINE.json configurations, through the C-ABI.

* config 4 -- the benchmarked path itself: the bench's whole job (50k users x 100k POIs,
  d = H = 64, h ~ U{1..200}, the bench's seeds) through catalog._score_topk_pairs with the bench's
  default knobs (fp16x6 tables, CU-masked overlap, 512-column blocks, fused running top-k,
  longest-first order). Every user's top-50 against the per-user ("direct") kernels; 32 users
  spread over h against the CPU restatements (torch_cpu + the numpy oracle for two).
* config 2 -- P = 50k, d = H = 64, h <= 100: a 600-user slice through both routes vs each other
  and vs the oracle.
* config 5 -- P = 1M, d = H = 128, h <= 200: 8 users through the direct route (full rows + top-50)
  and a forced pairs route over one column block, against the oracle (sampled candidates + the
  winners for every user, the full row for one user).

Tie rule: tests/_helpers.assert_topk_equivalent with 4 fp32 ulps; every test
prints how many tie runs were compared as sets and how many of them are not exact fp32 ties.
"""
import numpy as np
import pytest
import torch

from _helpers import SCORE_ATOL, TIE_STATS, assert_topk_equivalent
from oracle import nais_oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TIE_ULPS = 4


def _model(p, P, D, H):
    from poi_recommendation_models_amd.model import NAIS_basic
    m = NAIS_basic(P, D, H, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m.report_nan = False
    return m.to(DEV).eval()


def _compare_lists(ids_a, sc_a, ids_b, sc_b, users):
    """Tie-aware comparison of two [n, k] top-k sets (a = reference side); rows whose ids are
    identical and scores within SCORE_ATOL are accepted vectorised, the rest one by one."""
    same = np.all(ids_a == ids_b, axis=1) & np.all(np.abs(sc_a - sc_b) <= SCORE_ATOL, axis=1)
    runs = 0
    for r in np.nonzero(~same)[0]:
        runs += assert_topk_equivalent(ids_a[r], sc_a[r], ids_b[r], sc_b[r], tie_ulps=TIE_ULPS)
    return int((~same).sum()), runs


def _stats(tag, before):
    d = {k: TIE_STATS[k] - before[k] for k in TIE_STATS}
    print(f"{tag}: tie runs compared as sets {d['set_runs']} over {d['lists']} lists, "
          f"{d['inexact_runs']} of them not exact fp32 ties")


@pytest.fixture(scope="module")
def config4_job():
    """The bench's whole config-4 job through the pairs route with the bench's knobs, once per
    module: (data, params, ids, scores)."""
    from poi_recommendation_models_amd import catalog
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    U, P, D, H, K = 50_000, 100_000, 64, 64, 50
    data = make_checkins(U, P, 200, seed=2024)                   # bench.py's workload
    p = init_nais_params(P, D, H, seed=7, emb_std=0.3, bias_std=0.1)
    m = _model(p, P, D, H)
    assert m.precision == "fp16x6"
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    ev = []
    ids, sc = _score_topk_pairs(m, csr, np.arange(U), K, None, None, None, None, force=True, events=ev)
    settings = {k: n for k, a, b, n in ev if a is None}
    assert settings["table_cus"] not in (0, torch.cuda.get_device_properties(DEV).multi_processor_count)
    assert catalog.PAIR_FUSED_TOPK and catalog.PAIR_LPT_ORDER and catalog.PAIR_BLOCK_COLS == 512
    return data, p, m, csr, ids.cpu().numpy(), sc.cpu().numpy()


def test_config4_bench_job_pairs_vs_direct(config4_job):
    """Every one of the 50k users' top-50 lists: pairs route (the bench) against the per-user
    kernels (a self-comparison of the build's two routes; the oracle check is the next test)."""
    from poi_recommendation_models_amd.catalog import score_topk
    before = dict(TIE_STATS)
    data, p, m, csr, ids_p, sc_p = config4_job
    U, K = data.num_users, 50
    users = np.arange(U)
    ids_d, sc_d = score_topk(m, csr, users, K, strategy="direct")
    ids_d, sc_d = ids_d.cpu().numpy(), sc_d.cpu().numpy()
    hist_ok = all(not np.isin(ids_p[u], data.history(u)).any() for u in range(0, U, 97))
    assert hist_ok
    assert not np.isnan(sc_p).any()
    nd, runs = _compare_lists(ids_d, sc_d, ids_p, sc_p, users)
    print(f"config 4: {U} users, {nd} lists differ from the direct route in some position "
          f"(resolved by the tie rule, {runs} tie runs), max |score| diff at equal positions "
          f"{np.max(np.abs(sc_p - sc_d)):.3g}")
    _stats("config 4 pairs vs direct", before)


def _config4_oracle_users(h, n=32):
    """n users spread over the history lengths: the shortest, the longest and the quantiles
    in between (distinct users)."""
    order = np.argsort(h, kind="stable")
    pos = np.unique(np.round(np.linspace(0, len(order) - 1, n)).astype(np.int64))
    return [int(u) for u in order[pos]]


def test_config4_bench_job_vs_reference_restatement(config4_job):
    """32 users of the bench job, spread over h (shortest, longest, quantiles),
    against the CPU restatements: each user's full catalog through oracle/torch_cpu.py (the
    reference's loop in torch CPU ops, pinned to the reference's own outputs by
    tests/test_torch_cpu_baseline.py), tie-aware top-50 and scores; for 2 of them (the shortest
    and the median history) also the numpy oracle (oracle/nais_oracle.py)."""
    from oracle import torch_cpu
    before = dict(TIE_STATS)
    data, p, m, csr, ids_p, sc_p = config4_job
    P, K = data.num_pois, 50
    h = data.hist_len()
    users = _config4_oracle_users(h)
    assert len(users) == 32 and h[users[0]] == h.min() and h[users[-1]] == h.max()
    tm = torch_cpu.TorchNAIS(p)
    worst = 0.0
    for i, u in enumerate(users):
        hist = data.history(u)
        rows, cand = torch_cpu.candidates(hist, P)
        with torch.no_grad():
            ref = torch.cat([tm(rows[c:c + 1024], cand[c:c + 1024])
                             for c in range(0, len(cand), 1024)]).numpy()
        cand = cand.numpy()
        if i in (0, len(users) // 2):     # the shortest and the median also through numpy
            ocand, oref = nais_oracle.catalog_scores_basic(p, hist, P, chunk=4096)
            np.testing.assert_array_equal(ocand, cand)
            assert np.max(np.abs(oref - ref)) <= 1e-6
        rid, rsc = nais_oracle.topk_ids(cand, ref, K)
        lookup = dict(zip(cand.tolist(), ref.tolist()))
        assert_topk_equivalent(rid, rsc, ids_p[u], sc_p[u], tie_ulps=TIE_ULPS, lookup=lookup)
        got = np.array([lookup[int(c)] for c in ids_p[u]])
        d = float(np.max(np.abs(got - sc_p[u])))
        assert d <= SCORE_ATOL
        worst = max(worst, d)
    print(f"config 4: {len(users)} users (h = {h[users[0]]} .. {h[users[-1]]}) vs the restatement: "
          f"max |score - reference restatement| over their top-50 {worst:.3g}")
    _stats("config 4 vs restatement", before)


def test_config4_bench_job_sampled_oracle_2048_users(config4_job):
    """2,048 of the bench job's users spread over h (every h from 1 to 200
    several times), each against the CPU restatement on a sampled candidate set -- its top-50
    winners plus 500 random candidates -- as config 5 does below:
      * the winners' restated scores within SCORE_ATOL of the job's top-50 scores;
      * no sampled non-winner beats the weakest winner in the restatement by more than the
        4-ulp tie allowance (the selection is right on the sample);
      * the pairs route's full score rows of these users (nais_pair_gather) within SCORE_ATOL of
        the restatement on every sampled candidate.
    The restatement is oracle/torch_cpu.py (the reference's ops in torch CPU, pinned to its outputs
    by tests/test_torch_cpu_baseline.py); every 64th user also through the numpy oracle."""
    from oracle import torch_cpu
    from poi_recommendation_models_amd.catalog import score_catalog
    data, p, m, csr, ids_p, sc_p = config4_job
    P, K = data.num_pois, 50
    h = data.hist_len()
    users = _config4_oracle_users(h, 2048)
    assert len(users) >= 2000 and h[users[0]] == h.min() and h[users[-1]] == h.max()
    tm = torch_cpu.TorchNAIS(p)
    rng = np.random.default_rng(4)
    worst_w = worst_s = 0.0
    for b0 in range(0, len(users), 512):
        ub = users[b0:b0 + 512]
        full = score_catalog(m, csr, ub, strategy="pairs").cpu().numpy()
        for i, u in enumerate(ub):
            hist = data.history(u)
            cand = nais_oracle.complement_candidates(hist, P)
            extra = rng.choice(cand, 500, replace=False)
            probe = np.concatenate([ids_p[u].astype(np.int64), extra[~np.isin(extra, ids_p[u])]])
            with torch.no_grad():
                ref = tm(torch.as_tensor(hist).expand(len(probe), len(hist)),
                         torch.as_tensor(probe)).numpy()
            if (b0 + i) % 64 == 0:
                oref, _ = nais_oracle.forward_basic(p, np.broadcast_to(hist, (len(probe), len(hist))), probe)
                assert np.max(np.abs(oref - ref)) <= 1e-6, u
            dw = float(np.max(np.abs(ref[:K] - sc_p[u])))
            assert dw <= SCORE_ATOL, (u, dw)
            weakest = float(ref[:K].min())
            over = ref[K:] - weakest
            assert np.all(over <= TIE_ULPS * np.spacing(np.float32(weakest))), (u, float(over.max()))
            ds = float(np.max(np.abs(full[i][probe] - ref)))
            assert ds <= SCORE_ATOL, (u, ds)
            worst_w, worst_s = max(worst_w, dw), max(worst_s, ds)
    print(f"config 4: {len(users)} users (h = {h[users[0]]} .. {h[users[-1]]}) on sampled candidates "
          f"vs the restatement: max |winner score diff| {worst_w:.3g}, max |row score diff| {worst_s:.3g}")


def test_config2_slice_both_routes():
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    before = dict(TIE_STATS)
    U, P, D, H, K = 600, 50_000, 64, 64, 50
    data = make_checkins(U, P, 100, seed=202)
    p = init_nais_params(P, D, H, seed=203, emb_std=0.3, bias_std=0.1)
    m = _model(p, P, D, H)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    users = np.arange(U)
    ia, sa = score_topk(m, csr, users, K, strategy="direct")
    ib, sb = score_topk(m, csr, users, K, strategy="pairs")
    ia, sa, ib, sb = (x.cpu().numpy() for x in (ia, sa, ib, sb))
    nd, _ = _compare_lists(ia, sa, ib, sb, users)
    print(f"config 2 slice: {nd} of {U} lists differ between the routes (tie rule)")
    for u in (0, 1, 2):
        cand, ref = nais_oracle.catalog_scores_basic(p, data.history(u), P, chunk=4096)
        rid, rsc = nais_oracle.topk_ids(cand, ref, K)
        lookup = dict(zip(cand.tolist(), ref.tolist()))
        for ids, sc in ((ia, sa), (ib, sb)):
            assert_topk_equivalent(rid, rsc, ids[u], sc[u], tie_ulps=TIE_ULPS, lookup=lookup)
    _stats("config 2", before)


def test_config5_slice_direct_and_pairs_block():
    from poi_recommendation_models_amd.catalog import (DeviceCSR, _score_topk_pairs, score_catalog,
                                                       score_topk)
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    before = dict(TIE_STATS)
    U, P, D, H, K = 8, 1_000_000, 128, 128, 50
    data = make_checkins(U, P, 200, seed=505)
    p = init_nais_params(P, D, H, seed=506, emb_std=0.3, bias_std=0.1)
    m = _model(p, P, D, H)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    users = np.arange(U)
    full = score_catalog(m, csr, users).cpu().numpy()            # direct route, fp16x6
    ids, sc = score_topk(m, csr, users, K, strategy="direct")
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    rng = np.random.default_rng(7)
    h = data.hist_len()
    for u in range(U):
        hist = data.history(u)
        assert np.all(full[u][hist] == -1.0)
        cand = nais_oracle.complement_candidates(hist, P)
        oid, osc = nais_oracle.topk_ids(cand, full[u][cand], K)   # top-k == our own full row's
        np.testing.assert_array_equal(ids[u], oid)
        np.testing.assert_array_equal(sc[u], osc)
        probe = np.unique(np.concatenate([ids[u], rng.choice(cand, 1500, replace=False)]))
        ref, _ = nais_oracle.forward_basic(p, np.broadcast_to(hist, (len(probe), len(hist))), probe)
        assert np.max(np.abs(full[u][probe] - ref)) <= SCORE_ATOL, (u, np.max(np.abs(full[u][probe] - ref)))
    # one full oracle row (the shortest history) -> tie-aware top-50 against the reference order
    u = int(np.argmin(h))
    cand, ref = nais_oracle.catalog_scores_basic(p, data.history(u), P, chunk=8192)
    rid, rsc = nais_oracle.topk_ids(cand, ref, K)
    assert_topk_equivalent(rid, rsc, ids[u], sc[u], tie_ulps=TIE_ULPS,
                           lookup=dict(zip(cand.tolist(), ref.tolist())))
    assert np.max(np.abs(full[u][cand] - ref)) <= SCORE_ATOL
    # the pairs route forced over one 4,096-column block of the catalog
    c0, c1 = 400_000, 404_096
    pid, psc = _score_topk_pairs(m, csr, users, K, None, None, None, None, force=True, cols=(c0, c1))
    pid, psc = pid.cpu().numpy(), psc.cpu().numpy()
    for u in range(U):
        cand = nais_oracle.complement_candidates(data.history(u), P)
        cand = cand[(cand >= c0) & (cand < c1)]
        ref, _ = nais_oracle.forward_basic(p, np.broadcast_to(data.history(u), (len(cand), h[u])), cand)
        rid, rsc = nais_oracle.topk_ids(cand, ref, K)
        assert_topk_equivalent(rid, rsc, pid[u], psc[u], tie_ulps=TIE_ULPS,
                               lookup=dict(zip(cand.tolist(), ref.tolist())))
        did, dsc = nais_oracle.topk_ids(cand, full[u][cand], K)   # the direct route's block top-k
        assert_topk_equivalent(did, dsc, pid[u], psc[u], tie_ulps=TIE_ULPS)
    _stats("config 5", before)


def test_config4_bench_job_every_user_vs_torch_restatement(config4_job):
    """Every one of the bench job's 50,000 users (VERDICT r5 'What's weak' 1: 47,952 of them were
    only compared with the build's other route) against the reference's ops restated in torch
    (oracle/torch_cpu.TorchNAIS, pinned to the reference's outputs by
    tests/test_torch_cpu_baseline.py), run through PyTorch's own GPU kernels -- independent of
    this package's -- on a sampled candidate set per user: the job's top-50 winners, the build's
    ranks 51-60 (the selection boundary) and 40 random other candidates:
      * the winners' restated scores within SCORE_ATOL of the job's scores;
      * no boundary or random candidate beats the weakest winner in the restatement by more
        than the 4-ulp tie allowance."""
    from oracle import torch_cpu
    from poi_recommendation_models_amd.catalog import _score_topk_pairs
    data, p, m, csr, ids_p, sc_p = config4_job
    U, P, K, KB, NR = data.num_users, data.num_pois, 50, 60, 40
    ids60, _ = _score_topk_pairs(m, csr, np.arange(U), KB, None, None, None, None, force=True)
    ids60 = ids60.cpu().numpy()
    tm = torch_cpu.TorchNAIS(p, device=DEV)
    rng = np.random.default_rng(44)
    h = data.hist_len()
    worst_w, worst_over, ties, checked = 0.0, -1.0, 0, 0
    for hl in np.unique(h):
        us = np.nonzero(h == hl)[0]
        hist = np.stack([data.history(u) for u in us])                       # [n_u, hl]
        probes = np.empty((len(us), K + 10 + NR), np.int64)
        for i, u in enumerate(us):
            win = ids_p[u].astype(np.int64)
            bnd = ids60[u, K:KB].astype(np.int64)
            bnd = bnd[~np.isin(bnd, win)]
            extra = rng.integers(0, P, 4 * NR)
            extra = extra[~np.isin(extra, hist[i]) & ~np.isin(extra, win) & ~np.isin(extra, bnd)]
            rest = np.concatenate([bnd, extra])[:10 + NR]
            probes[i] = np.concatenate([win, rest])
        uh = torch.as_tensor(hist, device=DEV).repeat_interleave(probes.shape[1], dim=0)
        tg = torch.as_tensor(probes.reshape(-1), device=DEV)
        ref = tm(uh, tg).view(len(us), -1).cpu().numpy()
        dw = np.abs(ref[:, :K] - sc_p[us])
        worst_w = max(worst_w, float(dw.max()))
        assert dw.max() <= SCORE_ATOL, (int(hl), float(dw.max()))
        weakest = ref[:, :K].min(axis=1)
        over = ref[:, K:] - weakest[:, None]
        allow = TIE_ULPS * np.spacing(weakest.astype(np.float32))[:, None]
        bad = over > allow
        assert not bad.any(), (int(hl), us[np.nonzero(bad.any(1))[0][:5]].tolist(), float(over.max()))
        ties += int((over > 0).sum())
        worst_over = max(worst_over, float(over.max()))
        checked += len(us)
    assert checked == U
    print(f"config 4, all {U} users vs the torch restatement on the device: max |winner score diff| "
          f"{worst_w:.3g}; {ties} sampled candidates above the weakest winner, all within "
          f"{TIE_ULPS} ulps (max excess {worst_over:.3g})")


def test_config4_bench_job_every_user_full_catalog(config4_job):
    """Every one of the bench job's 50,000 users against EVERY candidate of the catalog (not a
    sample): tests/_torch_pairs.py forms the reference's e and e*s for all 10^10 (history POI,
    candidate) pairs in torch fp32 ops on the device (rocBLAS GEMMs, a sparse CSR product for the
    per-user sums -- none of this package's kernels), keeps each user's top-60 over the whole
    catalog and scores the job's own winners. Asserted: the winners' checker scores within
    SCORE_ATOL of the job's, and no candidate anywhere beats a user's weakest winner by more than
    the 4-ulp tie allowance. The checker is pinned to the numpy oracle by
    tests/test_torch_pairs_checker.py."""
    from _torch_pairs import check_against_full_catalog, full_catalog_topk
    data, p, m, csr, ids_p, sc_p = config4_job
    ti, tv, at = full_catalog_topk(p, data.indptr, data.indices, data.num_pois, 60, ids_p, DEV)
    dw, same, over = check_against_full_catalog(ids_p, sc_p, ti, tv, at, SCORE_ATOL, TIE_ULPS)
    print(f"config 4, all {data.num_users} users x all {data.num_pois} POIs vs the torch pairs checker: "
          f"max |winner score diff| {dw:.3g}; {same} users' top-50 equal the checker's as sets; "
          f"largest excess of a non-winner over the weakest winner {over:.3g} (allowed: {TIE_ULPS} ulps)")


def test_config4_region_distance_job_every_user_full_catalog():
    """The bench's region_distance leg (north_star's variant: bench.py rd_job -- same users and
    POIs, 1,024 regions, the POI coordinates) through the pairs route, every user against every
    candidate of the catalog with the torch pairs checker's region_distance form (model.py:246-297:
    [E | region] rows, sigmoid(dist_layer(100 |ll|)) features), as the test above."""
    from _torch_pairs import check_against_full_catalog, full_catalog_topk
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs
    from poi_recommendation_models_amd.model import NAIS_region_distance_Embedding
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    U, P, D, H, K = 50_000, 100_000, 64, 64, 50
    data = make_checkins(U, P, 200, seed=2024)                   # bench.py's workload
    p = init_nais_params(P, D, H, seed=11, emb_std=0.3, bias_std=0.1, variant="region_distance",
                         num_regions=1024)
    m = NAIS_region_distance_Embedding(P, D, H, 0.5, 1024, 1)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m.report_nan = False
    m = m.to(DEV).eval()
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    ev = []
    ids, sc = _score_topk_pairs(m, csr, np.arange(U), K, data.region_of, data.place_coords, None, None,
                                force=True, events=ev)
    assert any(kind == "bounded" for kind, *_ in ev)
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    del m
    ti, tv, at = full_catalog_topk(p, data.indptr, data.indices, P, 60, ids, DEV,
                                   region_of=data.region_of, coords=data.place_coords)
    dw, same, over = check_against_full_catalog(ids, sc, ti, tv, at, SCORE_ATOL, TIE_ULPS)
    print(f"config 4 region_distance, all {U} users x all {P} POIs vs the torch pairs checker: max "
          f"|winner score diff| {dw:.3g}; {same} users' top-50 equal the checker's as sets; largest "
          f"excess of a non-winner over the weakest winner {over:.3g} (allowed: {TIE_ULPS} ulps)")


def test_config2_job_every_user_full_catalog():
    """Config 2 (bench.py --config 2: 10,000 users x 50,000 POIs, d = H = 64, h <= 100, the bench's
    seeds) through the pairs route with the bench's knobs: every user against every candidate
    with the torch pairs checker (tests/_torch_pairs.py), as the config-4 test above."""
    from _torch_pairs import check_against_full_catalog, full_catalog_topk
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    U, P, D, H, K = 10_000, 50_000, 64, 64, 50
    data = make_checkins(U, P, 100, seed=2024)
    p = init_nais_params(P, D, H, seed=7, emb_std=0.3, bias_std=0.1)
    m = _model(p, P, D, H)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    ids, sc = _score_topk_pairs(m, csr, np.arange(U), K, None, None, None, None, force=True)
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    ti, tv, at = full_catalog_topk(p, data.indptr, data.indices, P, 60, ids, DEV)
    dw, same, over = check_against_full_catalog(ids, sc, ti, tv, at, SCORE_ATOL, TIE_ULPS)
    print(f"config 2, all {U} users x all {P} POIs vs the torch pairs checker: max |winner score diff| "
          f"{dw:.3g}; {same} users' top-50 equal the checker's as sets; largest excess {over:.3g}")


def test_config5_direct_64_users_full_catalog():
    """Config 5 (200,000 users x 1,000,000 POIs, d = H = 128, h <= 200; bench.py --config 5 times
    the direct route on the first users): the first 64 users through the direct route, each
    against all 10^6 candidates with the torch pairs checker (its rows: the 64 users' distinct
    history POIs only)."""
    from _torch_pairs import check_against_full_catalog, full_catalog_topk
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    U, P, D, H, K, NU = 200_000, 1_000_000, 128, 128, 50, 64
    data = make_checkins(U, P, 200, seed=2024)
    p = init_nais_params(P, D, H, seed=7, emb_std=0.3, bias_std=0.1)
    m = _model(p, P, D, H)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, DEV)
    ids, sc = score_topk(m, csr, np.arange(NU), K, strategy="direct")
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    ip = data.indptr[:NU + 1]
    ti, tv, at = full_catalog_topk(p, ip, data.indices[:ip[-1]], P, 60, ids, DEV, jchunk=4096)
    dw, same, over = check_against_full_catalog(ids, sc, ti, tv, at, SCORE_ATOL, TIE_ULPS)
    print(f"config 5, {NU} users x all {P} POIs (direct route) vs the torch pairs checker: max |winner "
          f"score diff| {dw:.3g}; {same} users' top-50 equal the checker's as sets; largest excess {over:.3g}")
