"""Multi-rank host logic on CPU (gloo, world_size 2): LPT user sharding and the top-k gather
reassemble exactly the single-process recommended lists. The per-rank scorer here is the
oracle (test infrastructure); on the GPUs it is catalog.score_topk."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

from _helpers import load_golden, params_from, positives_from
from oracle import nais_oracle
from poi_recommendation_models_amd.sharding import gather_topk, shard_users


def _rccl_calls_only(dist):
    """The list form of all_gather (and all_gather_object) is never what the product calls: every
    exchange in sharding.py is the concatenated all_gather_into_tensor RCCL runs on the GPUs."""
    def forbidden(*a, **k):
        raise AssertionError("sharding must use all_gather_into_tensor")
    dist.all_gather = forbidden
    dist.all_gather_object = forbidden


def test_shard_users_lpt_balance():
    rng = np.random.default_rng(0)
    h = rng.integers(1, 201, 5000)
    parts = shard_users(h, 100_000, 8)
    allu = np.sort(np.concatenate(parts))
    np.testing.assert_array_equal(allu, np.arange(5000))
    cost = (100_000 - h) * h
    loads = np.array([cost[p].sum() for p in parts])
    assert loads.max() / loads.mean() < 1.001
    assert [len(p) for p in shard_users(h[:3], 1000, 4)].count(0) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    z = load_golden("catalog_basic.npz")
    p = params_from(z, "trained")
    P, U = int(z["num_pois"]), int(z["num_users"])
    hl = np.diff(z["indptr"])
    mine = shard_users(hl, P, world)[rank]
    ids, sc = [], []
    for u in mine:
        cand, s = nais_oracle.catalog_scores_basic(p, z["indices"][z["indptr"][u]:z["indptr"][u + 1]], P)
        i, t = nais_oracle.topk_ids(cand, s, 50)
        ids.append(i)
        sc.append(t)
    ids = torch.as_tensor(np.array(ids).reshape(-1, 50))
    sc = torch.as_tensor(np.array(sc, dtype=np.float32).reshape(-1, 50))
    gi, gs = gather_topk(mine, ids, sc, U)
    q.put((rank, gi.numpy(), gs.numpy()))
    dist.destroy_process_group()


def test_gather_topk_world2_matches_single_process():
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    z = load_golden("catalog_basic.npz")
    p = params_from(z, "trained")
    P, U = int(z["num_pois"]), int(z["num_users"])
    ref = np.array([nais_oracle.topk_ids(*nais_oracle.catalog_scores_basic(
        p, z["indices"][z["indptr"][u]:z["indptr"][u + 1]], P), 50)[0] for u in range(U)])
    for rank, gi, gs in res:
        np.testing.assert_array_equal(gi, ref)
        assert not np.isnan(gs).any()


def _worker_tables(rank, world, port, q):
    import torch.distributed as dist
    from poi_recommendation_models_amd.sharding import allgather_rows, load_sharded_tables, row_block
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    P, d = 1001, 8                                  # not divisible by world: padding path
    full = torch.arange(P * d, dtype=torch.float32).reshape(P, d)
    s, e = row_block(P, rank, world)
    got = allgather_rows(full[s:e].clone(), P)
    ok1 = torch.equal(got, full)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.embed_history = torch.nn.Embedding(P, d)
            self.embed_target = torch.nn.Embedding(P, d)
            self.attn_layer1 = torch.nn.Linear(d, 4)
    torch.manual_seed(rank)                         # ranks start with different MLP weights
    m = M()
    load_sharded_tables(m, lambda name, a, b: full[a:b] * (2 if name == "embed_target" else 1))
    ok2 = torch.equal(m.embed_history.weight.data, full) and torch.equal(m.embed_target.weight.data, 2 * full)
    q.put((rank, ok1, ok2, m.attn_layer1.weight.data.clone().numpy()))
    dist.destroy_process_group()


def test_sharded_table_allgather_world2():
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_tables, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(r[1] and r[2] for r in res)
    np.testing.assert_array_equal(res[0][3], res[1][3])   # MLP broadcast from rank 0


def _worker_validation(rank, world, port, q, mode="env"):
    """validation.NAIS_validation inside a world-2 gloo group. mode "env" (NAIS_DISTRIBUTED_EVAL=1,
    run.py:112-116 unchanged) and "kw" (distributed=True) route to sharding.distributed_topk on
    every rank; "default" stays single-process, and only rank 0 calls (the DDP pattern that must
    not block in a collective). The device scorers are replaced by the oracle here (CPU test); the
    user sharding, the all-gather of the [users, k] blocks and the metrics are the product code."""
    import scipy.sparse as sp
    import torch.distributed as dist
    from poi_recommendation_models_amd import sharding
    from poi_recommendation_models_amd import validation as V
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    z = load_golden("catalog_basic.npz")
    p = params_from(z, "trained")
    P, U = int(z["num_pois"]), int(z["num_users"])
    calls = []

    def oracle_distributed_topk(model, train_matrix, num_users, k, group=None, **kw):
        calls.append(num_users)
        hl = np.diff(train_matrix.indptr)[:num_users]
        mine = shard_users(hl, P, dist.get_world_size(group))[dist.get_rank(group)]
        ids, sc = [], []
        for u in mine:
            hist = train_matrix.indices[train_matrix.indptr[u]:train_matrix.indptr[u + 1]]
            i, t = nais_oracle.topk_ids(*nais_oracle.catalog_scores_basic(p, hist, P), k)
            ids.append(i)
            sc.append(t)
        return gather_topk(mine, torch.as_tensor(np.array(ids).reshape(-1, k)),
                           torch.as_tensor(np.array(sc, dtype=np.float32).reshape(-1, k)),
                           num_users, group=group)
    sharding.distributed_topk = oracle_distributed_topk

    def oracle_score_topk(model, train_matrix, users, k, **kw):
        calls.append(("single", len(users)))
        ids = []
        for u in users:
            hist = train_matrix.indices[train_matrix.indptr[u]:train_matrix.indptr[u + 1]]
            ids.append(nais_oracle.topk_ids(*nais_oracle.catalog_scores_basic(p, hist, P), k)[0])
        return torch.as_tensor(np.array(ids).reshape(-1, k)), None
    V.score_topk = oracle_score_topk
    if mode == "env":
        os.environ["NAIS_DISTRIBUTED_EVAL"] = "1"

    class Model:                      # what _recommend_ids touches on the module
        report_nan = True
        _last_nan = torch.zeros((), dtype=torch.int32)

        def eval(self):
            return self

    class Args:
        topk = 50
    X = sp.csr_matrix((np.ones(len(z["indices"])), z["indices"], z["indptr"]), shape=(U, P))
    got = None
    if mode != "default" or rank == 0:
        got = np.array(V.NAIS_validation(Model(), Args(), U, positives_from(z, "test"),
                                         positives_from(z, "val"), X, [5, 10, 15, 20, 25, 30],
                                         **({"distributed": True} if mode == "kw" else {})))
    q.put((rank, calls, got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["env", "kw", "default"])
def test_validation_distributed_opt_in_world2(mode):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_validation, args=(r, 2, port, q, mode)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    z = load_golden("catalog_basic.npz")
    U = int(z["num_users"])
    if mode == "default":                                   # rank 0 alone, single-process path
        assert res[0][1] == [("single", U)] and res[1][1] == [] and res[1][2] is None
        np.testing.assert_array_equal(res[0][2], z["trained/metrics"])
        return
    # exactly the reference's 6-tuple: the scorer is the oracle, whose top-k
    # lists equal the fixture's (catalog_basic holds no tie run straddling a k,
    # test_oracle_golden.py::test_metric_fixtures_have_no_straddling_ties)
    for rank, calls, got in res:
        assert calls == [U], calls                          # went through the distributed path
        np.testing.assert_array_equal(got, z["trained/metrics"])
    np.testing.assert_array_equal(res[0][2], res[1][2])     # the same 6-tuple on every rank


def test_column_blocks_and_min_block_candidates_edges():
    """P % world != 0 (narrow last block) and worlds with empty blocks. The guard counts
    each user's candidates inside every rank's real block; distributed_plan falls back to user
    sharding whenever one block holds fewer than k."""
    import scipy.sparse as sp
    from poi_recommendation_models_amd.catalog import DeviceCSR
    from poi_recommendation_models_amd.sharding import column_blocks, distributed_plan, min_block_candidates
    blocks = column_blocks(1001, 8)                     # S = 126: last block [882, 1001) = 119 wide
    assert blocks[0] == (0, 126) and blocks[-1] == (882, 1001)
    assert sum(c1 - c0 for c0, c1 in blocks) == 1001
    empty = column_blocks(10, 8)                        # S = 2: ranks 5..7 own nothing
    assert empty[5:] == [(10, 10)] * 3 and sum(c1 - c0 for c0, c1 in empty) == 10
    # user 0: 76 history POIs all inside the last block -> 119 - 76 = 43 candidates there
    hist = [np.arange(882, 958), np.arange(0, 10)]
    indptr = np.array([0, 76, 86])
    X = sp.csr_matrix((np.ones(86), np.concatenate(hist), indptr), shape=(2, 1001))
    csr = DeviceCSR(X, torch.device("cpu"))
    assert min_block_candidates(csr, [0, 1], 1001, 8) == 43
    assert min_block_candidates(csr, [1], 1001, 8) == 116   # user 1: block 0 holds 126 - 10
    assert distributed_plan(csr, 2, 1001, 50, 8) == "users"   # 43 < k: user sharding
    assert min_block_candidates(csr, [1], 1001, 1) == 1001 - 10          # world 1: the whole catalog
    X2 = sp.csr_matrix((np.ones(2), np.array([0, 1]), np.array([0, 1, 2])), shape=(2, 10))
    csr2 = DeviceCSR(X2, torch.device("cpu"))
    assert min_block_candidates(csr2, [0, 1], 10, 8) == 0    # empty blocks have no candidates
    assert distributed_plan(csr2, 2, 10, 1, 8) == "users"


def _fake_topk_rows(scores, ld, ncols, n, k, out_ids, out_scores, short, stream):
    """nais_topk_rows (include/nais.h) restated in numpy over the raw CPU pointers: per row the
    k largest non-negative entries, (score desc, column asc), NaN first."""
    import ctypes
    s = np.ctypeslib.as_array((ctypes.c_float * (n * ld)).from_address(scores)).reshape(n, ld)[:, :ncols]
    oi = np.ctypeslib.as_array((ctypes.c_int32 * (n * k)).from_address(out_ids)).reshape(n, k)
    os_ = np.ctypeslib.as_array((ctypes.c_float * (n * k)).from_address(out_scores)).reshape(n, k)
    for r in range(n):
        cols = np.nonzero(~(s[r] < 0))[0]
        i, t = nais_oracle.topk_ids(cols, s[r][cols], k)
        oi[r, :len(i)], os_[r, :len(i)] = i, t
        oi[r, len(i):], os_[r, len(i):] = -1, np.nan
    return 0


def _worker_columns(rank, world, port, q):
    """sharding.distributed_topk_pairs over a world-3 gloo group with P % 3 != 0: each rank's
    column block is scored by the oracle (the device's _score_topk_pairs on the GPUs), the
    all-gather and merge_topk are the product code (nais_topk_rows restated in numpy on CPU)."""
    import torch.distributed as dist
    from poi_recommendation_models_amd import _capi, catalog, sharding
    from poi_recommendation_models_amd.catalog import DeviceCSR
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    P, U, K = 301, 9, 20                       # blocks [0, 101) [101, 202) [202, 301): 99 wide
    p, hist = _columns_case(P, U)
    import scipy.sparse as sp
    indptr = np.concatenate([[0], np.cumsum([len(h) for h in hist])])
    X = sp.csr_matrix((np.ones(indptr[-1]), np.concatenate(hist), indptr), shape=(U, P))
    csr = DeviceCSR(X, torch.device("cpu"))

    def oracle_block(model, csr_, users, k, region_of, coords, latlon_mat, stream, force, cols=None, **kw):
        c0, c1 = cols
        ids, sc = [], []
        for u in users:
            cand, s = nais_oracle.catalog_scores_basic(p, hist[u], P)
            inb = (cand >= c0) & (cand < c1)
            i, t = nais_oracle.topk_ids(cand[inb], s[inb], k)
            ids.append(i)
            sc.append(t)
        return torch.as_tensor(np.array(ids, dtype=np.int64)), torch.as_tensor(np.array(sc, np.float32))

    class Lib:
        nais_topk_rows = staticmethod(_fake_topk_rows)

    class Model:
        def _check_device(self):
            return torch.device("cpu")
    catalog._score_topk_pairs = oracle_block
    _capi.load = lambda *a: Lib()
    _capi.stream_handle = lambda dev: None
    mbc = sharding.min_block_candidates(csr, range(U), P, world)
    ids, sc = sharding.distributed_topk_pairs(Model(), csr, range(U), K)
    q.put((rank, mbc, ids.numpy(), sc.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _columns_case(P, U):
    from poi_recommendation_models_amd.synthetic import init_nais_params
    p = init_nais_params(P, 16, 16, seed=31, emb_std=0.3, bias_std=0.1)
    rng = np.random.default_rng(32)
    hist = [np.sort(rng.choice(P, int(rng.integers(1, 30)), replace=False)) for _ in range(U)]
    hist[0] = np.arange(202, 202 + 79)          # fills 79 of the narrow last block's 99 columns
    hist[1] = np.array([], dtype=np.int64)      # empty history: every score 0.5 (ties by id)
    return p, hist


def test_column_sharded_merge_world3_p_not_divisible():
    """a world-3 column-sharded job with P = 301 (narrow last block of 99
    columns), one user holding 79 of them (20 candidates left there, = k) and an empty-history
    user: every rank gets the single-process top-k, ids and scores exactly."""
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_columns, args=(r, 3, port, q)) for r in range(3)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(3)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    P, U, K = 301, 9, 20
    p, hist = _columns_case(P, U)
    assert all(r[1] == 20 for r in res)         # user 0's last block keeps exactly k candidates
    for u in range(U):
        cand, s = nais_oracle.catalog_scores_basic(p, hist[u], P)
        rid, rsc = nais_oracle.topk_ids(cand, s, K)
        for rank, _, ids, sc in res:
            np.testing.assert_array_equal(ids[u], rid)
            np.testing.assert_array_equal(sc[u], rsc)


def _fake_merge_f64(keys, ids, n, m, k, out_ids, out_scores, out_keys, stream):
    """nais_topk_merge_f64 (include/nais.h) restated in numpy over raw CPU pointers."""
    import ctypes
    kk = np.ctypeslib.as_array((ctypes.c_double * (n * m)).from_address(keys)).reshape(n, m)
    ii = np.ctypeslib.as_array((ctypes.c_int64 * (n * m)).from_address(ids)).reshape(n, m)
    oi = np.ctypeslib.as_array((ctypes.c_int64 * (n * k)).from_address(out_ids)).reshape(n, k)
    os_ = np.ctypeslib.as_array((ctypes.c_float * (n * k)).from_address(out_scores)).reshape(n, k)
    for r in range(n):
        ok = ii[r] >= 0
        i, t = nais_oracle.topk_ids(ii[r][ok], kk[r][ok], k)
        oi[r, :len(i)], os_[r, :len(i)] = i, t.astype(np.float32)
        oi[r, len(i):], os_[r, len(i):] = -1, np.nan
    return 0


PRIOR = (0.052, -1.37, 0.2)


def _prior_case():
    from poi_recommendation_models_amd.synthetic import init_nais_params
    P, U = 151, 6
    p = init_nais_params(P, 16, 16, seed=41, emb_std=0.3, bias_std=0.1)
    rng = np.random.default_rng(42)
    coords = np.stack([40.7 + rng.random(P) * 0.2, -74.0 + rng.random(P) * 0.2], 1)
    hist = [np.sort(rng.choice(P, int(rng.integers(1, 12)), replace=False)) for _ in range(U)]
    return P, U, p, coords, hist


def _blend_rows(p, coords, hist, P, cols):
    """(candidate ids in [c0, c1), f32 score, f64 G) of one user (oracle restatements)."""
    from oracle import powerlaw_oracle
    cand, s = nais_oracle.catalog_scores_basic(p, hist, P)
    keep = (cand >= cols[0]) & (cand < cols[1])
    cl = [tuple(c) for c in coords.tolist()]
    G = np.array([powerlaw_oracle.predict(PRIOR[0], PRIOR[1], cl, hist, int(c)) for c in cand[keep]])
    return cand[keep], s[keep], G


def _worker_prior(rank, world, port, q):
    """sharding.distributed_topk_pairs with a prior over a world-2 gloo group: each rank's column
    block is scored and blended by the oracle (the device's _score_topk_pairs on the GPUs) with the
    max G all-reduced by the product code (sharding.allreduce_gmax, as _score_topk_pairs calls it);
    the all-gather (all_gather_into_tensor, the RCCL call) and the f64 merge (merge_topk_f64 over
    nais_topk_merge_f64 restated in numpy) are the product code."""
    import torch.distributed as dist
    from oracle import powerlaw_oracle
    from poi_recommendation_models_amd import _capi, catalog, sharding
    from poi_recommendation_models_amd.catalog import DeviceCSR
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    P, U, p, coords, hist = _prior_case()
    K = 10
    import scipy.sparse as sp
    indptr = np.concatenate([[0], np.cumsum([len(h) for h in hist])])
    X = sp.csr_matrix((np.ones(indptr[-1]), np.concatenate(hist), indptr), shape=(U, P))
    csr = DeviceCSR(X, torch.device("cpu"))
    seen = {}

    def oracle_block(model, csr_, users, k, region_of, coords_, latlon_mat, stream, force, cols=None,
                     prior=None, group=None, return_keys=False, **kw):
        assert prior is not None and return_keys and group is not None
        rows = [_blend_rows(p, coords, hist[u], P, cols) for u in users]
        gmax = torch.tensor([max(g.max(), 0.0) for _, _, g in rows], dtype=torch.float64).view(torch.int64)
        seen["local_max"] = gmax.view(torch.float64).clone().numpy()
        sharding.allreduce_gmax(gmax, group)
        gm = gmax.view(torch.float64).numpy()
        seen["gmax"] = gm.copy()
        ids, keys = [], []
        for u, (cand, s, G) in enumerate(rows):
            gn = G / gm[u] if gm[u] != 0 else G
            i, t = nais_oracle.topk_ids(cand, powerlaw_oracle.blend(s, gn, PRIOR[2]), k)
            ids.append(i)
            keys.append(t)
        keys = torch.as_tensor(np.array(keys, dtype=np.float64))
        return torch.as_tensor(np.array(ids, dtype=np.int64)), keys.to(torch.float32), keys

    class Lib:
        nais_topk_merge_f64 = staticmethod(_fake_merge_f64)

    class Model:
        def _check_device(self):
            return torch.device("cpu")
    catalog._score_topk_pairs = oracle_block
    _capi.load = lambda *a: Lib()
    _capi.stream_handle = lambda dev: None
    mi, ms = sharding.distributed_topk_pairs(Model(), csr, range(U), K, prior=(*PRIOR[:2], PRIOR[2], coords))
    q.put((rank, seen["local_max"], seen["gmax"], mi.numpy(), ms.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_column_sharded_prior_max_allreduce_world2():
    """the prior over column shards normalises by the max G of the WHOLE
    catalog (MAX all-reduce of each user's per-shard max) and merges on the f64 blended score:
    the merged top-k equals the single-process blended top-k (run.py:537-539) exactly."""
    from oracle import powerlaw_oracle
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_prior, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    P, U, p, coords, hist = _prior_case()
    K = 10
    np.testing.assert_array_equal(res[0][2], np.maximum(res[0][1], res[1][1]))   # the global max
    assert np.any(res[0][1] != res[1][1])             # the shards' own maxima do differ
    for u in range(U):
        cand, s, G = _blend_rows(p, coords, hist[u], P, (0, P))
        b = powerlaw_oracle.blend(s, np.asarray(powerlaw_oracle.normalize(list(G))), PRIOR[2])
        rid, rsc = nais_oracle.topk_ids(cand, b, K)
        for rank, _, gm, mi, ms in res:
            assert gm[u] == G.max()
            np.testing.assert_array_equal(mi[u], rid)
            np.testing.assert_array_equal(ms[u], rsc.astype(np.float32))


def test_env_opt_in_without_group_falls_back(monkeypatch):
    """NAIS_DISTRIBUTED_EVAL=1 left in the environment of a single-process run
    evaluates in this process (with a warning); distributed=True without a group still raises."""
    import warnings
    from poi_recommendation_models_amd import validation
    monkeypatch.setenv("NAIS_DISTRIBUTED_EVAL", "1")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert validation._want_distributed(None) is False
    assert any("NAIS_DISTRIBUTED_EVAL" in str(x.message) for x in w)
    with pytest.raises(RuntimeError):
        validation._want_distributed(True)
    monkeypatch.setenv("NAIS_DISTRIBUTED_EVAL", "0")
    assert validation._want_distributed(None) is False


@pytest.mark.parametrize("world,k,route", [(2, 50, "pairs"), (8, 256, "pairs"), (16, 256, "users"),
                                           (3, 1000, "users")])
def test_prior_route_respects_merge_cap(monkeypatch, world, k, route):
    """a prior job takes the column-sharded route only while the f64 merge holds the
    world * k candidates per user (nais_topk_merge_f64: <= 2048); otherwise the user-sharded one."""
    import torch.distributed as dist
    from poi_recommendation_models_amd import catalog, sharding
    taken = []
    monkeypatch.setattr(dist, "get_rank", lambda group=None: 0)
    monkeypatch.setattr(dist, "get_world_size", lambda group=None: world)
    monkeypatch.setattr(sharding, "distributed_plan", lambda *a, **kw: "pairs")
    monkeypatch.setattr(sharding, "distributed_topk_pairs", lambda *a, **kw: taken.append("pairs"))
    monkeypatch.setattr(catalog, "score_topk", lambda *a, **kw: (None, None))
    monkeypatch.setattr(sharding, "gather_topk", lambda *a, **kw: taken.append("users"))

    class Model:
        _pairs_only = False

        def eval(self):
            pass

        def _check_device(self):
            return torch.device("cpu")

        def _item_tables(self):
            return (torch.empty(4000, 1),)
    import scipy.sparse as sp
    X = sp.csr_matrix((np.ones(3), np.array([0, 1, 2]), np.array([0, 3])), shape=(1, 4000))
    sharding.distributed_topk(Model(), X, 1, k, prior=(0.05, -1.3, 0.2, None))
    assert taken == [route]


@pytest.mark.parametrize("world", [2, 3])
def test_every_collective_world_n_gloo(tmp_path, world):
    """tests/collectives_worker.py over gloo at world 2 / 3 (fresh torch.distributed.run children):
    every collective sharding.py issues -- the packed int32 / wide / f64 top-k exchanges, the f64
    row all-gather, the int64 MAX / MIN all-reduces, the module broadcast, the sharded table load
    with P not divisible by the world -- bit-identical to its numpy restatement. The GPU test
    (tests/test_gpu_rccl.py) runs the same worker over RCCL."""
    import _collectives
    res = _collectives.run(world, "gloo", str(tmp_path / "gloo.npz"))
    names = _collectives.assert_matches_expected(res, world, device_merges=False)
    assert len(names) == 17


def _tau_case(rank, k=5, m=7):
    """Rank r's lower-bound lists: u64 keys (score bits << 32 | ~id) sorted descending, some short."""
    rng = np.random.default_rng(100 + rank)
    keys = np.zeros((m, k), dtype=np.uint64)
    cnt = np.zeros(m, dtype=np.int32)
    for u in range(m):
        c = k if u % 3 else rng.integers(0, k + 1)
        sc = np.sort(rng.random(c).astype(np.float32))[::-1]
        ids = rng.choice(1000, c, replace=False) + 1000 * rank
        kk = (sc.view(np.uint32).astype(np.uint64) | np.uint64(0x80000000)) << np.uint64(32)
        kk |= (np.uint64(0xFFFFFFFF) - ids.astype(np.uint64))
        keys[u, :c] = np.sort(kk)[::-1]
        keys[u, c:] = np.uint64(0xDEADBEEFDEADBEEF)   # stale entries past the count are ignored
        cnt[u] = c
    return keys, cnt


def _worker_tau(rank, world, port, q):
    import torch.distributed as dist
    from poi_recommendation_models_amd.sharding import global_kth_keys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _rccl_calls_only(dist)
    keys, cnt = _tau_case(rank)
    tau = global_kth_keys(torch.from_numpy(keys.view(np.int64)), torch.from_numpy(cnt), 5)
    q.put((rank, tau.numpy().view(np.uint64)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_kth_lower_key_world_n(world):
    """The bounded route's global threshold: per user the k-th largest of every rank's valid
    lower-bound keys (unsigned order), 0 when the ranks hold fewer than k together."""
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_tau, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    cases = [_tau_case(r) for r in range(world)]
    for u in range(7):
        allk = sorted((int(kk) for keys, cnt in cases for kk in keys[u, :cnt[u]]), reverse=True)
        want = allk[4] if len(allk) >= 5 else 0
        for _, tau in res:
            assert int(tau[u]) == want
