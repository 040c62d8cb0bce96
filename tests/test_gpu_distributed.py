"""GPU, 2 processes on the box's one GPU over gloo: the multi-GPU evaluation entry points
(sharding.distributed_topk / NAIS_validation_distributed) give every rank the single-process
result -- through the column-sharded pairs route when the histories share POIs and through the
user-sharded per-user kernels when they do not (sharding.distributed_plan)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _data(kind):
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins
    if kind == "shared":          # 200 users x U{1..80} items over 2,000 POIs: sharing ~4
        data = make_checkins(200, 2000, 80, seed=21)
    elif kind == "shared_odd":    # 1,002 POIs: two column shards of 501, narrower than a table
        data = make_checkins(200, 1002, 80, seed=21)    # block and odd (pitch rounded up to 504)
    else:                         # 12 users, little overlap: sharing ~1
        data = make_checkins(12, 3000, 30, seed=22)
    p = init_nais_params(data.num_pois, 32, 32, seed=23, emb_std=0.3, bias_std=0.1)
    return data, p


def _model(p, P):
    from poi_recommendation_models_amd.model import NAIS_basic
    m = NAIS_basic(P, 32, 32, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m.precision = "fp16x6"
    return m.to("cuda:0").eval()


def _worker(rank, world, port, kind, out):
    import torch.distributed as dist
    from poi_recommendation_models_amd import sharding
    from poi_recommendation_models_amd.catalog import DeviceCSR
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data, p = _data(kind)
    m = _model(p, data.num_pois)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
    plan = sharding.distributed_plan(csr, data.num_users, data.num_pois, 50, world, m)
    ids, sc = sharding.distributed_topk(m, csr, data.num_users, 50)
    np.savez(f"{out}_{rank}.npz", ids=ids.cpu().numpy(), sc=sc.cpu().numpy(), plan=plan)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind,plan", [("shared", "pairs"), ("shared_odd", "pairs"), ("sparse", "users")])
def test_distributed_topk_two_ranks_equal_single(kind, plan):
    import torch.multiprocessing as mp
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r")
        mp.start_processes(_worker, args=(2, _free_port(), kind, out), nprocs=2, join=True,
                           start_method="spawn")
        res = [np.load(f"{out}_{r}.npz") for r in range(2)]
        data, p = _data(kind)
        m = _model(p, data.num_pois)
        csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
        ids, sc = score_topk(m, csr, range(data.num_users), 50,
                             strategy="pairs" if plan == "pairs" else "direct")
        for r in res:
            assert str(r["plan"]) == plan
            np.testing.assert_array_equal(r["ids"], ids.cpu().numpy())
            np.testing.assert_array_equal(r["sc"], sc.cpu().numpy())


def _positives(data, seed):
    rng = np.random.default_rng(seed)
    return [[int(x) for x in rng.choice(data.num_pois, 5, replace=False)] for _ in range(data.num_users)]


def _worker_validation(rank, world, port, kind, out):
    """validation.NAIS_validation itself, called by every rank inside the process group with the
    distributed route switched on (NAIS_DISTRIBUTED_EVAL=1: run.py's call sites unchanged)."""
    import torch.distributed as dist
    from poi_recommendation_models_amd import validation as V
    torch.cuda.set_device(0)
    os.environ["NAIS_DISTRIBUTED_EVAL"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data, p = _data(kind)
    m = _model(p, data.num_pois)

    class Args:
        topk = 50
    got = V.NAIS_validation(m, Args(), data.num_users, _positives(data, 1), _positives(data, 2),
                            data.to_scipy(), [5, 10, 20, 50])
    np.savez(f"{out}_{rank}.npz", got=np.array(got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["shared", "sparse"])
def test_validation_autoroute_two_ranks_equal_single(kind):
    """run.py:112-116 unchanged under torchrun + NAIS_DISTRIBUTED_EVAL=1: NAIS_validation in a 2-rank group (column-sharded
    pairs or user-sharded route) returns the single-process 6-tuple on every rank."""
    import torch.multiprocessing as mp
    from poi_recommendation_models_amd import validation as V
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "v")
        mp.start_processes(_worker_validation, args=(2, _free_port(), kind, out), nprocs=2, join=True,
                           start_method="spawn")
        res = [np.load(f"{out}_{r}.npz")["got"] for r in range(2)]
    data, p = _data(kind)
    m = _model(p, data.num_pois)

    class Args:
        topk = 50
    ref = np.array(V.NAIS_validation(m, Args(), data.num_users, _positives(data, 1),
                                     _positives(data, 2), data.to_scipy(), [5, 10, 20, 50]))
    for r in res:
        np.testing.assert_array_equal(r, ref)


def _worker_prior(rank, world, port, out, kind="shared"):
    import torch.distributed as dist
    from poi_recommendation_models_amd import sharding
    from poi_recommendation_models_amd.catalog import DeviceCSR
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data, p = _data(kind)
    m = _model(p, data.num_pois)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
    plan = sharding.distributed_plan(csr, data.num_users, data.num_pois, 50, world, m)
    prior = (0.052, -1.37, 0.2, data.place_coords)
    ids, sc = sharding.distributed_topk(m, csr, data.num_users, 50, prior=prior)
    np.savez(f"{out}_{rank}.npz", ids=ids.cpu().numpy(), sc=sc.cpu().numpy(), plan=plan)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["shared", "shared_odd"])
def test_distributed_prior_column_shards_equal_single(kind):
    """the power-law prior no longer drops to user sharding at N > 1: two ranks
    own half the POI columns each, normalise by the all-reduced max G and merge on the f64 blended
    score -- ids and scores identical to the single-process blend of the pairs route."""
    import torch.multiprocessing as mp
    from poi_recommendation_models_amd.catalog import DeviceCSR, score_topk
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "p")
        mp.start_processes(_worker_prior, args=(2, _free_port(), out, kind), nprocs=2, join=True,
                           start_method="spawn")
        res = [np.load(f"{out}_{r}.npz") for r in range(2)]
    data, p = _data(kind)
    m = _model(p, data.num_pois)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
    prior = (0.052, -1.37, 0.2, data.place_coords)
    # bit-identical to the single-process pairs route (the same per-pair arithmetic and sums)
    ids, sc = score_topk(m, csr, range(data.num_users), 50, prior=prior, strategy="pairs")
    for r in res:
        assert str(r["plan"]) == "pairs"
        np.testing.assert_array_equal(r["ids"], ids.cpu().numpy())
        np.testing.assert_array_equal(r["sc"], sc.cpu().numpy())
    # the direct route sums in another order (ulps): same lists up to the tie rule
    from _helpers import assert_topk_equivalent
    di, ds = score_topk(m, csr, range(data.num_users), 50, prior=prior, strategy="direct")
    di, ds = di.cpu().numpy(), ds.cpu().numpy()
    for u in range(data.num_users):
        assert_topk_equivalent(di[u], ds[u], res[0]["ids"][u], res[0]["sc"][u], tie_ulps=4)


def test_topk_merge_f64_kernel():
    """nais_topk_merge_f64 against a numpy restatement: equal keys (ties by id), NaN keys first,
    padding (id -1) last, short rows, m not a power of two."""
    from oracle import nais_oracle
    from poi_recommendation_models_amd import _capi
    rng = np.random.default_rng(5)
    n, m, k = 37, 3 * 50, 50
    keys = np.round(rng.random((n, m)), 3)                   # many exact ties
    ids = np.stack([rng.permutation(100_000)[:m] for _ in range(n)]).astype(np.int64)
    keys[0, :7] = np.nan
    ids[1, 40:] = -1                                         # 40 valid candidates < k
    keys[2] = 0.5
    kt, it = torch.as_tensor(keys, device=DEV_), torch.as_tensor(ids, device=DEV_)
    oi = torch.empty(n, k, dtype=torch.int64, device=DEV_)
    os_ = torch.empty(n, k, dtype=torch.float32, device=DEV_)
    ok_ = torch.empty(n, k, dtype=torch.float64, device=DEV_)
    _capi.check(_capi.load().nais_topk_merge_f64(kt.data_ptr(), it.data_ptr(), n, m, k, oi.data_ptr(),
                                                 os_.data_ptr(), ok_.data_ptr(),
                                                 _capi.stream_handle(DEV_)), "merge")
    oi, os_, ok_ = oi.cpu().numpy(), os_.cpu().numpy(), ok_.cpu().numpy()
    for r in range(n):
        valid = ids[r] >= 0
        rid, rk = nais_oracle.topk_ids(ids[r][valid], keys[r][valid], k)
        np.testing.assert_array_equal(oi[r, :len(rid)], rid)
        np.testing.assert_array_equal(ok_[r, :len(rid)], rk)
        np.testing.assert_array_equal(os_[r, :len(rid)], rk.astype(np.float32))
        assert np.all(oi[r, len(rid):] == -1) and np.isnan(ok_[r, len(rid):]).all()


DEV_ = torch.device("cuda:0")
