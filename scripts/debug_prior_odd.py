"""Debug: the column-sharded prior route at P = 1002 (two shards of 501 columns) against the
single-process pairs route -- per-shard lists with their f64 keys, the first users that differ."""
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_distributed import _data, _free_port, _model  # noqa: E402

KIND = sys.argv[1] if len(sys.argv) > 1 else "shared_odd"


def worker(rank, world, port, out):
    import torch.distributed as dist
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs
    from poi_recommendation_models_amd.sharding import column_blocks
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data, p = _data(KIND)
    m = _model(p, data.num_pois)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
    c0, c1 = column_blocks(data.num_pois, world)[rank]
    prior = (0.052, -1.37, 0.2, data.place_coords)
    ev = []
    ids, sc, keys = _score_topk_pairs(m, csr, range(data.num_users), 50, None, None, None, None, force=True,
                                      cols=(c0, c1), prior=prior, group=dist.group.WORLD, return_keys=True,
                                      events=ev)
    plan = {k: v for k, _, _, v in ev if _ is None}
    print(rank, plan, flush=True)
    np.savez(f"{out}_{rank}.npz", ids=ids.cpu().numpy(), sc=sc.cpu().numpy(), keys=keys.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "p")
        mp.start_processes(worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
        res = [dict(np.load(f"{out}_{r}.npz")) for r in range(2)]
    data, p = _data(KIND)
    m = _model(p, data.num_pois)
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, data.num_pois, torch.device("cuda:0"))
    prior = (0.052, -1.37, 0.2, data.place_coords)
    ev = []
    ids, sc, keys = _score_topk_pairs(m, csr, range(data.num_users), 900, None, None, None, None,
                                      force=True, prior=prior, return_keys=True, events=ev)
    print("single plan", {k: v for k, _, _, v in ev if _ is None})
    ids, keys = ids.cpu().numpy(), keys.cpu().numpy()
    lut = [dict(zip(ids[u].tolist(), keys[u].tolist())) for u in range(len(ids))]
    bad = 0
    for r in range(2):
        for u in range(len(res[r]["ids"])):
            for i, c in enumerate(res[r]["ids"][u].tolist()):
                kk = res[r]["keys"][u][i]
                ref = lut[u].get(c)
                if ref is None or not (ref == kk or (np.isnan(ref) and np.isnan(kk))):
                    bad += 1
                    if bad <= 12:
                        print(f"rank {r} user {u} pos {i} id {c} key {kk!r} single {ref!r}")
    print("mismatched (id, key) entries:", bad)


if __name__ == "__main__":
    main()
