"""Debug, one process: the column-sharded prior route (P = 1002, shards [0, 501) and [501, 1002))
with the collectives replaced by local captures, against the single-process pairs route and the
per-user prior rows (nais_powerlaw_prior) -- where does each user's max G come from."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_distributed import _data, _model  # noqa: E402
from poi_recommendation_models_amd import sharding  # noqa: E402
from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs, prior_rows  # noqa: E402

data, p = _data("shared_odd")
P, U = data.num_pois, data.num_users
m = _model(p, P)
dev = torch.device("cuda:0")
csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
prior = (0.052, -1.37, 0.2, data.place_coords)
G, gm_rows = prior_rows(csr, range(U), prior[0], prior[1], data.place_coords, dev)
G, gm_rows = G.cpu().numpy(), gm_rows.cpu().numpy()
cap = {}
sharding.agree_min = lambda v, d, g=None: v


def run(cols, force=None):
    def ar(bits, group=None):
        cap[cols] = bits.view(torch.float64).cpu().numpy().copy()
        if force is not None:
            bits.copy_(torch.as_tensor(force, device=bits.device).view(torch.int64))
        return bits
    sharding.allreduce_gmax = ar
    return _score_topk_pairs(m, csr, range(U), 50, None, None, None, None, force=True, cols=cols,
                             prior=prior, group=object(), return_keys=True)


run((0, 501))
run((501, 1002))
gl = np.maximum(cap[(0, 501)], cap[(501, 1002)])
print("local max rank0 / rank1 vs per-user rows max (first 12 users):")
for u in range(12):
    g = G[u]
    print(u, cap[(0, 501)][u], cap[(501, 1002)][u], "rows:", gm_rows[u],
          "argmax col", int(np.argmax(np.where(g >= 0, g, -1))), "max rows[0:501]",
          float(np.max(np.where(g[:501] >= 0, g[:501], -1))), "max rows[501:]",
          float(np.max(np.where(g[501:] >= 0, g[501:], -1))))
print("users where the sharded max differs from the rows' max:",
      [int(u) for u in np.nonzero(gl != gm_rows)[0]])
