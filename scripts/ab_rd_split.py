#!/usr/bin/env python3
"""A/B of the table / gather CU split for bench.py's region_distance leg (config 4, the leg's
params), interleaved: python scripts/ab_rd_split.py CUS [CUS ...] (-1 = the model's pick)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poi_recommendation_models_amd import catalog  # noqa: E402
from poi_recommendation_models_amd.catalog import DeviceCSR, _score_topk_pairs  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_region_distance_Embedding  # noqa: E402
from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins  # noqa: E402

dev = torch.device("cuda", 0)
U, P, D, H, K = 50_000, 100_000, 64, 64, 50
data = make_checkins(U, P, 200, seed=2024)
p = init_nais_params(P, D, H, seed=11, emb_std=0.3, bias_std=0.1, variant="region_distance", num_regions=1024)
m = NAIS_region_distance_Embedding(P, D, H, 0.5, 1024, 1)
m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
m = m.to(dev).eval()
m.report_nan = False
csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
users = np.arange(U)
for rnd in range(2):
    for c in (int(x) for x in sys.argv[1:]):
        catalog.PAIR_TABLE_CUS = c
        job = lambda ev=None: _score_topk_pairs(m, csr, users, K, data.region_of, data.place_coords, None, None,
                                                force=True, events=ev)
        job()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(3):
            ev = []
            job(ev)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t) / 3 * 1e3
        cus = [n for k_, a, b, n in ev if k_ == "table_cus"]
        print("round", rnd, "table_cus", c, "->", cus, "ms %.1f" % ms, flush=True)
