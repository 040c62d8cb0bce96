"""Debug: per-user catalog scores of the in-tree library vs the oracle for wide x3b shapes."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import nais_oracle
from poi_recommendation_models_amd.catalog import DeviceCSR, score_catalog
from poi_recommendation_models_amd.model import NAIS_basic
from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins

import os
SH = eval(os.environ.get('SHAPES', '((128, 64, 3), (64, 128, 3), (128, 128, 3), (128, 128, 40), (64, 128, 40))'))
for D, H, hmax in SH:
    P = 700
    data = make_checkins(3, P, hmax, seed=5)
    p = init_nais_params(P, D, H, seed=6, emb_std=0.3, bias_std=0.1)
    m = NAIS_basic(P, D, H, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to("cuda:0").eval()
    m.precision = "fp16x3"
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, torch.device("cuda:0"))
    full = score_catalog(m, csr, range(3), strategy="direct").cpu().numpy()
    for u in range(3):
        cand, ref = nais_oracle.catalog_scores_basic(p, data.history(u), P)
        d = np.abs(full[u][cand] - ref)
        print(D, H, hmax, u, "h", len(data.history(u)), "maxdiff %.3g" % d.max(), "argmax", cand[d.argmax()] % 256,
              "bad frac %.3f" % (d > 1e-4).mean())
