"""The torch-CPU restatement behind bench.py's cpu_baseline (oracle/torch_cpu.py) reproduces the
reference's own per-user scores and top-50 lists (tests/golden/catalog_basic.npz, captured from
validation.NAIS_validation by tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from _helpers import assert_topk_equivalent, load_golden, params_from
from oracle import torch_cpu


@pytest.mark.parametrize("tag", ["init", "trained"])
def test_torch_cpu_restatement_matches_reference(tag):
    z = load_golden("catalog_basic.npz")
    p = params_from(z, tag)
    P, U = int(z["num_pois"]), int(z["num_users"])
    m = torch_cpu.TorchNAIS(p)
    torch.set_num_threads(2)
    worst = 0.0
    for u in range(U):
        hist = z["indices"][z["indptr"][u]:z["indptr"][u + 1]]
        ids, sc, ncand = torch_cpu.recommend_user(m, hist, P, 50)
        assert ncand == P - len(hist)
        key = f"{tag}/full_scores_u{u}"
        if key in z.files:
            rows, cand = torch_cpu.candidates(hist, P)
            full = torch.cat([m(rows[i:i + 1024], cand[i:i + 1024]) for i in range(0, len(cand), 1024)])
            worst = max(worst, float(np.max(np.abs(full.numpy() - z[key]))))
        assert_topk_equivalent(z[f"{tag}/topk_ids"][u], z[f"{tag}/topk_scores"][u], ids, sc,
                               tie_ulps=4)
    assert worst <= 1e-6, worst


@pytest.mark.parametrize("tag", ["init", "trained"])
def test_torch_cpu_region_distance_matches_reference(tag):
    """The region_distance restatement behind bench.py's region_distance self-check reproduces the
    reference's own NAIS_region_distance_validation lists (catalog_region_distance.npz)."""
    z = load_golden("catalog_region_distance.npz")
    p = params_from(z, tag)
    P, U = int(z["num_pois"]), int(z["num_users"])
    m = torch_cpu.TorchNAISRegionDistance(p)
    torch.set_num_threads(2)
    worst = 0.0
    for u in range(U):
        hist = z["indices"][z["indptr"][u]:z["indptr"][u + 1]]
        cand, sc = torch_cpu.region_distance_scores(m, hist, P, z["region_of"], z["coords"])
        key = f"{tag}/full_scores_u{u}"
        if key in z.files:
            worst = max(worst, float(np.max(np.abs(sc - z[key]))))
        order = np.lexsort((cand, -sc.astype(np.float64)))[:50]
        assert_topk_equivalent(z[f"{tag}/topk_ids"][u], z[f"{tag}/topk_scores"][u], cand[order],
                               sc[order], tie_ulps=4)
    assert worst <= 1e-6, worst
