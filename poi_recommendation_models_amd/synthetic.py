"""Seeded synthetic check-in data shaped like the reference's datasets.

The reference loads private datasets (`run.py:854`, `datasets.py:349-442`) that are not in
its repository, so every test and benchmark here runs on synthetic data with the same
structure:

* `train_matrix` -- a user x POI CSR matrix; a user's history is `indices[indptr[u]:indptr[u+1]]`
  in ascending POI order, exactly what `train_matrix.getrow(uid).indices` yields for a
  `dok_matrix(...).tocsr()` built by `datasets.Dataset.split_data` (`datasets.py:386-406`).
* `place_coords` -- float64 (lat, lng) per POI, uniform in a Tokyo-sized box
  (`datasets.py:407-415` reads them from `poi_coos.txt`).
* `region_of` -- POI -> region id (`businessRegionEmbedList`, `run.py:149-152`).
* `test_positive` / `val_positive` -- per-user lists of held-out POIs that are not in the
  training history (`datasets.py:400-402`).

History lengths are h_u ~ U{1..h_max}.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class CheckinData:
    num_users: int
    num_pois: int
    indptr: np.ndarray        # int64 [U+1]
    indices: np.ndarray       # int64 [nnz], ascending within each user
    place_coords: np.ndarray  # float64 [P, 2]
    region_of: np.ndarray     # int64 [P]
    num_regions: int
    test_positive: list
    val_positive: list

    def history(self, u: int) -> np.ndarray:
        return self.indices[self.indptr[u]:self.indptr[u + 1]]

    def hist_len(self) -> np.ndarray:
        return np.diff(self.indptr)

    def to_scipy(self):
        import scipy.sparse as sp
        data = np.ones(len(self.indices), dtype=np.float64)
        return sp.csr_matrix((data, self.indices, self.indptr),
                             shape=(self.num_users, self.num_pois))


def _distinct_sorted(rng: np.random.Generator, P: int, h: int) -> np.ndarray:
    if h * 4 < P:
        # rejection-free for sparse picks: oversample then unique
        while True:
            cand = np.unique(rng.integers(0, P, size=h + h // 2 + 8))
            if len(cand) >= h:
                pick = rng.choice(len(cand), size=h, replace=False)
                return np.sort(cand[pick])
    return np.sort(rng.choice(P, size=h, replace=False))


def make_checkins(num_users: int, num_pois: int, h_max: int, seed: int = 0,
                  num_regions: int = 1024, h_min: int = 1, n_test: int = 3,
                  n_val: int = 2, empty_positive_every: int = 0) -> CheckinData:
    """Seeded synthetic dataset (h_u ~ U{h_min..h_max}, distinct, sorted)."""
    rng = np.random.default_rng(seed)
    P = int(num_pois)
    h = rng.integers(h_min, h_max + 1, size=num_users)
    h = np.minimum(h, P - 1)
    indptr = np.zeros(num_users + 1, dtype=np.int64)
    np.cumsum(h, out=indptr[1:])
    indices = np.empty(int(indptr[-1]), dtype=np.int64)
    test_pos, val_pos = [], []
    for u in range(num_users):
        hist = _distinct_sorted(rng, P, int(h[u]))
        indices[indptr[u]:indptr[u + 1]] = hist
        if empty_positive_every and u % empty_positive_every == 0:
            test_pos.append([])
            val_pos.append([])
            continue
        # held-out positives outside the history (datasets.py:120-145 split semantics)
        extra = rng.integers(0, P, size=n_test + n_val + 8)
        extra = [int(x) for x in dict.fromkeys(extra.tolist()) if x not in set(hist.tolist())]
        test_pos.append(extra[:n_test])
        val_pos.append(extra[n_test:n_test + n_val])
    lat = 35.55 + 0.3 * rng.random(P)
    lng = 139.45 + 0.4 * rng.random(P)
    coords = np.stack([lat, lng], axis=1).astype(np.float64)
    region_of = rng.integers(0, num_regions, size=P).astype(np.int64)
    return CheckinData(num_users, P, indptr, indices, coords, region_of, num_regions,
                       test_pos, val_pos)


def init_nais_params(num_pois: int, embed_size: int, hidden: int, seed: int = 0,
                     emb_std: float = 0.01, variant: str = "basic",
                     num_regions: int = 0, bias_std: float = 0.0) -> dict:
    """float32 parameters with the reference's initialisation (model.py:30-38).

    Embeddings ~ N(0, emb_std) (0.01 is the reference init, 0.3 a 'trained-like' set);
    Linear weights use torch's default Kaiming-uniform bound 1/sqrt(fan_in); attn_layer1
    bias is zeroed (model.py:36-38). The dist_layer bias is zeroed too (model.py:227-229).
    `bias_std` > 0 draws the two biases from N(0, bias_std) instead, to exercise the bias
    path the way a trained model would. Keys are the reference state_dict names (model.py:15-26, 106-117, 198-215).
    """
    rng = np.random.default_rng(seed)
    f32 = np.float32
    p = {}
    if variant == "basic":
        d_item, din = embed_size, embed_size
    elif variant == "distance":
        d_item, din = embed_size, embed_size + 2
    else:
        d_item, din = embed_size // 2, embed_size
        if variant == "region_distance":
            din = embed_size + 2
    p["embed_history.weight"] = rng.normal(0, emb_std, (num_pois, d_item)).astype(f32)
    p["embed_target.weight"] = rng.normal(0, emb_std, (num_pois, d_item)).astype(f32)
    if variant not in ("basic", "distance"):
        p["embed_region.weight"] = rng.normal(0, emb_std, (num_regions, embed_size // 2)).astype(f32)
    b1 = 1.0 / np.sqrt(din)
    p["attn_layer1.weight"] = rng.uniform(-b1, b1, (hidden, din)).astype(f32)
    p["attn_layer1.bias"] = (rng.normal(0, bias_std, hidden) if bias_std > 0
                             else np.zeros(hidden)).astype(f32)
    b2 = 1.0 / np.sqrt(hidden)
    p["attn_layer2.weight"] = rng.uniform(-b2, b2, (1, hidden)).astype(f32)
    if variant in ("region_distance", "distance"):
        if variant == "region_distance":
            p["embed_distance.weight"] = rng.normal(0, 0.01, (1, embed_size)).astype(f32)
        bd = 1.0 / np.sqrt(2.0)
        p["dist_layer.weight"] = rng.uniform(-bd, bd, (2, 2)).astype(f32)
        p["dist_layer.bias"] = (rng.normal(0, bias_std, 2) if bias_std > 0
                                else np.zeros(2)).astype(f32)
    return p
