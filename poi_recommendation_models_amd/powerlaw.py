"""Power-law geographical prior (same API and semantics as powerLaw.py:7-92).

`PowerLaw.fit_distance_distribution` builds the pair-distance histogram of every user's
history on the GPU (`nais_distance_histogram`, the reference's O(sum h^2) Python double loop,
powerLaw.py:41-55) and runs the reference's 2000-step gradient descent on the host
(powerLaw.py:66-84, same float64 arithmetic, same `np.random.random()` initialisation).
`prior_rows` / `catalog.score_topk(..., prior=(a, b, alpha, coords))` evaluate
`predict` for whole catalogs on the device (`nais_powerlaw_prior`). `dist`, `pr_d` and
`predict` are also provided as host scalar functions with the reference's exact formula.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from . import _capi


def dist(loc1, loc2):                                          # powerLaw.py:7-21
    lat1, long1 = loc1[0], loc1[1]
    lat2, long2 = loc2[0], loc2[1]
    if abs(lat1 - lat2) < 1e-6 and abs(long1 - long2) < 1e-6:
        return 0.0
    d2r = math.pi / 180.0
    phi1, phi2 = (90.0 - lat1) * d2r, (90.0 - lat2) * d2r
    theta1, theta2 = long1 * d2r, long2 * d2r
    cos = (math.sin(phi1) * math.sin(phi2) * math.cos(theta1 - theta2) +
           math.cos(phi1) * math.cos(phi2))
    return math.acos(cos) * 6371


def read_poi_coos(poi_file):                                   # powerLaw.py:23-30
    poi_coos = {}
    for line in open(poi_file, "r").readlines():
        lid, lat, lng = line.strip().split()
        poi_coos[int(lid)] = (float(lat), float(lng))
    return poi_coos


def distance_histogram(check_in_matrix, poi_coos, device="cuda", nbins=20100):
    """Counts of int(dist) over all history pairs i < j of all users (GPU); returns a dict."""
    from .catalog import device_csr
    dev = torch.device(device)
    csr = device_csr(check_in_matrix, dev)
    coords = torch.as_tensor(np.ascontiguousarray(np.asarray(poi_coos, dtype=np.float64))).to(dev)
    hist = torch.empty(nbins, dtype=torch.int64, device=dev)
    over = torch.empty(1, dtype=torch.int64, device=dev)
    rc = _capi.load().nais_distance_histogram(coords.data_ptr(), csr.indptr.data_ptr(),
                                              csr.indices.data_ptr(), csr.shape[0], hist.data_ptr(),
                                              nbins, over.data_ptr(), _capi.stream_handle(dev))
    _capi.check(rc, "nais_distance_histogram")
    if int(over.item()) != 0:
        raise ValueError(f"{int(over.item())} pair distances are NaN (acos domain) or >= {nbins} km")
    h = hist.cpu().numpy()
    return {int(k): int(h[k]) for k in np.nonzero(h)[0]}


class PowerLaw(object):                                        # powerLaw.py:32-92
    def __init__(self, a=None, b=None):
        self.a = a
        self.b = b
        self.check_in_matrix = None
        self.visited_lids = {}
        self.poi_coos = None

    @staticmethod
    def compute_distance_distribution(check_in_matrix, poi_coos, device="cuda"):
        counts = distance_histogram(check_in_matrix, poi_coos, device)
        total = 1.0 * sum(counts.values())
        distribution = sorted(((k, v / total) for k, v in counts.items()), key=lambda kv: kv[0])
        return zip(*distribution[1:])

    def fit_distance_distribution(self, check_in_matrix, poi_coos, device="cuda"):
        self.check_in_matrix = check_in_matrix
        for uid in range(check_in_matrix.shape[0]):
            self.visited_lids[uid] = check_in_matrix.getrow(uid).indices
        ctime = time.time()
        print("Fitting distance distribution...", )
        self.poi_coos = poi_coos
        x, t = self.compute_distance_distribution(check_in_matrix, poi_coos, device)
        x = np.log10(x)
        t = np.log10(t)
        w0, w1 = np.random.random(), np.random.random()
        max_iterations, lambda_w, alpha = 2000, 0.1, 1e-5
        for _ in range(max_iterations):
            d_w0, d_w1 = 0.0, 0.0
            for n in range(len(x)):
                d_w0 += (w0 + w1 * x[n] - t[n])
                d_w1 += (w0 + w1 * x[n] - t[n]) * x[n]
            w0 -= alpha * (d_w0 + lambda_w * w0)
            w1 -= alpha * (d_w1 + lambda_w * w1)
        print("Done. Elapsed time:", time.time() - ctime, "s")
        self.a, self.b = 10 ** w0, w1

    def pr_d(self, d):                                         # powerLaw.py:86-88
        d = max(0.01, d)
        return self.a * (d ** self.b)

    def predict(self, uid, lj):                                # powerLaw.py:90-92
        lj = self.poi_coos[lj]
        return np.prod([self.pr_d(dist(self.poi_coos[li], lj)) for li in self.visited_lids[uid]])
