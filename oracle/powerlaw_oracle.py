"""CPU oracle for the power-law geo prior -- TEST INFRASTRUCTURE ONLY.

Pure-Python float64 restatement of `powerLaw.py` (reference), used as the parity checker
for the device prior epilogue. Only tests/, smoke() and bench.py's cpu_baseline import it.

* `dist`        <- powerLaw.py:7-21 (spherical law of cosines, 1e-6 early-out)
* `pr_d`        <- powerLaw.py:86-88
* `predict`     <- powerLaw.py:90-92 (np.prod over the CSR-order history)
* `normalize`   <- run.py:55-59
* `blend`       <- run.py:537-539 (commented in the reference; f32 prediction, f64 prior)
* `fit`         <- powerLaw.py:41-84 (histogram of int-km pair distances + 2000-step GD)
"""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np


def dist(loc1, loc2):
    lat1, long1 = loc1[0], loc1[1]
    lat2, long2 = loc2[0], loc2[1]
    if abs(lat1 - lat2) < 1e-6 and abs(long1 - long2) < 1e-6:
        return 0.0
    d2r = math.pi / 180.0
    phi1 = (90.0 - lat1) * d2r
    phi2 = (90.0 - lat2) * d2r
    theta1 = long1 * d2r
    theta2 = long2 * d2r
    cos = (math.sin(phi1) * math.sin(phi2) * math.cos(theta1 - theta2) +
           math.cos(phi1) * math.cos(phi2))
    return math.acos(cos) * 6371


def pr_d(a, b, d):
    d = max(0.01, d)
    return a * (d ** b)


def predict(a, b, coords, history, poi):
    lj = coords[poi]
    return np.prod([pr_d(a, b, dist(coords[li], lj)) for li in history])


def normalize(scores):
    max_score = max(scores)
    if not max_score == 0:
        scores = [s / max_score for s in scores]
    return scores


def blend(pred_f32, prior_f64, alpha):
    """(1-alpha)*prediction + alpha*G: the f32 term is formed in f32, the sum in f64."""
    lhs = (np.asarray(pred_f32, dtype=np.float32) * np.float32(1 - alpha)).astype(np.float32)
    return lhs.astype(np.float64) + alpha * np.asarray(prior_f64, dtype=np.float64)


def distance_distribution(indptr, indices, coords):
    distribution = defaultdict(int)
    for u in range(len(indptr) - 1):
        lids = indices[indptr[u]:indptr[u + 1]]
        for i in range(len(lids)):
            for j in range(i + 1, len(lids)):
                distribution[int(dist(coords[lids[i]], coords[lids[j]]))] += 1
    total = 1.0 * sum(distribution.values())
    for k in distribution:
        distribution[k] /= total
    distribution = sorted(distribution.items(), key=lambda kv: kv[0])
    return zip(*distribution[1:])


def fit(indptr, indices, coords, w0, w1, max_iterations=2000):
    """powerLaw.py:57-84 with the two np.random.random() draws passed in explicitly."""
    x, t = distance_distribution(indptr, indices, coords)
    x = np.log10(x)
    t = np.log10(t)
    lambda_w, alpha = 0.1, 1e-5
    for _ in range(max_iterations):
        d_w0, d_w1 = 0.0, 0.0
        for n in range(len(x)):
            d_w0 += (w0 + w1 * x[n] - t[n])
            d_w1 += (w0 + w1 * x[n] - t[n]) * x[n]
        w0 -= alpha * (d_w0 + lambda_w * w0)
        w1 -= alpha * (d_w1 + lambda_w * w1)
    return 10 ** w0, w1
