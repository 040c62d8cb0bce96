"""CPU oracle for the data layer -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement, loop for loop, of the reference's datasets.py, used to check the
vectorised product loader (poi_recommendation_models_amd/data.py) on inputs larger than the
golden fixtures:

* `read_raw_data`     <- datasets.py:361-371 (count matrix + per-(user, POI) max time > 0)
* `split_data`        <- datasets.py:373-402 with train_test_val_split_with_time :112-145
* `read_poi_coos`     <- datasets.py:404-416 (dict insertion order; the O(P^2) dist_matrix /
                         nearPOI of :417-418 are not built)
* `get_region_num`    <- datasets.py:146-181
* `get_region`        <- datasets.py:7-87, with `haversine` restated from the haversine
                         package's published formula (mean Earth radius 6371.0088 km): the
                         package is not installed, so this part is "parity unpinned".
Pinned against tests/golden/datasets.npz (made by running the reference's datasets.py).
"""
from __future__ import annotations

import math


def read_raw_data(rows):
    """rows: iterable of (uid, lid, time). Returns (count, tmax) dicts keyed (uid, lid)."""
    count, tmax = {}, {}
    for uid, lid, t in rows:
        count[(uid, lid)] = count.get((uid, lid), 0.0) + 1
        if tmax.get((uid, lid), 0.0) < t:
            tmax[(uid, lid)] = t
    return count, tmax


def split_data(count, tmax, U, test_size=0.2, val_size=0.1):
    """Returns (train dict {(u, lid): freq}, test_positive, val_positive)."""
    by_user = {}
    for (u, l) in count:               # dok -> csr keeps insertion (first check-in) order
        by_user.setdefault(u, []).append(l)
    train, test_pos, val_pos = {}, [], []
    for u in range(U):
        places = by_user.get(u, [])
        freq = [count[(u, l)] for l in places]
        times = [tmax[(u, l)] for l in places]
        li = [(places[i], times[i], freq[i]) for i in range(len(places))]
        li.sort(key=lambda x: -x[1])
        test = li[:int(len(li) * test_size)]
        train_ = li[int(len(li) * test_size):]
        val_num = int(len(li) * val_size)
        if val_num == 0:
            val_num = 1
        val = train_[:val_num]
        for p, _, f in train_[val_num:]:
            train[(u, p)] = f
        test_pos.append([p for p, _, _ in test])
        val_pos.append([p for p, _, _ in val])
    return train, test_pos, val_pos


def read_poi_coos(lines):
    poi_coos = {}
    for line in lines:
        lid, lat, lng = line.strip().split()
        poi_coos[int(lid)] = (float(lat), float(lng))
    return [[v[0], v[1]] for v in poi_coos.values()]


def get_region_num(pairs):
    """pairs: [(poi, region)] in file order. Returns (sorted [(poi, idx)], count)."""
    data = [[int(p), int(r)] for p, r in pairs]
    data.sort(key=lambda x: x[1])
    idx, before, new = 0, data[0][1], []
    for p, r in data:
        if r != before:
            idx += 1
            before = r
        new.append([p, idx])
    new.sort(key=lambda x: x[0])
    return new, max(new, key=lambda x: x[1])[1] + 1


def haversine_m(p1, p2):
    lat1, lng1, lat2, lng2 = map(math.radians, (p1[0], p1[1], p2[0], p2[1]))
    lat, lng = lat2 - lat1, lng2 - lng1
    d = math.sin(lat * 0.5) ** 2 + math.cos(lat1) * math.cos(lat2) * math.sin(lng * 0.5) ** 2
    return 2 * 6371008.8 * math.asin(math.sqrt(d))


def get_region(place_coords, size):
    """Region id per POI (-1 if none), the grid walk of datasets.py:7-83."""
    la_max, la_min, lo_max, lo_min = -55000, 55000, -55000, 55000
    places = []
    for lid in range(len(place_coords)):
        la, lo = place_coords[lid]
        la_min, la_max = min(la_min, la), max(la_max, la)
        lo_min, lo_max = min(lo_min, lo), max(lo_max, lo)
        places.append((lid, la, lo))
    w1 = haversine_m((la_max, lo_max), (la_max, lo_min))
    w2 = haversine_m((la_min, lo_max), (la_min, lo_min))
    h1 = haversine_m((la_max, lo_max), (la_min, lo_max))
    colnum = int((w2 + w1) / 2 / size)
    rownum = int(h1 / size)
    alpha = (la_max - la_min) / rownum
    delta = (lo_max - lo_min) / colnum
    region = [-1] * len(place_coords)
    for i in range(rownum):
        lat_min = la_min + alpha * i
        lat_max = la_min + alpha * (i + 1)
        target = [x for x in places if lat_min <= x[1] <= lat_max]
        for j in range(colnum):
            lng_max = lo_min + delta * (j + 1)
            for lid, la, lo in target:
                if region[lid] >= 0:
                    continue
                if lo < lng_max and la < lat_max:
                    region[lid] = colnum * i + j
                elif j == colnum - 1 and i == rownum - 1:
                    if lo <= lng_max and la <= lat_max:
                        region[lid] = colnum * i + j
                elif j == colnum - 1:
                    if lo <= lng_max and la < lat_max:
                        region[lid] = colnum * i + j
                elif i == rownum - 1:
                    if lo < lng_max and la <= lat_max:
                        region[lid] = colnum * i + j
    return region
