"""Data layer compatible with the reference's datasets.py: the same files, the
same split, vectorised (numpy) so that Gowalla-scale check-in files load in seconds.

Files (the reference's formats):
  checkins.txt            "uid lid time" per check-in            (datasets.py:361-365)
  poi_coos.txt            "lid lat lng" per POI                  (datasets.py:408-411)
  poi_region.txt          "poi<TAB>region"                       (datasets.py:84-87)
  poi_region_sorted.txt   "poi<TAB>dense region id" (csv, \\r\\n)  (datasets.py:146-181)

`Dataset(user_num, poi_num, directory_path).generate_data()` returns the reference's
(train_matrix, test_positive, val_positive, place_coords): per user, check-ins sorted by their
latest time (newest first, ties in order of first appearance in checkins.txt), the newest
int(0.2 L) are test, the next max(1, int(0.1 L)) validation, the rest train with their check-in counts (datasets.py:112-145,
373-402). The reference's O(P^2) side products -- POI_POI_Graph, user_POI_Graph (datasets.py:
378-379), dist_matrix and nearPOI (:417-418) -- are not built (none is on the NAIS path; at
P = 100k they are 80 GB each). `write_synthetic` writes a dataset directory in these formats.
"""
from __future__ import annotations

import csv
import os

import numpy as np
import scipy.sparse as sp

EARTH_RADIUS_M = 6371008.8   # the haversine package's mean Earth radius (6371.0088 km)


# ---------------------------------------------------------------- check-ins and the split
def read_checkins(path):
    """checkins.txt -> (uid int64, lid int64, time float64) arrays."""
    try:
        import pandas as pd
        df = pd.read_csv(path, sep=r"\s+", header=None, names=["u", "l", "t"],
                         dtype={"u": np.int64, "l": np.int64, "t": np.float64}, engine="c")
        return df["u"].to_numpy(), df["l"].to_numpy(), df["t"].to_numpy()
    except ImportError:
        a = np.loadtxt(path, dtype=np.float64, ndmin=2)
        return a[:, 0].astype(np.int64), a[:, 1].astype(np.int64), a[:, 2]


def raw_matrices(uid, lid, time, user_num, poi_num):
    """read_raw_data (datasets.py:361-371): check-in counts and, per (user, POI), the latest time
    (kept only if > 0, as the reference's dok update `if stored < time` starting from 0).
    Within a row, POIs are in order of their first check-in in the file -- dok_matrix.tocsr()
    keeps insertion order, and that order breaks time ties in the split."""
    uid, lid, time = np.asarray(uid, np.int64), np.asarray(lid, np.int64), np.asarray(time, np.float64)
    key = uid * poi_num + lid
    uk, first, inv, cnt = np.unique(key, return_index=True, return_inverse=True, return_counts=True)
    tmax = np.full(len(uk), -np.inf)
    np.maximum.at(tmax, inv, time)
    o = np.lexsort((first, uk // poi_num))            # by user, then first appearance
    rows, cols = uk[o] // poi_num, uk[o] % poi_num
    indptr = np.r_[0, np.cumsum(np.bincount(rows, minlength=user_num))]
    count = sp.csr_matrix((cnt[o].astype(np.float64), cols, indptr), shape=(user_num, poi_num))
    keep = tmax[o] > 0
    tind = np.r_[0, np.cumsum(np.bincount(rows[keep], minlength=user_num))]
    tmat = sp.csr_matrix((tmax[o][keep], cols[keep], tind), shape=(user_num, poi_num))
    return count, tmat


def split_with_time(count, tmat, test_size=0.2, val_size=0.1):
    """split_data + train_test_val_split_with_time (datasets.py:112-145, 373-402), vectorised."""
    count, tmat = count.tocsr(), tmat.tocsr()
    if count.nnz != tmat.nnz or not (np.array_equal(count.indptr, tmat.indptr)
                                     and np.array_equal(count.indices, tmat.indices)):
        raise ValueError("every (user, POI) needs a check-in time > 0: the reference pairs "
                         "count and time entries by position (datasets.py:383-387)")
    U, P = count.shape
    L = np.diff(count.indptr)
    rows = np.repeat(np.arange(U), L)
    # newest first within each row, ties in row (first check-in) order -- Python's stable sort
    o = np.argsort(-tmat.data, kind="stable")
    o = o[np.argsort(rows[o], kind="stable")]
    pos = np.arange(count.nnz) - np.repeat(count.indptr[:-1], L)   # rank within the row
    n_test = (L * test_size).astype(np.int64)                       # int(len(li) * test_size)
    n_val = np.maximum((L * val_size).astype(np.int64), 1)
    nt, nv = np.repeat(n_test, L), np.repeat(n_val, L)
    is_test = pos < nt
    is_val = (pos >= nt) & (pos < nt + nv)
    is_train = pos >= nt + nv
    place = count.indices[o].astype(np.int64)
    freq = count.data[o]
    # the reference fills train_matrix after random.shuffle(train), so its within-row order is
    # random (it only changes fp summation order downstream); here rows are ascending
    train = sp.csr_matrix((freq[is_train], (rows[is_train], place[is_train])), shape=(U, P))
    train.sum_duplicates()
    train.sort_indices()

    def lists(mask):
        cnt = np.bincount(rows[mask], minlength=U)
        return [x.tolist() for x in np.split(place[mask], np.cumsum(cnt)[:-1])]
    return train, lists(is_test), lists(is_val)


def read_poi_coos(path):
    """place_coords of datasets.py:404-416: rows in order of each lid's first appearance (dict
    insertion order), values from its last line. Returns a float64 [P, 2] array."""
    a = np.loadtxt(path, dtype=np.float64, ndmin=2)
    lid = a[:, 0].astype(np.int64)
    _, first = np.unique(lid, return_index=True)
    _, last_rev = np.unique(lid[::-1], return_index=True)
    last = len(lid) - 1 - last_rev
    order = np.argsort(first, kind="stable")
    return a[last[order]][:, 1:3].copy()


class Dataset:
    """datasets.Dataset (datasets.py:347-442) with the same constructor and methods."""

    def __init__(self, user_num, _poi_num, directory_path):
        self.user_num = user_num
        self.poi_num = _poi_num
        self.directory_path = directory_path
        self.checkin_file = "checkins.txt"
        self.poi_file = "poi_coos.txt"

    def read_raw_data(self):
        u, l, t = read_checkins(self.directory_path + self.checkin_file)
        return raw_matrices(u, l, t, self.user_num, self.poi_num)

    def split_data(self, raw_matrix, time_matrix, random_seed=0):
        return split_with_time(raw_matrix, time_matrix)

    def read_poi_coos(self, near_POI_num=50):
        self.place_coos = read_poi_coos(self.directory_path + self.poi_file).tolist()
        return self.place_coos

    def generate_data(self, random_seed=0, near_POI_num=50):
        raw_matrix, time_matrix = self.read_raw_data()
        train_matrix, test_positive, val_positive = self.split_data(raw_matrix, time_matrix, random_seed)
        place_coords = self.read_poi_coos(near_POI_num)
        return train_matrix, test_positive, val_positive, place_coords


# ---------------------------------------------------------------- regions
def get_region_num(path):
    """datasets.py:146-181: dense region ids (in order of the original ids) into
    poi_region_sorted.txt (poi order); returns the number of regions."""
    pairs = np.loadtxt(path + "poi_region.txt", dtype=np.int64, delimiter="\t", ndmin=2)
    o = np.argsort(pairs[:, 1], kind="stable")
    reg = pairs[o, 1]
    dense = np.r_[0, np.cumsum(reg[1:] != reg[:-1])]
    new = np.stack([pairs[o, 0], dense], 1)
    new = new[np.argsort(new[:, 0], kind="stable")]
    with open(path + "poi_region_sorted.txt", "w", newline="") as f:
        csv.writer(f, delimiter="\t").writerows(new.tolist())
    num = int(dense.max()) + 1
    print("region num: {}".format(num))
    return num


def read_region_list(path):
    """businessRegionEmbedList of run.py:149-152 (region id per POI, poi_region_sorted.txt)."""
    with open(path + "poi_region_sorted.txt") as f:
        return np.array([int(line.split("\t")[1].strip()) for line in f if line.strip()], np.int64)


def haversine_m(lat1, lng1, lat2, lng2):
    """The haversine package's great-circle distance in metres (vectorised)."""
    lat1, lng1, lat2, lng2 = (np.radians(np.asarray(x, np.float64)) for x in (lat1, lng1, lat2, lng2))
    lat, lng = lat2 - lat1, lng2 - lng1
    d = np.sin(lat * 0.5) ** 2 + np.cos(lat1) * np.cos(lat2) * np.sin(lng * 0.5) ** 2
    return 2 * EARTH_RADIUS_M * np.arcsin(np.sqrt(d))


def region_grid(place_coords, size):
    """Region id per POI (-1 if none) of get_region (datasets.py:7-83): a rownum x colnum grid of
    ~size-metre cells over the bounding box; a POI takes the first cell, in row-major order, whose
    band [lat_min_i, lat_max_i] holds it and whose (half-open, closed on the last row / column)
    bounds accept it. Vectorised over POIs per band."""
    pc = np.asarray(place_coords, np.float64)
    la, lo = pc[:, 0], pc[:, 1]
    la_min, la_max = min(55000, float(la.min())), max(-55000, float(la.max()))
    lo_min, lo_max = min(55000, float(lo.min())), max(-55000, float(lo.max()))
    w1 = float(haversine_m(la_max, lo_max, la_max, lo_min))
    w2 = float(haversine_m(la_min, lo_max, la_min, lo_min))
    h1 = float(haversine_m(la_max, lo_max, la_min, lo_max))
    colnum = int((w2 + w1) / 2 / size)
    rownum = int(h1 / size)
    alpha = (la_max - la_min) / rownum
    delta = (lo_max - lo_min) / colnum
    lng_max = np.array([lo_min + delta * (j + 1) for j in range(colnum)])
    region = np.full(len(pc), -1, np.int64)
    for i in range(rownum):
        lat_lo = la_min + alpha * i
        lat_hi = la_min + alpha * (i + 1)
        idx = np.nonzero((region < 0) & (la >= lat_lo) & (la <= lat_hi))[0]
        if len(idx) == 0:
            continue
        a, o = la[idx], lo[idx]
        strict = a < lat_hi
        last_row = i == rownum - 1
        # first j < colnum-1 with lng < lng_max_j (allowed if lat < lat_hi, or on the last row)
        j = np.searchsorted(lng_max[:-1], o, side="right")
        ok_inner = (j < colnum - 1) & (strict | last_row)
        # otherwise the last column: lng <= lng_max_last, and lat < lat_hi unless last row
        ok_last = ~ok_inner & (o <= lng_max[-1]) & (strict | last_row)
        jj = np.where(ok_inner, j, colnum - 1)
        take = ok_inner | ok_last
        region[idx[take]] = colnum * i + jj[take]
    return region


def get_region(place_coords, size, path):
    """get_region (datasets.py:7-87): writes poi_region.txt ("poi<TAB>region")."""
    region = region_grid(place_coords, size)
    with open(path + "poi_region.txt", "w") as f:
        for i, r in enumerate(region.tolist()):
            f.write("{}\t{}\n".format(i, int(r)))
    return region


# ---------------------------------------------------------------- synthetic datasets
def write_synthetic(path, user_num, poi_num, h_min=1, h_max=20, seed=0, box=(35.5, 35.8, 139.5, 139.9),
                    region_size=None, checkins_per_poi=(1, 3)):
    """A dataset directory in the reference's formats: checkins.txt (each user visits h ~ U{h_min..h_max}
    distinct POIs, 1-3 times each, unix-like times), poi_coos.txt (uniform in `box` =
    (lat0, lat1, lng0, lng1), a Tokyo-sized box by default) and, with region_size (metres),
    poi_region.txt from get_region. Returns the path."""
    os.makedirs(path, exist_ok=True)
    if not path.endswith("/"):
        path += "/"
    r = np.random.default_rng(seed)
    h = r.integers(h_min, h_max + 1, user_num)
    uid = np.repeat(np.arange(user_num), h)
    lid = np.concatenate([r.choice(poi_num, k, replace=False) for k in h]) if user_num else np.zeros(0, np.int64)
    reps = r.integers(checkins_per_poi[0], checkins_per_poi[1] + 1, len(uid))
    uid, lid = np.repeat(uid, reps), np.repeat(lid, reps)
    t = np.round(r.uniform(1.2e9, 1.3e9, len(uid)), 1)
    perm = r.permutation(len(uid))
    with open(path + "checkins.txt", "w") as f:
        f.writelines(f"{a}\t{b}\t{c!r}\n" for a, b, c in zip(uid[perm].tolist(), lid[perm].tolist(),
                                                           t[perm].tolist()))
    lat = r.uniform(box[0], box[1], poi_num)
    lng = r.uniform(box[2], box[3], poi_num)
    with open(path + "poi_coos.txt", "w") as f:
        f.writelines(f"{i}\t{a!r}\t{b!r}\n" for i, (a, b) in enumerate(zip(lat.tolist(), lng.tolist())))
    if region_size:
        get_region(np.stack([lat, lng], 1), region_size, path)
    return path
