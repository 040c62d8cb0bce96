"""Golden fixtures for the data layer, produced by the REFERENCE's own
datasets.py on synthetic files in the reference's formats. Run here only (needs /root/reference):

    python tests/golden/make_golden_datasets.py [/root/reference]

Writes tests/golden/datasets.npz:
  case{0,1}/checkins_{uid,lid,time}   the checkins.txt rows ("uid lid time", datasets.py:361-365)
  case{0,1}/train_{indptr,indices,data}  Dataset.split_data's train_matrix (datasets.py:368-402)
  case{0,1}/{test,val}_{flat,len}     its test_positive / val_positive lists
  region/poi, region/region           poi_region.txt ("poi\\tregion", datasets.py:84-87)
  region/sorted, region/num           get_region_num's poi_region_sorted.txt and count (:146-181)
Dataset.read_poi_coos and get_region call `haversine` (not installed), so they are not run here;
their restatements are tested against pure-Python loops in tests/test_data.py (parity unpinned
for the haversine formula itself).
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402


def synth_checkins(rng, U, P, max_pois, empty_users=(), tie_every=0):
    rows = []
    for u in range(U):
        if u in empty_users:
            continue
        k = int(rng.integers(1, max_pois + 1))
        pois = rng.choice(P, k, replace=False)
        for lid in pois:
            for _ in range(int(rng.integers(1, 4))):
                t = float(np.round(rng.uniform(1.2e9, 1.3e9), 1))
                rows.append((u, int(lid), t))
        if tie_every and u % tie_every == 0 and k > 2:   # equal max times inside a user
            t0 = float(np.round(rng.uniform(1.2e9, 1.3e9), 1))
            rows.append((u, int(pois[0]), t0 + 1e8))
            rows.append((u, int(pois[1]), t0 + 1e8))
    order = rng.permutation(len(rows))
    return [rows[i] for i in order]


def main(ref_path="/root/reference"):
    load_reference(ref_path)
    import datasets
    rng = np.random.default_rng(77)
    out = {}
    cases = [dict(U=80, P=400, max_pois=40, empty_users=(), tie_every=7),
             dict(U=50, P=300, max_pois=12, empty_users=(3, 17, 49), tie_every=0)]
    for ci, c in enumerate(cases):
        rows = synth_checkins(rng, c["U"], c["P"], c["max_pois"], set(c["empty_users"]), c["tie_every"])
        with tempfile.TemporaryDirectory() as d:
            with open(os.path.join(d, "checkins.txt"), "w") as f:
                for u, lid, t in rows:
                    f.write(f"{u}\t{lid}\t{t}\n")
            ds = datasets.Dataset(c["U"], c["P"], d + "/")
            raw, tm = ds.read_raw_data()
            train, test_pos, val_pos = ds.split_data(raw, tm)
        pre = f"case{ci}/"
        out[pre + "checkins_uid"] = np.array([r[0] for r in rows], np.int64)
        out[pre + "checkins_lid"] = np.array([r[1] for r in rows], np.int64)
        out[pre + "checkins_time"] = np.array([r[2] for r in rows], np.float64)
        out[pre + "shape"] = np.array([c["U"], c["P"]], np.int64)
        train = train.tocsr()
        out[pre + "train_indptr"] = train.indptr.astype(np.int64)
        out[pre + "train_indices"] = train.indices.astype(np.int64)
        out[pre + "train_data"] = train.data.astype(np.float64)
        for name, lst in (("test", test_pos), ("val", val_pos)):
            out[pre + name + "_flat"] = np.array([int(x) for l in lst for x in l], np.int64)
            out[pre + name + "_len"] = np.array([len(l) for l in lst], np.int64)
    # get_region_num: region ids sparse and unordered, POIs listed in file order
    P = 300
    reg = rng.choice(np.arange(10, 5000, 7), 40, replace=False)
    region = reg[rng.integers(0, len(reg), P)]
    poi = rng.permutation(P)
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "poi_region.txt"), "w") as f:
            for p_, r_ in zip(poi, region):
                f.write(f"{p_}\t{r_}\n")
        num = datasets.get_region_num(d + "/")
        with open(os.path.join(d, "poi_region_sorted.txt")) as f:
            srt = [[int(x) for x in line.strip().split("\t")] for line in f if line.strip()]
    out["region/poi"] = poi.astype(np.int64)
    out["region/region"] = region.astype(np.int64)
    out["region/sorted"] = np.array(srt, np.int64)
    out["region/num"] = np.int64(num)
    np.savez_compressed(os.path.join(HERE, "datasets.npz"), **out)
    print("wrote", os.path.join(HERE, "datasets.npz"))


if __name__ == "__main__":
    main(*sys.argv[1:])
