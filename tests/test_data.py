"""Data layer: poi_recommendation_models_amd/data.py against the reference's own
datasets.py outputs (tests/golden/datasets.npz) and against the loop-level restatement in
oracle/datasets_oracle.py on larger synthetic inputs. CPU only."""
import os

import numpy as np
import pytest

from _helpers import load_golden
from oracle import datasets_oracle as O
from poi_recommendation_models_amd import data as D


def _write_checkins(path, uid, lid, time):
    with open(os.path.join(path, "checkins.txt"), "w") as f:
        for u, l, t in zip(uid.tolist(), lid.tolist(), time.tolist()):
            f.write(f"{u}\t{l}\t{t}\n")


def _assert_train_equal(train, z, pre):
    """train_matrix equality up to the within-row order, which the reference takes from
    random.shuffle (datasets.py:124-127 then :385-386)."""
    ip = z[pre + "train_indptr"]
    np.testing.assert_array_equal(train.indptr, ip)
    for u in range(len(ip) - 1):
        ref = dict(zip(z[pre + "train_indices"][ip[u]:ip[u + 1]].tolist(),
                       z[pre + "train_data"][ip[u]:ip[u + 1]].tolist()))
        got = dict(zip(train.indices[ip[u]:ip[u + 1]].tolist(), train.data[ip[u]:ip[u + 1]].tolist()))
        assert got == ref, u


def _lists(flat, lens):
    out, o = [], 0
    for n in lens.tolist():
        out.append(flat[o:o + n].tolist())
        o += n
    return out


@pytest.mark.parametrize("case", [0, 1])
def test_split_matches_reference(case, tmp_path):
    z = load_golden("datasets.npz")
    pre = f"case{case}/"
    U, P = z[pre + "shape"].tolist()
    _write_checkins(tmp_path, z[pre + "checkins_uid"], z[pre + "checkins_lid"], z[pre + "checkins_time"])
    train, test_pos, val_pos, _ = None, None, None, None
    ds = D.Dataset(U, P, str(tmp_path) + "/")
    train, test_pos, val_pos = ds.split_data(*ds.read_raw_data())
    _assert_train_equal(train, z, pre)
    assert test_pos == _lists(z[pre + "test_flat"], z[pre + "test_len"])
    assert val_pos == _lists(z[pre + "val_flat"], z[pre + "val_len"])


@pytest.mark.parametrize("case", [0, 1])
def test_oracle_split_matches_reference(case):
    z = load_golden("datasets.npz")
    pre = f"case{case}/"
    U, P = z[pre + "shape"].tolist()
    rows = zip(z[pre + "checkins_uid"].tolist(), z[pre + "checkins_lid"].tolist(),
               z[pre + "checkins_time"].tolist())
    train, test_pos, val_pos = O.split_data(*O.read_raw_data(rows), U)
    import scipy.sparse as sp
    keys = sorted(train)
    m = sp.csr_matrix(([train[k] for k in keys], ([k[0] for k in keys], [k[1] for k in keys])),
                      shape=(U, P))
    _assert_train_equal(m, z, pre)
    assert test_pos == _lists(z[pre + "test_flat"], z[pre + "test_len"])
    assert val_pos == _lists(z[pre + "val_flat"], z[pre + "val_len"])


def test_region_num_matches_reference(tmp_path):
    z = load_golden("datasets.npz")
    with open(tmp_path / "poi_region.txt", "w") as f:
        for p, r in zip(z["region/poi"].tolist(), z["region/region"].tolist()):
            f.write(f"{p}\t{r}\n")
    num = D.get_region_num(str(tmp_path) + "/")
    assert num == int(z["region/num"])
    got = np.loadtxt(tmp_path / "poi_region_sorted.txt", dtype=np.int64, delimiter="\t")
    np.testing.assert_array_equal(got, z["region/sorted"])
    np.testing.assert_array_equal(D.read_region_list(str(tmp_path) + "/"), z["region/sorted"][:, 1])
    new, n2 = O.get_region_num(zip(z["region/poi"].tolist(), z["region/region"].tolist()))
    assert n2 == num and np.array_equal(np.array(new), z["region/sorted"])


def test_split_matches_oracle_at_scale(tmp_path):
    """Synthetic files (D.write_synthetic) with repeated check-ins and equal latest times."""
    U, P = 600, 3000
    path = D.write_synthetic(str(tmp_path / "ds"), U, P, h_min=1, h_max=60, seed=5)
    uid, lid, t = D.read_checkins(path + "checkins.txt")
    t = np.where(uid % 5 == 0, np.floor(t / 1e7) * 1e7, t)     # many ties in some users
    cnt, tm = D.raw_matrices(uid, lid, t, U, P)
    train, test_pos, val_pos = D.split_with_time(cnt, tm)
    otrain, otest, oval = O.split_data(*O.read_raw_data(zip(uid.tolist(), lid.tolist(), t.tolist())), U)
    keys = sorted(otrain)
    tc = train.tocoo()
    assert list(zip(tc.row.tolist(), tc.col.tolist())) == keys
    np.testing.assert_array_equal(tc.data, [otrain[k] for k in keys])
    assert test_pos == otest and val_pos == oval
    # the dataset class reads the same
    tr2, te2, va2, pc = D.Dataset(U, P, path).generate_data()
    assert (tr2 != D.split_with_time(*D.raw_matrices(uid, lid, D.read_checkins(path + "checkins.txt")[2], U, P))[0]).nnz == 0
    assert len(pc) == P


def test_nonpositive_time_rejected():
    with pytest.raises(ValueError, match="time > 0"):
        D.split_with_time(*D.raw_matrices([0, 0], [1, 2], [5.0, 0.0], 1, 4))


def test_poi_coos_dict_order(tmp_path):
    lines = ["5 35.1 139.1", "2 35.2 139.2", "5 35.3 139.3", "0 35.4 139.4"]
    (tmp_path / "poi_coos.txt").write_text("\n".join(lines) + "\n")
    got = D.read_poi_coos(str(tmp_path / "poi_coos.txt"))
    assert got.tolist() == O.read_poi_coos(lines) == [[35.3, 139.3], [35.2, 139.2], [35.4, 139.4]]


@pytest.mark.parametrize("seed,size", [(0, 200), (1, 350), (2, 1000)])
def test_region_grid_matches_loop(seed, size):
    r = np.random.default_rng(seed)
    P = 1500
    pc = np.stack([r.uniform(35.5, 35.8, P), r.uniform(139.5, 139.9, P)], 1)
    pc[:4] = [[35.5, 139.5], [35.8, 139.9], [35.5, 139.9], [35.8, 139.5]]   # the corners
    got = D.region_grid(pc, size)
    want = O.get_region(pc.tolist(), size)
    np.testing.assert_array_equal(got, want)
    # points exactly on interior grid lines (band and column boundaries)
    la_min, la_max, lo_min, lo_max = pc[:, 0].min(), pc[:, 0].max(), pc[:, 1].min(), pc[:, 1].max()
    rows = int(D.haversine_m(la_max, lo_max, la_min, lo_max) / size)
    w = (D.haversine_m(la_max, lo_max, la_max, lo_min) + D.haversine_m(la_min, lo_max, la_min, lo_min)) / 2
    cols = int(w / size)
    alpha, delta = (la_max - la_min) / rows, (lo_max - lo_min) / cols
    extra = [[la_min + alpha * 3, lo_min + delta * 2], [la_min + alpha * (rows - 1), lo_max],
             [la_max, lo_min + delta * 5], [la_min + alpha * 1, lo_min + delta * 1]]
    pc2 = np.concatenate([pc, extra])
    np.testing.assert_array_equal(D.region_grid(pc2, size), O.get_region(pc2.tolist(), size))


def test_get_region_file_and_synthetic_regions(tmp_path):
    path = D.write_synthetic(str(tmp_path / "ds"), 20, 400, seed=3, region_size=500)
    got = np.loadtxt(path + "poi_region.txt", dtype=np.int64, delimiter="\t")
    assert got[:, 0].tolist() == list(range(400)) and (got[:, 1] >= 0).all()
    n = D.get_region_num(path)
    lst = D.read_region_list(path)
    assert len(lst) == 400 and lst.min() == 0 and lst.max() == n - 1
