"""Config 4 through the "pairs" strategy, phase by phase (HIP events on one stream):
distinct history items (nais_pair_rows), pair tables (nais_pair_table), per-user gathers
(nais_pair_gather), top-50 (nais_topk_rows). All 50k users x 100k POIs, d = H = 64.

    python scripts/bench_pairs.py [--users 50000 --pois 100000 --precision fp16x3 --col-block 0]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from poi_recommendation_models_amd import _capi  # noqa: E402
from poi_recommendation_models_amd.catalog import DeviceCSR  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_basic  # noqa: E402
from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=50_000)
    ap.add_argument("--pois", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--precision", default="fp16x3")
    ap.add_argument("--col-block", type=int, default=0, help="0: as large as memory allows")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    U, P, D, K = a.users, a.pois, a.dim, 50
    t0 = time.perf_counter()
    data = make_checkins(U, P, a.h_max, seed=2024)
    p = init_nais_params(P, D, D, seed=7, emb_std=0.3, bias_std=0.1)
    m = NAIS_basic(P, D, D, 0.5)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=False)
    m = m.to(dev).eval()
    m.precision = a.precision
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    print(f"setup {time.perf_counter() - t0:.1f} s", flush=True)
    lib = _capi.load()
    prm = m.nais_params()
    st = torch.cuda.current_stream(dev).cuda_stream
    users = torch.arange(U, dtype=torch.int32, device=dev)
    rowmap = torch.empty(P, dtype=torch.int32, device=dev)
    items = torch.empty(P, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(lib.nais_pair_rows_workspace_size(P), dtype=torch.uint8, device=dev)
    scores = torch.empty(U, P, dtype=torch.float32, device=dev)
    ids = torch.empty(U, K, dtype=torch.int32, device=dev)
    top = torch.empty(U, K, dtype=torch.float32, device=dev)
    ctr = torch.zeros(2, dtype=torch.int32, device=dev)
    _capi.check(lib.nais_pair_rows(csr.indptr.data_ptr(), csr.indices.data_ptr(), users.data_ptr(), U, P,
                                   rowmap.data_ptr(), items.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
                                   ws.numel(), st), "rows")
    J = int(cnt.item())
    free = torch.cuda.mem_get_info(dev)[0]
    W = a.col_block or int(min(P, (int(free * 0.7) // (8 * J)) // 256 * 256))
    tab = torch.empty(2, J, W, dtype=torch.float32, device=dev)
    entries = int(data.hist_len().sum())
    print(f"J={J} entries={entries} sharing={entries / J:.1f} W={W} tables={tab.numel() * 4 / 1e9:.1f} GB",
          flush=True)
    res = []
    for rep in range(a.reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t_rows = t_tab = t_gat = 0.0
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        ev[0].record()
        _capi.check(lib.nais_pair_rows(csr.indptr.data_ptr(), csr.indices.data_ptr(), users.data_ptr(), U,
                                       P, rowmap.data_ptr(), items.data_ptr(), cnt.data_ptr(),
                                       ws.data_ptr(), ws.numel(), st), "rows")
        ev[1].record()
        torch.cuda.synchronize()
        t_rows = ev[0].elapsed_time(ev[1])
        for c0 in range(0, P, W):
            cols = min(W, P - c0)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            _capi.check(lib.nais_pair_table(prm, items.data_ptr(), J, c0, cols, None, None, None,
                                            tab[0].data_ptr(), tab[1].data_ptr(), W, None, st), "table")
            e[1].record()
            _capi.check(lib.nais_pair_gather(tab[0].data_ptr(), tab[1].data_ptr(), W, rowmap.data_ptr(),
                                             csr.indptr.data_ptr(), csr.indices.data_ptr(), users.data_ptr(),
                                             U, c0, cols, 0.5, scores.data_ptr(), P, 0, ctr.data_ptr(), st),
                        "gather")
            e[2].record()
            torch.cuda.synchronize()
            t_tab += e[0].elapsed_time(e[1])
            t_gat += e[1].elapsed_time(e[2])
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        _capi.check(lib.nais_topk_rows(scores.data_ptr(), P, P, U, K, ids.data_ptr(), top.data_ptr(),
                                       ctr[1:].data_ptr(), st), "topk")
        e[1].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - w0
        t_topk = e[0].elapsed_time(e[1])
        pairs = U * P - entries
        gbytes = entries * P * 8 + U * P * 4
        fl = J * P * (2 * D * D + 3 * D + 4 * D)
        res.append({"wall_s": wall, "pairs_per_s": pairs / wall, "rows_ms": t_rows, "table_ms": t_tab,
                    "table_tflops": fl / (t_tab * 1e-3) / 1e12, "gather_ms": t_gat,
                    "gather_GBps": gbytes / (t_gat * 1e-3) / 1e9, "topk_ms": t_topk})
        print(json.dumps(res[-1]), flush=True)
    # parity spot check: 3 users against the direct kernel
    from poi_recommendation_models_amd.catalog import score_catalog
    ref = score_catalog(m, csr, [0, 1, 2])
    print("max |pairs - direct| (3 users):", float((scores[:3] - ref).abs().max()))


if __name__ == "__main__":
    main()
