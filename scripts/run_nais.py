"""train_NAIS of run.py:62-127 on the MI355X path, end to end: dataset files (the reference's
formats, data.Dataset) -> NAISTrainer epochs (device batches + fused step) -> NAIS_validation
every `--eval-every` epochs (catalog scoring + top-k on the device) -> the reference's printout.

    python scripts/run_nais.py --data ./data/Tokyo/ --users 3725 --pois 10768
    python scripts/run_nais.py --synthetic 2000 8000           # writes a synthetic dataset first
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from poi_recommendation_models_amd import data, validation  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_basic  # noqa: E402
from poi_recommendation_models_amd.trainer import NAISTrainer  # noqa: E402


class Args:
    """run.py:830-844, at factor_num = hidden_dim = 64 (the fused training kernels' shape; the
    reference's default 128 runs the general kernels, DESIGN.md "General training kernels")."""
    lr = 0.01
    lamda = 0.0
    epochs = 50
    topk = 50
    factor_num = 64
    hidden_dim = 64
    num_ng = 4
    beta = 0.5


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data")
    ap.add_argument("--users", type=int)
    ap.add_argument("--pois", type=int)
    ap.add_argument("--synthetic", type=int, nargs=2, metavar=("USERS", "POIS"))
    ap.add_argument("--h-max", type=int, default=40)
    ap.add_argument("--epochs", type=int, default=Args.epochs)
    ap.add_argument("--eval-every", type=int, default=5)
    ap.add_argument("--factor", type=int, default=Args.factor_num)
    ap.add_argument("--lr", type=float, default=Args.lr)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    torch.manual_seed(a.seed)
    if a.synthetic:
        a.users, a.pois = a.synthetic
        a.data = data.write_synthetic(tempfile.mkdtemp(prefix="nais_ds_") + "/", a.users, a.pois,
                                      h_min=5, h_max=a.h_max, seed=a.seed)
    args = Args()
    args.lr, args.factor_num, args.hidden_dim, args.epochs = a.lr, a.factor, a.factor, a.epochs
    t0 = time.time()
    train_matrix, test_positive, val_positive, _ = data.Dataset(a.users, a.pois, a.data).generate_data()
    print(f"data: {a.users} users, {a.pois} POIs, {train_matrix.nnz} train pairs ({time.time() - t0:.1f} s)")
    k_list = [5, 10, 15, 20, 25, 30]
    model = NAIS_basic(a.pois, args.factor_num, args.factor_num, args.beta).to("cuda")   # run.py:86
    trainer = NAISTrainer(model, train_matrix, lr=args.lr, weight_decay=args.lamda, num_ng=args.num_ng)
    history = []
    for e in range(args.epochs):
        start = time.time()
        loss = trainer.epoch()
        print("Train Epoch: {}; time: {:.2f} sec; loss: {:.4f}".format(e + 1, time.time() - start, loss))
        rec = None
        if (e + 1) % a.eval_every == 0:
            model.eval()
            with torch.no_grad():
                start = time.time()
                rec = validation.NAIS_validation(model, args, a.users, test_positive, val_positive,
                                                 train_matrix, k_list)
            print("eval time: {:.2f} sec; val recall@10 {:.4f}; test recall@10 {:.4f}".format(
                time.time() - start, rec[1][1], rec[4][1]))
        history.append((loss, rec))
    return history


if __name__ == "__main__":
    main()
