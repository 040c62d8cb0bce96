"""End to end on the device: dataset files in the reference's formats -> data.Dataset split ->
NAISTrainer epochs (device batches + fused training step) -> NAIS_validation (catalog scoring +
top-k) -> metrics, i.e. train_NAIS of run.py:62-127 through scripts/run_nais.py."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


def test_run_nais_synthetic():
    import run_nais
    hist = run_nais.main(["--synthetic", "300", "1500", "--epochs", "6", "--eval-every", "3",
                          "--factor", "32", "--lr", "0.05", "--h-max", "30"])
    losses = [h[0] for h in hist]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
    for _, rec in hist[2::3]:
        assert rec is not None and len(rec) == 6
        for lst in rec:
            assert len(lst) == 6 and all(0.0 <= x <= 1.0 for x in lst)
