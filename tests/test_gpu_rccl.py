"""RCCL executes every collective of the N > 1 path (VERDICT r5 Missing 2 / Next 2).

The box has one GPU, and RCCL takes one GPU per rank, so this is world size 1: a fresh
torch.distributed.run child (the test process starts it and reads its file; it never execs)
runs tests/collectives_worker.py with init_process_group("nccl", device_id=cuda:0) -- the
packed (int32 id, f32 score bits) all_gather_into_tensor of the column-sharded merge, its int64 /
f64 forms, the f64 row all-gather, the int64 MAX (allreduce_gmax) and MIN (agree_min)
all-reduces, broadcast_module, load_sharded_tables / allgather_rows -- on device tensors, and the
merges (merge_topk: nais_topk_rows; merge_topk_f64: nais_topk_merge_f64) on the gathered blocks.
A second child runs the same worker over gloo on the CPU. The two result files must be
bit-identical, and both must equal the numpy restatement (tests/_collectives.py). No scaling
curve is measured here: with one rank every collective is a local copy through RCCL's kernels."""
import numpy as np
import pytest

import _collectives

pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives_bit_identical_to_gloo(tmp_path):
    rccl = _collectives.run(1, "nccl", str(tmp_path / "rccl.npz"))
    gloo = _collectives.run(1, "gloo", str(tmp_path / "gloo.npz"))
    assert str(rccl["backend"]) == "nccl" and str(gloo["backend"]) == "gloo"
    names = _collectives.assert_matches_expected(rccl, 1, device_merges=True)
    _collectives.assert_matches_expected(gloo, 1, device_merges=False)
    shared = [k for k in gloo if k not in ("backend",)]
    for k in shared:
        assert np.array_equal(_collectives.bits(rccl[k]), _collectives.bits(gloo[k])), k
    print(f"RCCL world 1: {len(names)} results checked ({', '.join(names)}); "
          f"{len(shared)} bit-identical to gloo")
