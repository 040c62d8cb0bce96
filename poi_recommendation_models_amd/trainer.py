"""The NAIS training loops of run.py on the device (SURVEY.md 8(f1) + 8(f2)): NAIS_basic
(run.py:91-111), NAIS_regionEmbedding (run.py:139-200), NAIS_region_distance_Embedding
(run.py:206-262) and NAIS_distance_Embedding (run.py:365-430).

    for buid in shuffled users:                                   run.py:96-99
        user_history, train_data, train_label = get_NAIS_batch(...)   batches.py:24-50  -> GPU
        optimizer.zero_grad(); prediction = model(...)            run.py:102-103
        loss = model.loss_func(...); loss.backward()              run.py:104-105     -> 1 call
        train_loss += loss.item(); optimizer.step()               run.py:107-109

`NAISTrainer.epoch(users)` runs that loop with two C-ABI calls per user -- `nais_make_train_batch`
(device-side negative sampling) and `nais_train_step` (forward, BCELoss, backward, Adagrad) --
and one host sync per epoch (the reference syncs on loss.item() every user). The region /
distance variants build get_NAIS_batch_region's extra inputs (batches.py:67-108) on the device too
-- the region ids of the history and target rows, and for the distance variants the
target_lat_long rows of run.py:240-245 (|coordinate differences| in float64, as latlon_mat holds
them, cast to float32) -- and step through `nais_train_step_ex`, which also updates embed_region /
dist_layer (torch.optim.Adagrad over model.parameters(), run.py:155, 222). The model's
parameters are updated in place; Adagrad's accumulators live in the trainer with torch's
semantics (state 'sum' and 'step' per parameter, `optimizer_state()` exports them).

The per-step arithmetic is the drop-in path's (NAIS_basic train-mode forward + backward +
optim.Adagrad), differing only in fp32 summation order; tests/test_gpu_train.py checks both
against the oracle. Batches follow get_NAIS_batch's distribution (shuffled positives as the
shared history, num_ng distinct uniform negatives per positive), not Python's random stream.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.autograd.graph import increment_version

from . import _capi
from .catalog import device_csr


class NAISTrainer:
    def __init__(self, model, train_matrix, lr=0.01, lr_decay=0.0, weight_decay=0.0, eps=1e-10,
                 initial_accumulator_value=0.0, num_ng=4, region_of=None, poi_coords=None):
        """region_of: businessRegionEmbedList (POI -> region id, run.py:148-151) for the region
        variants; poi_coords: [P, 2] (lat, lng) for the distance variants (latlon_mat's source,
        run.py:47-54)."""
        from .model import (NAIS_basic, NAIS_distance_Embedding, NAIS_region_distance_Embedding,
                            NAIS_regionEmbedding)
        if not isinstance(model, (NAIS_basic, NAIS_regionEmbedding, NAIS_region_distance_Embedding,
                                  NAIS_distance_Embedding)):
            raise NotImplementedError(f"NAISTrainer: {type(model).__name__} has no device training step")
        dev = model._check_device()
        self.region = model.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE)
        self.distance = model.VARIANT in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE)
        if self.region and region_of is None:
            raise ValueError(f"{type(model).__name__}: NAISTrainer needs region_of (businessRegionEmbedList)")
        if self.distance and poi_coords is None:
            raise ValueError(f"{type(model).__name__}: NAISTrainer needs poi_coords")
        self.region_of = (torch.as_tensor(np.asarray(region_of, dtype=np.int64)).to(dev)
                          if self.region else None)
        self.coords = (torch.as_tensor(np.ascontiguousarray(poi_coords, dtype=np.float64)).to(dev)
                       if self.distance else None)
        self.model, self.dev = model, dev
        self.csr = device_csr(train_matrix, dev)
        self.num_ng = int(num_ng)
        self.lr, self.lr_decay, self.weight_decay, self.eps = lr, lr_decay, weight_decay, eps
        self.step_count = 0
        ps = dict(model.named_parameters())
        self._names = ["embed_history.weight", "embed_target.weight", "attn_layer1.weight",
                       "attn_layer1.bias", "attn_layer2.weight"]
        if self.region:
            self._names.append("embed_region.weight")
        if self.distance:
            self._names += ["dist_layer.weight", "dist_layer.bias"]
        self.sums = {k: torch.full_like(ps[k], initial_accumulator_value) for k in self._names}
        P, D = ps["embed_history.weight"].shape
        H, DIN = ps["attn_layer1.weight"].shape
        self._g_eh = torch.zeros(P, D, device=dev)
        self._g_et = torch.zeros(P, D, device=dev)
        self._g_small = torch.zeros(H * DIN + 2 * H, device=dev)
        self._g_er = torch.zeros_like(ps["embed_region.weight"]) if self.region else None
        self._g_dist = torch.zeros(6, device=dev) if self.distance else None
        self._st_eh = torch.zeros(P, dtype=torch.int32, device=dev)
        self._st_et = torch.zeros(P, dtype=torch.int32, device=dev)
        self.loss_sum = torch.zeros(1, device=dev)
        self.bad_rows = torch.zeros(1, dtype=torch.int32, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._ws = torch.empty(0, dtype=torch.uint8, device=dev)
        self._bufs = {}

    # ------------------------------------------------------------------ batches (f2)
    def batch(self, uid, seed=None):
        """get_NAIS_batch(train_matrix, P, uid, num_ng) on the device: (hist [n], target [b],
        labels [b]); the reference's user_history is hist repeated b times. Region variants:
        + (hist_region [n], target_region [b]) as get_NAIS_batch_region (batches.py:67-108);
        distance variants: + target_lat_long [b, n, 2] f32 (run.py:240-245)."""
        n = int(self.csr.hist_len[uid])
        b = n * (1 + self.num_ng)
        key = (n, b)
        if key not in self._bufs:
            self._bufs = {key: (torch.empty(n, dtype=torch.int64, device=self.dev),
                                torch.empty(b, dtype=torch.int64, device=self.dev),
                                torch.empty(b, dtype=torch.float32, device=self.dev))}
        hist, tgt, lab = self._bufs[key]
        if seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        lib = _capi.load()
        _capi.check(lib.nais_make_train_batch(self.csr.indptr.data_ptr(), self.csr.indices.data_ptr(),
                                              int(uid), n, self.csr.shape[1], self.num_ng, seed,
                                              hist.data_ptr(), tgt.data_ptr(), lab.data_ptr(),
                                              self._err.data_ptr(),
                                              _capi.stream_handle(self.dev)), "nais_make_train_batch")
        out = (hist, tgt, lab)
        if self.region:       # businessRegionEmbedList[positives] / [train_data] (batches.py:96-101)
            out += (self.region_of.index_select(0, hist), self.region_of.index_select(0, tgt))
        if self.distance:
            out += (self.lat_long(hist, tgt),)
        return out

    def lat_long(self, hist, target):
        """target_lat_long [b, n, 2] f32 = latlon_mat[target, hist] (run.py:240-245): the absolute
        float64 coordinate differences of lat_lon_mat (run.py:47-54), cast to float32."""
        c = self.coords
        return (c.index_select(0, target)[:, None, :] - c.index_select(0, hist)[None, :, :]).abs_().to(
            torch.float32)

    # ------------------------------------------------------------------ one step (f1)
    def _opt_struct(self):
        o = _capi.NaisAdagradState()
        o.lr, o.lr_decay, o.weight_decay, o.eps = self.lr, self.lr_decay, self.weight_decay, self.eps
        o.step = self.step_count
        s = self.sums
        o.sum_embed_history = s["embed_history.weight"].data_ptr()
        o.sum_embed_target = s["embed_target.weight"].data_ptr()
        o.sum_w1 = s["attn_layer1.weight"].data_ptr()
        o.sum_b1 = s["attn_layer1.bias"].data_ptr()
        o.sum_w2 = s["attn_layer2.weight"].data_ptr()
        o.grad_embed_history = self._g_eh.data_ptr()
        o.grad_embed_target = self._g_et.data_ptr()
        o.grad_small = self._g_small.data_ptr()
        o.stamp_embed_history = self._st_eh.data_ptr()
        o.stamp_embed_target = self._st_et.data_ptr()
        return o

    def step(self, hist, target, labels, *side, dropout_seed=None, pred=None):
        """One fused step on a get_NAIS_batch batch given as the shared history hist [n] (or the
        reference's [b, n] user_history), target [b], labels [b]; `side` = what batch() adds for
        the variant: (hist_region, target_region) for the region variants ([n] or the reference's
        [b, n]), then target_lat_long [b, n, 2] for the distance variants."""
        m = self.model
        if hist.dim() == 2:
            hist = hist[0] if hist.shape[0] else hist.new_empty(0)
        hist = hist.to(torch.int64).contiguous()
        target = target.to(torch.int64).contiguous()
        labels = labels.to(torch.float32).contiguous()
        b, n = target.numel(), hist.numel()
        want = 2 * self.region + self.distance
        if len(side) != want:
            raise TypeError(f"{type(m).__name__}: step() takes {want} side input(s) after labels")
        sd = _capi.NaisTrainSide()
        keep = []
        if self.region:
            hreg, treg = side[0], side[1]
            if hreg.dim() == 2:
                hreg = hreg[0] if hreg.shape[0] else hreg.new_empty(0)
            hreg = hreg.to(torch.int64).contiguous()
            treg = treg.to(torch.int64).contiguous()
            keep += [hreg, treg]
            sd.hist_region, sd.target_region = _capi.ptr(hreg), _capi.ptr(treg)
        if self.distance:
            ll = side[-1].to(torch.float32)
            if tuple(ll.shape) != (b, n, 2):
                raise ValueError("target_lat_long must be [b, n, 2]")
            if not (ll.stride(2) == 1 and ll.stride(1) == 2):
                ll = ll.contiguous()
            keep.append(ll)
            sd.target_lat_long, sd.latlon_ld = ll.data_ptr(), ll.stride(0)
        drop = getattr(m, "drop", None)        # none in the two distance variants (model.py:268, 369)
        p = float(drop.p) if drop is not None and m.training else 0.0
        if dropout_seed is None:
            dropout_seed = int(torch.randint(0, 2**62, (1,)).item())
        self.step_count += 1
        lib = _capi.load()
        prm = m.nais_params()
        need = lib.nais_train_step_workspace_size(prm, b, n)
        if self._ws.numel() < need:
            self._ws = torch.empty(int(need * 1.25) + 256, dtype=torch.uint8, device=self.dev)
        args = (_capi.ptr(hist) if n else None, n, _capi.ptr(target) if b else None,
                _capi.ptr(labels) if b else None, b, p, dropout_seed, self.loss_sum.data_ptr(),
                self.bad_rows.data_ptr(), _capi.ptr(pred), self._ws.data_ptr(), self._ws.numel(),
                _capi.stream_handle(self.dev))
        if not (self.region or self.distance):
            _capi.check(lib.nais_train_step(prm, self._opt_struct(), *args), "nais_train_step")
            self._bump_versions()
            return
        os_ = _capi.NaisAdagradSide()
        if self.region:
            os_.sum_embed_region = self.sums["embed_region.weight"].data_ptr()
            os_.grad_embed_region = self._g_er.data_ptr()
        if self.distance:
            os_.sum_dist_w = self.sums["dist_layer.weight"].data_ptr()
            os_.sum_dist_b = self.sums["dist_layer.bias"].data_ptr()
            os_.grad_dist = self._g_dist.data_ptr()
        _capi.check(lib.nais_train_step_ex(prm, sd, self._opt_struct(), os_, *args), "nais_train_step_ex")
        self._bump_versions()
        del keep

    def _bump_versions(self):
        """The fused step writes the parameters through raw pointers: bump their version counters
        as an in-place torch op would, so version-keyed caches (model._score_params' padded copies
        for embed widths off the kernels' native set) are rebuilt before the next scoring call."""
        for q in self.model.parameters():
            increment_version(q)

    def epoch(self, users=None, shuffle=True):
        """One pass of run.py:96-109 over `users` (default: every user, shuffled as run.py:96-97).
        Returns train_loss (the sum of the per-user mean BCE losses, run.py:107)."""
        if users is None:
            users = np.arange(self.csr.shape[0])
        users = np.asarray(users, dtype=np.int64)
        if shuffle:
            users = users[torch.randperm(len(users)).numpy()]
        self.model.train()
        self.loss_sum.zero_()
        P = self.csr.shape[1]
        for u in users.tolist():
            n = int(self.csr.hist_len[u])
            if n == 0:
                continue   # empty batch: the reference's step changes nothing
            if n * (1 + self.num_ng) > P:
                raise ValueError(f"user {u}: {n} positives x {1 + self.num_ng} rows exceed {P} POIs "
                                 "(get_NAIS_batch cannot draw enough negatives)")
            self.step(*self.batch(u))
        return self.finish()

    def finish(self):
        """Host sync: the accumulated loss; raises like the reference's BCELoss if a batch had a
        NaN prediction (its update and all later ones were skipped)."""
        bad = int(self.bad_rows.item())
        if bad:
            raise RuntimeError(f"all elements of input should be between 0 and 1 ({bad} NaN "
                               "predictions: a single-item history equal to its target, "
                               "model.py:92-95); the updates from that batch on were skipped")
        if int(self._err.item()):
            raise RuntimeError("nais_make_train_batch: history length disagrees with the CSR")
        return float(self.loss_sum.item())

    def optimizer_state(self):
        """torch.optim.Adagrad-style per-parameter state {name: {'step', 'sum'}}."""
        return {k: {"step": torch.tensor(float(self.step_count)), "sum": self.sums[k]}
                for k in self._names}
