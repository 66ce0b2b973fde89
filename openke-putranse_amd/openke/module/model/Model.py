import ctypes
import threading

import numpy as np
import torch
import torch.nn as nn

from ... import _native
from ..BaseModule import BaseModule

_MODES = {"normal": 0, "head_batch": 1, "tail_batch": 2}
# per-thread torch.Generator of Model.seeded (None: the default generator, as the reference's constructors use)
_INIT = threading.local()


class Model(BaseModule):
    """Base of the translational models (openke/module/model/Model.py). Scoring goes through the HIP
    kernels of libputranse_hip.so (pt_score); there is no torch-op or CPU scoring path."""

    native_model = None   # _native.PT_TRANSE / PT_TRANSH

    def __init__(self, ent_tot, rel_tot):
        super(Model, self).__init__()
        self.ent_tot = ent_tot
        self.rel_tot = rel_tot

    # -- initialisation from a private generator ---------------------------------------------------
    @classmethod
    def seeded(cls, seed, ent_tot, rel_tot, **param):
        """The module `torch.manual_seed(seed); cls(ent_tot, rel_tot, **param)` builds - bit for bit the same
        tables (nn.Embedding's normal_ draws, then the xavier / uniform init, in the constructor's order) -
        drawn from a private torch.Generator seeded with `seed` instead of the process-global one. Thread-safe:
        Parallel_Universe_Config builds a wave's universes on a thread pool with it (torch releases the GIL
        inside the draws)."""
        _INIT.gen = torch.Generator().manual_seed(int(seed))
        try:
            return cls(ent_tot, rel_tot, **param)
        finally:
            _INIT.gen = None

    @staticmethod
    def _generator():
        return getattr(_INIT, "gen", None)

    @staticmethod
    def _embedding(rows, dim):
        """nn.Embedding(rows, dim) with its default N(0, 1) init drawn from the active generator."""
        gen = getattr(_INIT, "gen", None)
        if gen is None:
            return nn.Embedding(rows, dim)
        w = torch.empty(rows, dim)
        w.normal_(generator=gen)
        return nn.Embedding(rows, dim, _weight=w)

    # -- native plumbing --------------------------------------------------------------------------
    def tables(self):
        """(ent, rel, norm_vector or None) weight tensors."""
        nv = getattr(self, "norm_vector", None)
        return (self.ent_embeddings.weight, self.rel_embeddings.weight, nv.weight if nv is not None else None)

    def native_desc(self, opt=_native.PT_SGD, lr=0.0, margin=0.0, accs=(None, None, None)):
        ent, rel, nv = self.tables()
        for t in (ent, rel, nv):
            if t is None:
                continue
            if not t.is_cuda:
                raise RuntimeError("model tables are on %s: call model.cuda() first (the MI355X build has no "
                                   "CPU path)" % t.device)
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("model tables must be contiguous float32")
        d = _native.ModelDesc()
        d.model = self.native_model
        d.p_norm = int(self.p_norm)
        d.norm_flag = 1 if self.norm_flag else 0
        d.opt = opt
        d.lr = float(lr)
        d.margin = float(margin)
        d.ent_total = ent.shape[0]
        d.rel_total = rel.shape[0]
        d.dim = ent.shape[1]
        d.ent = ent.data_ptr()
        d.rel = rel.data_ptr()
        d.normv = nv.data_ptr() if nv is not None else None
        ea, ra, na = accs
        d.ent_acc = ea.data_ptr() if ea is not None else None
        d.rel_acc = ra.data_ptr() if ra is not None else None
        d.norm_acc = na.data_ptr() if na is not None else None
        return d

    def _ids(self, x, dev):
        if isinstance(x, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64))
        elif not torch.is_tensor(x):
            x = torch.as_tensor(x, dtype=torch.int64)
        return x.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()

    def native_score(self, data):
        """||h + r - t||_p of every triple in `data` as the reference's forward computes it."""
        _native.require_gpu()
        mode = data.get("mode", "normal")
        dev = self.ent_embeddings.weight.device
        h = self._ids(data["batch_h"], dev)
        t = self._ids(data["batch_t"], dev)
        r = self._ids(data["batch_r"], dev)
        if mode == "normal":
            n = h.numel()
            if not (t.numel() == n and r.numel() == n):
                raise ValueError("normal mode needs equal-length h, t, r")
        elif mode == "head_batch":
            n = h.numel()
        elif mode == "tail_batch":
            n = t.numel()
        else:
            raise ValueError("unknown mode %r" % mode)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        desc = self.native_desc()
        _native.check(_native.lib().pt_score(ctypes.byref(desc), _MODES[mode], _native.ptr(h), _native.ptr(t),
                                             _native.ptr(r), n, _native.ptr(out), _native.stream()))
        return out

    def forward(self):
        raise NotImplementedError

    def predict(self):
        raise NotImplementedError
