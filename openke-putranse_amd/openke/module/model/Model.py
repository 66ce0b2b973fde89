import copy
import ctypes
import math
import threading

import numpy as np
import torch
import torch.nn as nn

from ... import _native
from ..BaseModule import BaseModule

_MODES = {"normal": 0, "head_batch": 1, "tail_batch": 2}
# per-thread torch.Generator of Model.seeded (None: the default generator, as the reference's constructors use);
# per-thread recording state of Model.device_seeded (plan / dev)
_INIT = threading.local()
_DEVICE_INIT_OK = {}


_MODULE_CONTAINERS = (dict, set, list)


def _clone_module(src):
    """A new module object with src's attributes: every container (parameter / buffer / submodule / hook dicts)
    copied, so nothing registered on one is shared with the other. Tensors are replaced by the caller."""
    m = object.__new__(type(src))
    m.__dict__.update({k: (type(v)(v) if isinstance(v, _MODULE_CONTAINERS) else v) for k, v in src.__dict__.items()})
    return m


def _named_plan(model, plan):
    """A recorded init plan with each table named by its submodule (("normal" | "xavier", name) or
    ("uniform", name, lo, hi)), so it can be replayed on a model of other sizes."""
    names = {sub.weight.data_ptr(): n for n, sub in model._modules.items() if isinstance(sub, nn.Embedding)}
    out = []
    for x in plan:
        if x[0] == "normal":
            out.append(("normal", names[x[2].data_ptr()]))
        else:
            out.append((x[0], names[x[1].data_ptr()]) + tuple(x[2:4] if x[0] == "uniform" else ()))
    return out


def _clone_model(template, ent_tot, rel_tot, device):
    """What the constructor builds for (ent_tot, rel_tot) with the template's parameters, assembled from the
    template (Model.device_seeded: the constructor's Python work per universe was most of a wave's host time):
    the same attributes and submodules, each nn.Embedding table allocated on `device` (uninitialised: the init
    kernel fills it) with the rows the constructor gives it (ent_tot for the entity table, rel_tot for the relation
    tables), every other parameter a copy of the template's (a constant such as the margin). Returns
    (model, its init plan in device_seeded's recorded form)."""
    tm, named, t_ent, t_rel = template
    m = _clone_module(tm)
    m.ent_tot, m.rel_tot = ent_tot, rel_tot
    for name, sub in tm._modules.items():
        if isinstance(sub, nn.Embedding):
            n_rows = ent_tot if name == "ent_embeddings" else rel_tot
            e = _clone_module(sub)
            e.num_embeddings = n_rows
            e._parameters["weight"] = nn.Parameter(torch.empty(n_rows, sub.embedding_dim, device=device),
                                                   requires_grad=sub.weight.requires_grad)
            m._modules[name] = e
        else:
            m._modules[name] = copy.deepcopy(sub)
    for name, p in tm._parameters.items():
        m._parameters[name] = None if p is None else nn.Parameter(p.detach().clone(), requires_grad=p.requires_grad)
    plan = []
    for x in named:
        w = m._modules[x[1]].weight.data
        if x[0] == "normal":
            plan.append(("normal", w.numel(), x[1]))
        elif x[0] == "xavier":
            plan.append(("uniform", w) + _xavier_bounds(w))
        else:
            plan.append(("uniform", w, x[2], x[3]))
    return m, plan


def _xavier_bounds(w):
    """nn.init.xavier_uniform_'s (-a, a) for a 2-D tensor (gain 1): a = sqrt(3) * sqrt(2 / (fan_in + fan_out))."""
    fan_in, fan_out = nn.init._calculate_fan_in_and_fan_out(w)
    a = math.sqrt(3.0) * (1.0 * math.sqrt(2.0 / float(fan_in + fan_out)))
    return (-a, a)


def _normal_draws(numels):
    """32-bit MT19937 outputs torch's CPU normal_ consumes for float tensors of these sizes, in order, from a freshly
    seeded generator (aten/src/ATen/native/cpu/DistributionTemplates.h, normal_kernel): a contiguous tensor of at
    least 16 elements draws one uniform float per element plus 16 more when the size is not a multiple of 16
    (normal_fill recomputes the last 16); a smaller one takes Box-Muller normal_distribution<double> samples, two
    random64 (4 outputs) per generated pair, the second sample cached in the generator for the next element."""
    draws, cached = 0, False
    for n in numels:
        if n >= 16:
            draws += n + (16 if n % 16 else 0)
            continue
        for _ in range(n):
            if cached:
                cached = False
            else:
                draws += 4
                cached = True
    return draws


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

    @classmethod
    def device_seeded(cls, specs, device):
        """[cls.seeded(seed, ent_tot, rel_tot, **param) for (seed, ent_tot, rel_tot, param) in specs] with the same
        tables bit for bit, drawn on the GPU (pt_torch_init_tables: the torch CPU generator's MT19937 and its float
        uniform_, one workgroup per model) straight into device tensors: no CPU draws, no host-to-device copy.
        Each constructor runs in a recording mode - its nn.Embedding tables allocated on `device` uninitialised,
        its normal_ draws counted (_normal_draws) and its xavier / uniform inits recorded - and one launch fills
        every model. Verified against seeded() once per process and class (device_init_ok); raises if the
        constructor's draw order is one the kernel does not express (a uniform init before a normal_)."""
        models, jobs = [], []
        templates = {}   # constructor parameters -> (a model built by the constructor, its recorded plan)
        for seed, ent_tot, rel_tot, param in specs:
            key = tuple(sorted(param.items()))
            t = templates.get(key)
            cloned = False
            if t is None or ent_tot == rel_tot:
                _INIT.plan = []
                _INIT.dev = device
                try:
                    m = cls(ent_tot, rel_tot, **param)
                    plan = [("uniform",) + x[1:] if x[0] == "xavier" else x for x in _INIT.plan]
                    named = _named_plan(m, _INIT.plan)
                finally:
                    _INIT.plan = None
                    _INIT.dev = None
                if t is None and ent_tot != rel_tot and {x[1] for x in named} <= {"ent_embeddings", "rel_embeddings",
                                                                               "norm_vector"}:
                    templates[key] = (m, named, ent_tot, rel_tot)
            else:
                m, plan = _clone_model(t, ent_tot, rel_tot, device)
                cloned = True
            normals = [x[1] for x in plan if x[0] == "normal"]
            unis = [x for x in plan if x[0] == "uniform"]
            first_u = next((i for i, x in enumerate(plan) if x[0] == "uniform"), len(plan))
            if any(x[0] == "normal" for x in plan[first_u:]) or len(unis) > 4:
                raise NotImplementedError("device_seeded: %s's init order is not normal_* then uniform_*" % cls.__name__)
            j = _native.TorchInitJob()
            j.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
            j.skip = _normal_draws(normals)
            j.ntab = len(unis)
            for k, (_, w, lo, hi) in enumerate(unis):
                j.numel[k] = w.numel()
                j.lo[k], j.hi[k] = float(lo), float(hi)
                j.out[k] = w.data_ptr()
            jobs.append(j)
            # (a constructed model's small non-table parameters - the constants, a margin - to the device; a clone
            # copied them from the template, which is there already)
            models.append(m if cloned else m.to(device))
        if jobs:
            arr = (_native.TorchInitJob * len(jobs))(*jobs)
            with torch.cuda.device(device):
                _native.check(_native.lib().pt_torch_init_tables(arr, len(jobs), _native.stream()))
        return models

    @classmethod
    def device_init_ok(cls, device):
        """Whether device_seeded reproduces seeded() bit for bit under this torch build: checked once per process
        and class on two small models (tables of at least and of fewer than 16 elements: torch's two normal_
        paths), so a torch whose CPU generator differs makes callers keep the CPU construction."""
        key = (cls, str(device))
        if key not in _DEVICE_INIT_OK:
            specs = [(12345, 37, 3, {"dim": 20}), (77, 5, 1, {"dim": 3})]
            got = cls.device_seeded(specs, device)
            ok = True
            for (seed, e, r, param), m in zip(specs, got):
                ref = cls.seeded(seed, e, r, **param)
                for a, b in zip(ref.tables(), m.tables()):
                    if a is not None and not torch.equal(a.detach(), b.detach().cpu()):
                        ok = False
            _DEVICE_INIT_OK[key] = ok
        return _DEVICE_INIT_OK[key]

    @staticmethod
    def _generator():
        return getattr(_INIT, "gen", None)

    @staticmethod
    def _embedding(rows, dim):
        """nn.Embedding(rows, dim) with its default N(0, 1) init drawn from the active generator (device_seeded:
        allocated uninitialised on the device, its draws recorded)."""
        plan = getattr(_INIT, "plan", None)
        if plan is not None:
            w = torch.empty(rows, dim, device=_INIT.dev)
            plan.append(("normal", rows * dim, w))
            return nn.Embedding(rows, dim, _weight=w)
        gen = getattr(_INIT, "gen", None)
        if gen is None:
            return nn.Embedding(rows, dim)
        w = torch.empty(rows, dim)
        w.normal_(generator=gen)
        return nn.Embedding(rows, dim, _weight=w)

    def _xavier_uniform_(self, w):
        """nn.init.xavier_uniform_(w) from the active generator (device_seeded: recorded with torch's bound)."""
        plan = getattr(_INIT, "plan", None)
        if plan is not None:
            plan.append(("xavier", w) + _xavier_bounds(w))
            return
        nn.init.xavier_uniform_(w, generator=self._generator())

    def _uniform_(self, w, a, b):
        """nn.init.uniform_(w, a, b) from the active generator (device_seeded: recorded)."""
        plan = getattr(_INIT, "plan", None)
        if plan is not None:
            plan.append(("uniform", w, a, b))
            return
        nn.init.uniform_(tensor=w, a=a, b=b, generator=self._generator())

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
