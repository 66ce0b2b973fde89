"""The GPU initial-table kernel's algorithm (csrc/torch_init.hip, Model.device_seeded), restated in numpy and pinned
against torch's CPU generator: MT19937(seed mod 2^32), the draws nn.Embedding's normal_ consumes
(Model._normal_draws: tensors of >= 16 and of < 16 elements take different torch paths), then one 32-bit output per
element of xavier_uniform_ / uniform_ (TransE.py / TransH.py constructors, the reference's universe init after
torch.manual_seed(seed0 + k), Parallel_Universe_Config.py:157-177). No GPU."""
import math

import numpy as np
import pytest
import torch

from openke.module.model import TransE, TransH
from openke.module.model.Model import _normal_draws


class _MT:
    """MT19937 as torch's CPU generator runs it (init_genrand(seed mod 2^32), next_state, tempering)."""

    def __init__(self, seed):
        self.s = [seed & 0xFFFFFFFF]
        for j in range(1, 624):
            x = self.s[-1]
            self.s.append((1812433253 * (x ^ (x >> 30)) + j) & 0xFFFFFFFF)
        self.i = 624

    def next(self):
        if self.i >= 624:
            s = self.s
            for k in range(624):
                y = (s[k] & 0x80000000) | (s[(k + 1) % 624] & 0x7FFFFFFF)
                s[k] = s[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.s[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def _restated(seed, shapes, bounds):
    """The kernel's output: skip the normal_ draws of every table, then fill the tables in order."""
    mt = _MT(seed)
    for _ in range(_normal_draws([r * d for r, d in shapes])):
        mt.next()
    out = []
    for (r, d), (lo, hi) in zip(shapes, bounds):
        f_lo, f_hi = np.float32(lo), np.float32(hi)
        span = float(np.float32(f_hi - f_lo))
        v = np.array([np.float32((mt.next() & 0xFFFFFF) * 2.0 ** -24 * span + float(f_lo)) for _ in range(r * d)],
                     dtype=np.float32)
        out.append(v.reshape(r, d))
    return out


def _xavier_bounds(shapes):
    return [(-math.sqrt(3.0) * math.sqrt(2.0 / float(r + d)), math.sqrt(3.0) * math.sqrt(2.0 / float(r + d)))
            for r, d in shapes]


@pytest.mark.parametrize("cls,seed,ent,rel,dim", [(TransE, 4, 40, 3, 20), (TransE, 517, 33, 5, 7),
                                                  (TransE, 9, 3, 1, 5), (TransE, 13, 1, 1, 1),
                                                  (TransH, 21, 30, 2, 12), (TransH, 8, 4, 1, 3)])
def test_restated_init_equals_torch(cls, seed, ent, rel, dim):
    m = cls.seeded(seed, ent, rel, dim=dim)
    shapes = [(ent, dim), (rel, dim)] + ([(rel, dim)] if cls is TransH else [])
    got = _restated(seed, shapes, _xavier_bounds(shapes))
    for a, b in zip(m.tables(), got):
        assert np.array_equal(a.detach().numpy(), b)


def test_restated_uniform_range_init_equals_torch():
    """margin and epsilon given: nn.init.uniform_ with the embedding range instead of xavier."""
    m = TransE.seeded(31, 25, 4, dim=10, margin=6.0, epsilon=2.0)
    r = float(torch.Tensor([(6.0 + 2.0) / 10]).item())
    got = _restated(31, [(25, 10), (4, 10)], [(-r, r), (-r, r)])
    for a, b in zip(m.tables(), got):
        assert np.array_equal(a.detach().numpy(), b)


def test_normal_draw_rule():
    """_normal_draws against the generator state torch leaves after normal_ (the next output compared)."""
    for sizes in ([16], [17], [40, 3], [15, 5], [7], [1, 1, 1], [33, 2, 64]):
        g = torch.Generator().manual_seed(99)
        for n in sizes:
            torch.empty(n).normal_(generator=g)
        nxt = int(torch.empty(1).uniform_(0, 1, generator=g).item() * 2 ** 24)
        mt = _MT(99)
        for _ in range(_normal_draws(sizes)):
            mt.next()
        assert mt.next() & 0xFFFFFF == nxt, sizes


@pytest.mark.parametrize("cls,param", [(TransE, {"dim": 20}), (TransH, {"dim": 7, "p_norm": 2}),
                                       (TransE, {"dim": 10, "margin": 6.0, "epsilon": 2.0})])
def test_clone_model_matches_constructor(cls, param):
    """Model.device_seeded builds all but the first model of a parameter set by cloning it (_clone_model): the
    clone has the constructed model's attributes, submodules, parameter names / shapes / flags, and the init plan
    the constructor records for those sizes."""
    from openke.module.model import Model as M
    mod = __import__("openke.module.model.Model", fromlist=["_INIT"])
    cpu = torch.device("cpu")

    def record(e, r):
        mod._INIT.plan, mod._INIT.dev = [], cpu
        try:
            m = cls(e, r, **param)
            return m, list(mod._INIT.plan)
        finally:
            mod._INIT.plan, mod._INIT.dev = None, None
    t, tplan = record(300, 7)
    tmpl = (t, mod._named_plan(t, tplan), 300, 7)
    c, cplan = mod._clone_model(tmpl, 41, 3, cpu)
    ref, rplan = record(41, 3)
    assert type(c) is type(ref) and c.ent_tot == 41 and c.rel_tot == 3
    sd_c, sd_r = c.state_dict(), ref.state_dict()
    assert list(sd_c) == list(sd_r)
    for k in sd_r:
        assert sd_c[k].shape == sd_r[k].shape
        if "embeddings" not in k and "norm_vector" not in k:
            assert torch.equal(sd_c[k], sd_r[k])
    for (n1, p1), (n2, p2) in zip(c.named_parameters(), ref.named_parameters()):
        assert n1 == n2 and p1.requires_grad == p2.requires_grad and p1 is not dict(t.named_parameters()).get(n1)
    for name, sub in ref._modules.items():
        assert type(c._modules[name]) is type(sub)
        if isinstance(sub, torch.nn.Embedding):
            assert (c._modules[name].num_embeddings, c._modules[name].embedding_dim) == (sub.num_embeddings,
                                                                                         sub.embedding_dim)
    for k in ("dim", "p_norm", "norm_flag", "margin_flag", "epsilon"):
        assert getattr(c, k, None) == getattr(ref, k, None) or k == "margin"
    # the replayed plan: the same draws and bounds as the constructor records for these sizes
    norm = lambda p: [(x[0], x[1] if x[0] == "normal" else x[1].shape) + tuple(x[2:4] if x[0] != "normal" else ())
                      for x in p]
    rplan = [("uniform",) + x[1:] if x[0] == "xavier" else x for x in rplan]
    assert norm(cplan) == norm(rplan)
    # nothing shared with the template
    assert c._modules is not t._modules and c._parameters is not t._parameters
    assert c._modules["ent_embeddings"] is not t._modules["ent_embeddings"]
