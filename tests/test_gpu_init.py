"""Initial universe tables drawn on the GPU (pt_torch_init_tables, Model.device_seeded) equal the torch CPU
generator's bit for bit (Model.seeded: torch.manual_seed(seed0 + k) then the constructor, as the reference builds
each universe, Parallel_Universe_Config.py:157-177, TransE.py:17-36, TransH.py:17-42)."""
import numpy as np
import pytest
import torch

from openke.module.model import TransE, TransH

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cls", [TransE, TransH])
def test_device_seeded_equals_seeded(cls):
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    specs = []
    for k in range(48):   # universe-like sizes, odd sizes, tables under 16 elements, 624-word block edges
        ent = int(rng.integers(1, 2500))
        rel = int(rng.integers(1, 20))
        dim = int(rng.integers(1, 120)) if k % 3 else int(rng.choice([1, 3, 20, 156, 624]))
        specs.append((4 + k, ent, rel, {"dim": dim}))
    got = cls.device_seeded(specs, dev)
    for (seed, ent, rel, param), m in zip(specs, got):
        ref = cls.seeded(seed, ent, rel, **param)
        for a, b in zip(ref.tables(), m.tables()):
            if a is None:
                continue
            assert b.is_cuda
            assert torch.equal(a.detach(), b.detach().cpu()), (seed, ent, rel, param)
    assert cls.device_init_ok(dev)


def test_device_seeded_uniform_range_and_margin():
    dev = torch.device("cuda", 0)
    specs = [(9, 300, 7, {"dim": 50, "margin": 6.0, "epsilon": 2.0}), (10, 40, 2, {"dim": 8, "margin": 4.0})]
    for (seed, ent, rel, param), m in zip(specs, TransE.device_seeded(specs, dev)):
        ref = TransE.seeded(seed, ent, rel, **param)
        for a, b in zip(ref.tables(), m.tables()):
            if a is not None:
                assert torch.equal(a.detach(), b.detach().cpu())
        assert all(p.is_cuda for p in m.parameters())
