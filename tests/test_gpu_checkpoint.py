"""The one-rank checkpoint engine with device-resident universes (openke/config/_checkpoint.py): tables copied
device -> host once per segment on a side stream, the archive equal to torch.save's file for the same state as far
as torch.load can tell (CPU tables in both: torch.save of device tensors records 'cuda:0', the engine writes host
copies, as the multi-rank path always has), and a later checkpoint reusing the first one's universes."""
import collections

import numpy as np
import pytest
import torch

from openke.config import _checkpoint
from openke.module.model import Model, TransE, TransH

pytestmark = pytest.mark.gpu


def test_device_universes_archive_equals_torch_save(tmp_path):
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    sp = collections.defaultdict(Model)
    for u in range(40):
        cls = TransH if u % 4 == 0 else TransE
        sp[u] = cls.seeded(u, int(rng.integers(10, 400)), int(rng.integers(1, 9)), dim=int(rng.integers(4, 70)),
                           p_norm=1, norm_flag=True).to(dev)
    ar = _checkpoint.UniverseArchive()
    first = collections.defaultdict(Model, {u: sp[u] for u in range(25)})
    ar.write(str(tmp_path / "a.ckpt"), {"next_universe_id": 25, "trained_embedding_spaces": first})
    ar.write(str(tmp_path / "b.ckpt"), {"next_universe_id": 40, "trained_embedding_spaces": sp})
    assert len(ar._segments) == 2
    ref = collections.defaultdict(Model, {u: sp[u].cpu() if False else sp[u] for u in sp})
    got = torch.load(str(tmp_path / "b.ckpt"), weights_only=False)
    assert list(got["trained_embedding_spaces"]) == list(range(40))
    for u in range(40):
        g, w = got["trained_embedding_spaces"][u], ref[u]
        assert type(g) is type(w)
        sg, sw = g.state_dict(), w.state_dict()
        assert list(sg) == list(sw)
        for k in sw:
            assert sg[k].device.type == "cpu" and torch.equal(sg[k], sw[k].cpu()), (u, k)
