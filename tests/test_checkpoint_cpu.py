"""The one-rank checkpoint engine (openke/config/_checkpoint.py, csrc/zip_writer.cpp): the archive it writes is
the file torch.save writes for the same state (Parallel_Universe_Config.save_parameters, reference :890-899) as
far as torch.load can tell - same state keys and order, same universe classes, attributes, parameters and
values - whether the universes are serialized by this write or reused from an earlier one; ZIP64 archives load;
universes of a replaced state are dropped; a state the engine does not express falls back to torch.save."""
import collections
import zipfile
import zlib

import numpy as np
import pytest
import torch

from openke.config import _checkpoint
from openke.config.Parallel_Universe_Config import _Pickled
from openke.module.model import Model, TransE, TransH


def _spaces(lo, hi, rng):
    sp = collections.defaultdict(Model)
    for u in range(lo, hi):
        cls = TransH if u % 3 == 0 else TransE
        sp[u] = cls.seeded(u, int(rng.integers(5, 60)), int(rng.integers(1, 6)), dim=int(rng.integers(2, 9)),
                           p_norm=1, norm_flag=True)
    return sp


def _state(spaces):
    return {"initial_num_universes": None, "next_universe_id": len(spaces), "trained_embedding_spaces": spaces,
            "entity_id_mappings": _Pickled({3: {1: 0, 7: 1}}), "entity_universes": _Pickled({1: {3}, 7: {3}}),
            "min_margin": 1, "embedding_model": TransE, "embedding_model_param": {"dim": (2, 8), "p_norm": 1},
            "best_hit10": 0.25, "bad_counts": 0}


def _same(a, b):
    assert list(a.keys()) == list(b.keys())
    for k in a:
        if k != "trained_embedding_spaces":
            assert a[k] == b[k] and type(a[k]) is type(b[k]), k
            continue
        A, B = a[k], b[k]
        assert type(A) is type(B) and A.default_factory is B.default_factory and list(A) == list(B)
        for u in B:
            x, y = A[u], B[u]
            assert type(x) is type(y)
            assert x.__dict__.keys() == y.__dict__.keys()
            for n in x.__dict__:
                if n not in ("_parameters", "_buffers", "_modules"):
                    assert x.__dict__[n] == y.__dict__[n], (u, n)
            assert list(x._modules) == list(y._modules)
            sx, sy = x.state_dict(), y.state_dict()
            assert list(sx) == list(sy)
            for n in sy:
                assert sx[n].dtype == sy[n].dtype and sx[n].device.type == "cpu" and torch.equal(sx[n], sy[n]), (u, n)
            for px, py in zip(x.parameters(), y.parameters()):
                assert type(px) is type(py) and px.requires_grad == py.requires_grad


def test_archive_equals_torch_save_and_reuses_universes(tmp_path, monkeypatch):
    rng = np.random.default_rng(3)
    ar = _checkpoint.UniverseArchive()
    sp = _spaces(0, 20, rng)
    ar.write(str(tmp_path / "a.ckpt"), _state(sp))
    torch.save(_state(sp), str(tmp_path / "a_ref.ckpt"))
    _same(torch.load(str(tmp_path / "a.ckpt"), weights_only=False),
          torch.load(str(tmp_path / "a_ref.ckpt"), weights_only=False))
    # a later, larger checkpoint pickles only the new universes
    sp2 = collections.defaultdict(Model, sp)
    sp2.update(_spaces(20, 31, rng))
    seen = []
    orig = _checkpoint._shadow
    monkeypatch.setattr(_checkpoint, "_shadow", lambda m, f: seen.append(m) or orig(m, f))
    ar.write(str(tmp_path / "b.ckpt"), _state(sp2))
    assert len([m for m in seen if isinstance(m, (TransE, TransH))]) == 11
    torch.save(_state(sp2), str(tmp_path / "b_ref.ckpt"))
    _same(torch.load(str(tmp_path / "b.ckpt"), weights_only=False),
          torch.load(str(tmp_path / "b_ref.ckpt"), weights_only=False))
    z = zipfile.ZipFile(str(tmp_path / "b.ckpt"))
    assert z.testzip() is None
    names = [i.filename for i in z.infolist()]
    assert names[:4] == ["b/data.pkl", "b/.format_version", "b/.storage_alignment", "b/byteorder"]
    assert names[-2:] == ["b/version", "b/.data/serialization_id"]
    raw = open(str(tmp_path / "b.ckpt"), "rb").read()
    for i in z.infolist():   # torch's 64-byte data alignment
        off = i.header_offset
        start = off + 30 + int.from_bytes(raw[off + 26:off + 28], "little") + int.from_bytes(raw[off + 28:off + 30], "little")
        assert start % 64 == 0 and zlib.crc32(raw[start:start + i.file_size]) == i.CRC


def test_archive_drops_replaced_universes_and_loads_zip64(tmp_path):
    rng = np.random.default_rng(4)
    ar = _checkpoint.UniverseArchive()
    sp = _spaces(0, 12, rng)
    ar.write(str(tmp_path / "a.ckpt"), _state(sp))
    # a restored best state: universes 6.. replaced by other objects
    sp2 = collections.defaultdict(Model, {u: sp[u] for u in range(6)})
    sp2.update(_spaces(6, 9, rng))
    ar.write(str(tmp_path / "b.ckpt"), _state(sp2), force_zip64=True)
    assert sorted(ar._frags) == list(range(9)) and all(ar._frags[u][0] is sp2[u] for u in range(9))
    torch.save(_state(sp2), str(tmp_path / "b_ref.ckpt"))
    _same(torch.load(str(tmp_path / "b.ckpt"), weights_only=False),
          torch.load(str(tmp_path / "b_ref.ckpt"), weights_only=False))
    assert zipfile.ZipFile(str(tmp_path / "b.ckpt")).testzip() is None


def test_unsupported_state_falls_back_to_torch_save(tmp_path):
    sp = collections.defaultdict(Model)
    m = TransE.seeded(1, 10, 2, dim=4, p_norm=1, norm_flag=True)
    m.ent_embeddings.weight.data = m.ent_embeddings.weight.data.double()
    sp[0] = m
    _checkpoint.save(_checkpoint.UniverseArchive(), _state(sp), str(tmp_path / "a.ckpt"))
    got = torch.load(str(tmp_path / "a.ckpt"), weights_only=False)
    assert torch.equal(got["trained_embedding_spaces"][0].ent_embeddings.weight, m.ent_embeddings.weight)


def test_zip_writer_rejects_bad_arguments(tmp_path):
    from openke import _native
    L = _native.lib()
    r = (_native.ZipRecord * 1)()
    r[0].name, r[0].data, r[0].size = b"x/a", None, 5   # data missing
    assert L.pt_zip_write(str(tmp_path / "z").encode(), r, 1, 64, 1, 0) == 1
    r[0].size = 0
    assert L.pt_zip_write(str(tmp_path / "z").encode(), r, 1, 48, 1, 0) == 1   # alignment not a power of two
    assert L.pt_zip_write(str(tmp_path / "no_dir" / "z").encode(), r, 1, 64, 1, 0) == 2   # PT_EIO


def test_host_budget_falls_back_to_torch_save(tmp_path):
    """A run whose host copies would pass the archive's budget is written by torch.save (same file contents)."""
    rng = np.random.default_rng(6)
    sp = _spaces(0, 6, rng)
    ar = _checkpoint.UniverseArchive(max_host_bytes=64)
    _checkpoint.save(ar, _state(sp), str(tmp_path / "a.ckpt"))
    assert not ar._segments
    torch.save(_state(sp), str(tmp_path / "a_ref.ckpt"))
    _same(torch.load(str(tmp_path / "a.ckpt"), weights_only=False),
          torch.load(str(tmp_path / "a_ref.ckpt"), weights_only=False))
    assert _checkpoint.UniverseArchive().max_host_bytes <= 16 << 30


def test_replaced_table_is_serialized_again(tmp_path):
    """A universe whose table was replaced after an earlier checkpoint (`weight.data = ...`) is written with its
    new table, not the cached one."""
    rng = np.random.default_rng(8)
    sp = _spaces(0, 4, rng)
    ar = _checkpoint.UniverseArchive()
    ar.write(str(tmp_path / "a.ckpt"), _state(sp))
    w = sp[2].ent_embeddings.weight
    w.data = w.data * 2.0 + 1.0
    ar.write(str(tmp_path / "b.ckpt"), _state(sp))
    got = torch.load(str(tmp_path / "b.ckpt"), weights_only=False)["trained_embedding_spaces"]
    assert torch.equal(got[2].ent_embeddings.weight, sp[2].ent_embeddings.weight)
    assert torch.equal(got[1].ent_embeddings.weight, sp[1].ent_embeddings.weight)


def test_in_place_write_is_serialized_again(tmp_path):
    """In-place writes to a trained universe after a checkpoint (add_ / copy_ under no_grad, load_state_dict) bump the
    table's version counter, so the next checkpoint carries the new values; so do eval() and requires_grad changes.
    A write through `.data` (invisible to version counters) is picked up after UniverseArchive.forget."""
    rng = np.random.default_rng(9)
    sp = _spaces(0, 5, rng)
    ar = _checkpoint.UniverseArchive()
    ar.write(str(tmp_path / "a.ckpt"), _state(sp))
    with torch.no_grad():
        sp[1].ent_embeddings.weight.add_(0.5)
        sp[3].rel_embeddings.weight.copy_(torch.ones_like(sp[3].rel_embeddings.weight))
    sp[4].load_state_dict({k: v + 1.0 for k, v in sp[4].state_dict().items()})
    sp[0].eval()
    sp[2].ent_embeddings.weight.requires_grad_(False)
    for name in ("b", "c"):
        if name == "c":
            sp[2].rel_embeddings.weight.data.mul_(3.0)
            ar.forget(2)
        ar.write(str(tmp_path / (name + ".ckpt")), _state(sp))
        torch.save(_state(sp), str(tmp_path / (name + "_ref.ckpt")))
        _same(torch.load(str(tmp_path / (name + ".ckpt")), weights_only=False),
              torch.load(str(tmp_path / (name + "_ref.ckpt")), weights_only=False))


def test_module_with_foreign_tensor_falls_back(tmp_path):
    """A universe module holding a tensor that is neither a parameter nor a buffer (its storage would not be in the
    archive's segment) is written by torch.save, not as a fragment pointing at a missing record."""
    rng = np.random.default_rng(10)
    sp = _spaces(0, 3, rng)
    sp[1].extra = torch.arange(4.0)
    ar = _checkpoint.UniverseArchive()
    _checkpoint.save(ar, _state(sp), str(tmp_path / "a.ckpt"))
    assert not ar._frags and not ar._segments
    got = torch.load(str(tmp_path / "a.ckpt"), weights_only=False)
    assert torch.equal(got["trained_embedding_spaces"][1].extra, sp[1].extra)
