"""Host-side logic of the drop-in Parallel_Universe_Config (CPU, no GPU): the private-generator model factory
equals the reference's manual_seed + constructor init bit for bit, the private per-universe Python draws equal
the reference's globally seeded draws, the lazily registered id dictionaries equal the reference's per-entity
registration (Parallel_Universe_Config.py:179-207), and the default wave size is a multiple of valid_steps."""
import random
from collections import defaultdict

import numpy as np
import pytest
import torch

from openke import _native
from openke.config.Parallel_Universe_Config import Parallel_Universe_Config, universe_dim
from openke.module.model import TransE, TransH


@pytest.mark.parametrize("cls", [TransE, TransH])
@pytest.mark.parametrize("kw", [{"dim": 23, "p_norm": 1, "norm_flag": True}, {"dim": 8, "margin": 4.0, "epsilon": 2.0}])
def test_seeded_factory_equals_manual_seed_init(cls, kw):
    torch.manual_seed(11)
    a = cls(97, 5, **kw)
    state = torch.get_rng_state()
    b = cls.seeded(11, 97, 5, **kw)
    assert torch.equal(state, torch.get_rng_state())   # the process-global generator is untouched
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


class _Loader(object):
    def __init__(self):
        self.lib = _native.lib()
        self.entTotal, self.relTotal = 400, 9
        self.in_path = "unused/"
        self.batch_size, self.nbatches = 10, 20


def _config(**kw):
    return Parallel_Universe_Config(train_dataloader=_Loader(), valid_dataloader=object(), embedding_model=TransE,
                                    embedding_model_param={"dim": 8, "p_norm": 1, "norm_flag": True}, **kw)


def test_private_draws_equal_reference_draws():
    cfg = _config(min_lr=0.001, max_lr=0.1)
    for uid in range(20):
        random.seed(cfg.initial_random_seed + uid)   # set_random_seed(seed0 + uid) then the reference's order
        tc = random.randrange(cfg.min_triple_constraint, cfg.max_triple_constraint)
        bal = round(random.uniform(cfg.min_balance, cfg.max_balance), 2)
        margin = random.randrange(cfg.min_margin, cfg.max_margin)
        epochs = random.randrange(cfg.min_num_epochs, cfg.max_num_epochs)
        lr = round(random.uniform(cfg.min_lr, cfg.max_lr), 3)
        assert cfg._universe_draws(uid) == (tc, bal, margin, epochs, lr)


def test_lazy_id_maps_equal_reference_registration():
    rng = np.random.default_rng(4)
    cfg = _config()
    want_e, want_r = defaultdict(dict), defaultdict(dict)
    want_eu, want_ru = defaultdict(set), defaultdict(set)
    for uid in range(30):
        em = rng.choice(400, int(rng.integers(1, 120)), replace=False)
        rm = rng.choice(9, int(rng.integers(1, 9)), replace=False)
        for local, g in enumerate(em.tolist()):   # the reference's loop (:179-207)
            want_e[uid][g] = local
            want_eu[g].add(uid)
        for local, g in enumerate(rm.tolist()):
            want_r[uid][g] = local
            want_ru[g].add(uid)
        cfg._register_maps(uid, em, rm)
        if uid == 14:   # a read in between registers the pending universes; later ones stay pending
            assert dict(cfg.entity_universes) == dict(want_eu)
    assert {u: dict(m) for u, m in cfg.entity_id_mappings.items()} == dict(want_e)
    assert {u: dict(m) for u, m in cfg.relation_id_mappings.items()} == dict(want_r)
    assert dict(cfg.entity_universes) == dict(want_eu)
    assert dict(cfg.relation_universes) == dict(want_ru)
    assert cfg.gather_embedding_spaces(int(list(want_eu)[0]), int(list(want_ru)[0])) == \
        want_eu[list(want_eu)[0]] & want_ru[list(want_ru)[0]]
    # a replaced state (get_best_state / load) drops universes registered after it
    snap = cfg.get_state()
    cfg.best_state = snap
    cfg._register_maps(30, np.array([1, 2]), np.array([0]))
    cfg.get_best_state()
    assert 30 not in cfg.entity_id_mappings and 30 not in cfg.entity_universes[1]


def test_default_wave_size_is_a_multiple_of_valid_steps():
    for vs in (1, 5, 100, 128, 600, 1000):
        w = _config(valid_steps=vs).wave_size()
        assert w % vs == 0 and w >= vs and (vs > 512 or abs(w - 512) <= vs / 2)
    assert _config(valid_steps=100, universe_wave_size=7).wave_size() == 7


def test_universe_dim_range():
    assert universe_dim(20, 5) == 20
    dims = [universe_dim((20, 100), u) for u in range(200)]
    assert min(dims) >= 20 and max(dims) <= 100 and len(set(dims)) > 30
    assert dims[:3] == [int(np.random.default_rng(1000 + u).integers(20, 101)) for u in range(3)]


def test_checkpoint_layout_and_background_write(tmp_path):
    """save_parameters writes the reference's layout (Parallel_Universe_Config.py:890-899: plain dicts of the
    id maps and occurrence sets after torch.load) with the containers pre-pickled; a background write is a
    snapshot of the moment it was asked for (a universe registered afterwards is not in it) and completes at
    flush_checkpoint."""
    rng = np.random.default_rng(9)
    cfg = _config(checkpoint_dir=str(tmp_path) + "/")
    for uid in range(12):
        cfg._register_maps(uid, rng.choice(400, 50, replace=False), rng.choice(9, 4, replace=False))
        cfg.trained_embedding_spaces[uid] = TransE.seeded(uid, 50, 4, dim=8, p_norm=1, norm_flag=True)
    cfg.next_universe_id = 12
    want = {k: v for k, v in cfg.get_state().items()}
    cfg.save_model("bg.ckpt", background=True)
    cfg._register_maps(12, np.array([3, 4]), np.array([1]))   # after the snapshot
    cfg.flush_checkpoint()
    cfg.save_model("fg.ckpt")
    a = torch.load(str(tmp_path / "bg.ckpt"), weights_only=False)
    b = torch.load(str(tmp_path / "fg.ckpt"), weights_only=False)
    for k in ("entity_id_mappings", "relation_id_mappings", "entity_universes", "relation_universes"):
        assert type(a[k]) is type(want[k]), k
        assert {u: (dict(m) if isinstance(m, dict) else m) for u, m in a[k].items()} == \
            {u: (dict(m) if isinstance(m, dict) else m) for u, m in want[k].items()}, k
    assert 12 not in a["entity_id_mappings"] and 12 in b["entity_id_mappings"]
    assert a["next_universe_id"] == 12 and sorted(a["trained_embedding_spaces"]) == list(range(12))
    for u in range(12):
        sa, sw = a["trained_embedding_spaces"][u].state_dict(), cfg.trained_embedding_spaces[u].state_dict()
        for k in sw:
            assert torch.equal(sa[k], sw[k])


def _same_container(a, b):
    """Same type, default factory, key order, values (inner dicts: items in order; sets: members - a set's
    iteration order is not kept by a pickle round trip, the reference's checkpoints included)."""
    assert type(a) is type(b) and getattr(a, "default_factory", None) is getattr(b, "default_factory", None)
    assert list(a.keys()) == list(b.keys())
    for k in a:
        x, y = a[k], b[k]
        assert type(x) is type(y) and getattr(x, "default_factory", None) is getattr(y, "default_factory", None)
        assert (list(x.items()) if isinstance(x, dict) else x) == (list(y.items()) if isinstance(y, dict) else y), k


def test_checkpoint_maps_from_arrays_equal_dictionaries(tmp_path, monkeypatch):
    """While nobody read or replaced the id dictionaries, a checkpoint pickles them straight from the registered
    remap arrays (_map_pickle, pt_pickle_id_maps / pt_pickle_universe_sets) without building them; torch.load
    gives back exactly the reference's registration (:179-207): types, default factories, key order and values.
    Once a caller reads them the checkpoint pickles the dictionaries themselves, with the same result."""
    from openke.config import _map_pickle
    calls = []
    for fn in ("id_maps_stream", "universes_stream"):
        orig = getattr(_map_pickle, fn)
        monkeypatch.setattr(_map_pickle, fn, lambda *a, _o=orig, _n=fn: calls.append(_n) or _o(*a))
    rng = np.random.default_rng(21)
    cfg = _config(checkpoint_dir=str(tmp_path) + "/")
    from openke.config.Parallel_Universe_Config import defaultdict_int
    want = {"entity_id_mappings": defaultdict(defaultdict_int), "relation_id_mappings": defaultdict(defaultdict_int),
            "entity_universes": defaultdict(set), "relation_universes": defaultdict(set)}
    for uid in range(40):
        em = rng.choice(400, int(rng.integers(1, 150)), replace=False)
        rm = rng.choice(9, int(rng.integers(1, 9)), replace=False)
        for local, g in enumerate(em.tolist()):   # the reference's loop (:196-201)
            want["entity_universes"][g].add(uid)
            want["entity_id_mappings"][uid][g] = local
        for local, g in enumerate(rm.tolist()):
            want["relation_universes"][g].add(uid)
            want["relation_id_mappings"][uid][g] = local
        cfg._register_maps(uid, em, rm)
        cfg.trained_embedding_spaces[uid] = TransE.seeded(uid, len(em), len(rm), dim=4, p_norm=1, norm_flag=True)
    cfg.next_universe_id = 40
    cfg.save_model("fast.ckpt")
    assert sorted(calls) == ["id_maps_stream"] * 2 + ["universes_stream"] * 2
    assert len(cfg.__dict__["_pending_maps"]) == 40   # nothing materialised
    fast = torch.load(str(tmp_path / "fast.ckpt"), weights_only=False)
    for k in want:
        _same_container(fast[k], want[k])
    # a read exposes the dictionaries: the next checkpoint pickles them (same result)
    calls.clear()
    _same_container(cfg.entity_universes, want["entity_universes"])
    cfg.save_model("slow.ckpt")
    assert calls == []
    slow = torch.load(str(tmp_path / "slow.ckpt"), weights_only=False)
    for k in want:
        _same_container(slow[k], want[k])
    # replaced dictionaries (best state / load) are never re-derived from the arrays
    cfg2 = _config(checkpoint_dir=str(tmp_path) + "/")
    cfg2.entity_id_mappings = defaultdict(defaultdict_int)
    cfg2._register_maps(0, np.array([5, 6]), np.array([1]))
    assert cfg2.__dict__["_map_log"] is None


def test_pickle_map_streams_edge_cases():
    """No universes, universes without ids, and ids outside int32 (refused)."""
    import pickle
    from openke.config import _map_pickle
    from openke.config.Parallel_Universe_Config import defaultdict_int
    e = pickle.loads(_map_pickle.id_maps_stream([], []))
    assert e == {} and e.default_factory is defaultdict_int
    e = pickle.loads(_map_pickle.universes_stream([], []))
    assert e == {} and e.default_factory is set
    z = np.zeros(0, dtype=np.int64)
    m = pickle.loads(_map_pickle.id_maps_stream([3, 7], [z, np.array([9, 2])]))
    assert list(m.keys()) == [3, 7] and dict(m[3]) == {} and list(m[7].items()) == [(9, 0), (2, 1)]
    s = pickle.loads(_map_pickle.universes_stream([3, 7, 8], [np.array([4, 1]), z, np.array([1, 0])]))
    assert list(s.items()) == [(4, {3}), (1, {3, 8}), (0, {8})]
    with pytest.raises(Exception):
        _map_pickle.id_maps_stream([0], [np.array([1 << 31])])
    with pytest.raises(Exception):
        _map_pickle.universes_stream([1, 0], [np.array([1]), np.array([2])])   # universes not ascending


def test_pickle_map_entry_points_reject_bad_layouts():
    """pt_pickle_id_maps / pt_pickle_universe_sets: offsets not starting at 0, decreasing offsets, universes not
    ascending, negative ids and a too-small buffer are refused (PT_EINVAL); the size query matches the stream."""
    L = _native.lib()
    uids = np.array([0, 3], np.int64)
    off = np.array([0, 2, 3], np.int64)
    ids = np.array([5, 1, 7], np.int64)
    n = np.zeros(1, np.int64)
    for fn in (L.pt_pickle_id_maps, L.pt_pickle_universe_sets):
        assert fn(2, uids.ctypes.data, off.ctypes.data, ids.ctypes.data, None, 0, n.ctypes.data) == 0 and n[0] > 0
        out = np.zeros(int(n[0]), np.uint8)
        assert fn(2, uids.ctypes.data, off.ctypes.data, ids.ctypes.data, out.ctypes.data, len(out), n.ctypes.data) == 0
        assert fn(2, uids.ctypes.data, off.ctypes.data, ids.ctypes.data, out.ctypes.data, len(out) - 1,
                  n.ctypes.data) == 1
        for bad_u, bad_o, bad_i in ((uids, np.array([1, 2, 3], np.int64), ids), (uids, np.array([0, 2, 1], np.int64), ids),
                                    (np.array([3, 0], np.int64), off, ids), (uids, off, np.array([5, -1, 7], np.int64))):
            assert fn(2, bad_u.ctypes.data, bad_o.ctypes.data, bad_i.ctypes.data, None, 0, n.ctypes.data) == 1


def test_checkpoint_after_a_universe_registered_twice(tmp_path):
    """process_universe_mappings called twice for one next_universe_id: the reference merges the second call into the
    same dictionaries (:179-207). The checkpoint then pickles the materialised dictionaries instead of the streams
    (which require ascending universe ids) and holds the merged maps."""
    from openke.config.Parallel_Universe_Config import defaultdict_int
    cfg = _config(checkpoint_dir=str(tmp_path) + "/")
    want = {"entity_id_mappings": defaultdict(defaultdict_int), "relation_id_mappings": defaultdict(defaultdict_int),
            "entity_universes": defaultdict(set), "relation_universes": defaultdict(set)}
    regs = [(0, np.array([5, 9, 2]), np.array([1])), (1, np.array([3, 5]), np.array([0, 2])),
            (1, np.array([7, 3, 8]), np.array([2]))]
    for uid, em, rm in regs:
        for local, g in enumerate(em.tolist()):
            want["entity_universes"][g].add(uid)
            want["entity_id_mappings"][uid][g] = local
        for local, g in enumerate(rm.tolist()):
            want["relation_universes"][g].add(uid)
            want["relation_id_mappings"][uid][g] = local
        cfg._register_maps(uid, em, rm)
        cfg.trained_embedding_spaces[uid] = TransE.seeded(uid, len(em), len(rm), dim=4, p_norm=1, norm_flag=True)
    cfg.next_universe_id = 2
    cfg.save_model("twice.ckpt")
    assert cfg.__dict__["_map_log"] is None
    got = torch.load(str(tmp_path / "twice.ckpt"), weights_only=False)
    for k in want:
        _same_container(got[k], want[k])
