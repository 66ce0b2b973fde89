"""Multi-process (N > 1) logic of the universe path on CPU: universe sharding, the MIN combine of the
link-prediction score rows across ranks (gloo here; RCCL on the GPU box), and the (key, universe)
pair selection of eval_universes. No GPU needed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openke.config.Parallel_Universe_Config import lp_pairs_all, lookup_local, lp_pairs, min_combine, universe_owner


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_univ, E, n_keys, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        # every universe's contribution to every key row (the same on every rank: a pure function of
        # the universe id, like the real universes of seed0 + k)
        contrib = rng.uniform(0.0, 10.0, (n_univ, n_keys, E)).astype(np.float32)
        holds = rng.uniform(size=(n_univ, n_keys)) < 0.4
        rows = torch.full((n_keys, E), float("inf"))
        tup = torch.full((n_keys,), float("inf"))
        for u in range(n_univ):
            if universe_owner(u, world) != rank:
                continue
            for k in range(n_keys):
                if holds[u, k]:
                    rows[k] = torch.minimum(rows[k], torch.from_numpy(contrib[u, k]))
                    tup[k] = min(float(tup[k]), float(contrib[u, k].min()))
        min_combine([rows, tup])
        np.save(os.path.join(out_dir, "rows%d.npy" % rank), rows.numpy())
        np.save(os.path.join(out_dir, "tuple%d.npy" % rank), tup.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_min_combine_across_ranks_equals_single_process(world, tmp_path):
    n_univ, E, n_keys = 7, 13, 5
    mp.spawn(_worker, args=(world, _free_port(), n_univ, E, n_keys, str(tmp_path)), nprocs=world, join=True)
    rng = np.random.default_rng(0)
    contrib = rng.uniform(0.0, 10.0, (n_univ, n_keys, E)).astype(np.float32)
    holds = rng.uniform(size=(n_univ, n_keys)) < 0.4
    ref = np.full((n_keys, E), np.inf, dtype=np.float32)
    for u in range(n_univ):
        for k in range(n_keys):
            if holds[u, k]:
                ref[k] = np.minimum(ref[k], contrib[u, k])
    for r in range(world):
        np.testing.assert_array_equal(np.load(os.path.join(tmp_path, "rows%d.npy" % r)), ref)


def test_universe_owner_is_a_partition():
    for world in (1, 2, 4, 8):
        owners = [universe_owner(u, world) for u in range(100)]
        assert sorted(set(owners)) == list(range(world))
        counts = np.bincount(owners, minlength=world)
        assert counts.max() - counts.min() <= 1


def test_min_combine_single_process_is_identity():
    t = torch.tensor([1.0, float("inf")])
    min_combine([t])
    assert t[0] == 1.0 and t[1] == float("inf")


def test_lp_pairs_match_naive_selection():
    rng = np.random.default_rng(3)
    E, R = 200, 9
    em = rng.choice(E, 40, replace=False)
    rm = rng.choice(R, 4, replace=False)
    key_anchor = rng.integers(0, E, 300)
    key_rel = rng.integers(0, R, 300)
    key_side = rng.integers(0, 2, 300)
    got = lp_pairs(5, em, rm, key_anchor, key_rel, key_side)
    g2l_e = {int(g): l for l, g in enumerate(em)}
    g2l_r = {int(g): l for l, g in enumerate(rm)}
    want = [(k, 5, g2l_e[int(a)], g2l_r[int(r)], int(s)) for k, (a, r, s) in
            enumerate(zip(key_anchor, key_rel, key_side)) if int(a) in g2l_e and int(r) in g2l_r]
    assert got.dtype == np.int32 and got.shape == (len(want), 5)   # pt_lp_pair rows
    assert [tuple(int(x) for x in row) for row in got] == want
    assert len(want) > 0


def test_lp_pairs_all_matches_per_universe():
    rng = np.random.default_rng(5)
    E, R, n_u = 300, 11, 7
    ems = [rng.choice(E, int(rng.integers(0, 60)), replace=False) for _ in range(n_u)]
    rms = [rng.choice(R, int(rng.integers(0, 6)), replace=False) for _ in range(n_u)]
    key_anchor = rng.integers(0, E, 400)
    key_rel = rng.integers(0, R, 400)
    key_side = rng.integers(0, 2, 400)
    want = sorted(tuple(int(x) for x in row) for s in range(n_u)
                  for row in lp_pairs(s, ems[s], rms[s], key_anchor, key_rel, key_side))
    got = lp_pairs_all(ems, rms, key_anchor, key_rel, key_side)
    assert got.dtype == np.int32 and got.flags.c_contiguous
    assert [tuple(int(x) for x in row) for row in got] == want   # by key, then universe slot
    assert len(want) > 0
    assert len(lp_pairs_all([], [], key_anchor, key_rel, key_side)) == 0


def test_lookup_local_absent_and_empty():
    em = np.array([7, 3, 9], dtype=np.int64)
    order = np.argsort(em)
    np.testing.assert_array_equal(lookup_local(em[order], order, [3, 4, 9, 100, -1]), [1, -1, 2, -1, -1])
    np.testing.assert_array_equal(lookup_local(np.zeros(0, np.int64), np.zeros(0, np.int64), [1, 2]), [-1, -1])


# ---------------------------------------------------------------- placement + multi-rank checkpoints --
from openke import _native  # noqa: E402
from openke.config.Parallel_Universe_Config import Parallel_Universe_Config, place_universes, universe_cost  # noqa: E402
from openke.module.model import TransE  # noqa: E402

_CK_E, _CK_R, _CK_N = 60, 5, 7
_CK_PARAM = {"dim": 8, "p_norm": 1, "norm_flag": True}


def test_lpt_placement_balances_and_is_deterministic():
    rng = np.random.default_rng(11)
    costs = {k: universe_cost(int(rng.integers(50, 200)), int(rng.integers(500, 2000)), int(rng.integers(20, 101)))
             for k in range(512)}
    for world in (1, 2, 4, 8):
        owners = place_universes(costs, world)
        assert owners == place_universes(dict(reversed(list(costs.items()))), world)   # order-free
        loads = np.zeros(world)
        for k, r in owners.items():
            loads[r] += costs[k]
        # LPT bound: max load <= mean + the largest single cost
        assert loads.max() <= loads.sum() / world + max(costs.values()) + 1e-6
        rr = np.zeros(world)
        for k in costs:
            rr[k % world] += costs[k]
        assert loads.max() <= rr.max() + 1e-6   # never worse than round-robin here
    assert place_universes({}, 4) == {}
    assert place_universes({3: 1.0, 1: 1.0}, 2) == {1: 0, 3: 1}   # ties by id, then the lowest rank


class _StubTrainLoader(object):
    """The attributes Parallel_Universe_Config reads from its train loader at construction."""

    def __init__(self):
        self.lib = _native.lib()
        self.entTotal, self.relTotal = _CK_E, _CK_R
        self.in_path = "unused/"
        self.batch_size, self.nbatches = 10, 20


def _ck_config(ckpt_dir):
    return Parallel_Universe_Config(train_dataloader=_StubTrainLoader(), valid_dataloader=object(),
                                    embedding_model=TransE, embedding_model_param=dict(_CK_PARAM),
                                    checkpoint_dir=ckpt_dir, initial_num_universes=_CK_N)


def _ck_inject(cfg):
    """Commit _CK_N universes with seeded tables and id maps, as a training wave would (each rank keeps the
    modules of the universes it owns)."""
    for uid in range(_CK_N):
        rng = np.random.default_rng(uid)
        em = np.sort(rng.choice(_CK_E, 10 + 3 * uid, replace=False))
        rm = np.sort(rng.choice(_CK_R, 2 + uid % 3, replace=False))
        torch.manual_seed(100 + uid)
        kge = TransE(len(em), len(rm), **_CK_PARAM)
        cfg._commit({"id": uid, "kge": kge, "ent_remap": em, "rel_remap": rm, "losses": None, "tc": 100,
                     "balance": 0.3, "margin": 1, "epochs": 1, "lr": 0.01, "batch_size": 5, "train_total": 100})


def _ck_summary(cfg):
    return {uid: {k: v.detach().cpu().numpy() for k, v in sp.state_dict().items()}
            for uid, sp in cfg.trained_embedding_spaces.items()}


def _ck_worker(rank, world, port, ckpt_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _ck_config(ckpt_dir)
        _ck_inject(cfg)
        assert sorted(cfg.trained_embedding_spaces) == [u for u in range(_CK_N) if u % world == rank]
        state = torch.get_rng_state()
        cfg.save_model("multi.ckpt")
        assert torch.equal(state, torch.get_rng_state())   # rank 0's rebuild ran under a forked RNG
        assert os.path.exists(os.path.join(ckpt_dir, "multi.ckpt"))   # written before any rank returns
        for name in ("single.ckpt", "multi.ckpt"):
            re = _ck_config(ckpt_dir)
            re.load_parameters(name)
            np.save(os.path.join(ckpt_dir, "%s.rank%d.npy" % (name, rank)),
                    np.array([re.next_universe_id, sorted(re.trained_embedding_spaces), _ck_summary(re),
                              dict(re.universe_owners), {u: dict(m) for u, m in re.entity_id_mappings.items()}],
                             dtype=object), allow_pickle=True)
    finally:
        dist.destroy_process_group()


def _assert_same_spaces(a, b):
    assert sorted(a) == sorted(b)
    for uid in a:
        assert sorted(a[uid]) == sorted(b[uid])
        for k in a[uid]:
            np.testing.assert_array_equal(a[uid][k], b[uid][k])


def test_multi_rank_checkpoint_matches_single_process(tmp_path):
    """two gloo ranks commit the same injected universes (each holding its share),
    save_model gathers them to rank 0 which alone writes; the file equals the single-process checkpoint,
    and load_parameters re-shards either file over the two ranks (a partition, LPT-placed, same weights)."""
    ckpt_dir = str(tmp_path) + os.sep
    single = _ck_config(ckpt_dir)
    _ck_inject(single)
    single.save_model("single.ckpt")
    want = _ck_summary(single)
    mp.spawn(_ck_worker, args=(2, _free_port(), ckpt_dir), nprocs=2, join=True)
    a = torch.load(ckpt_dir + "single.ckpt", weights_only=False)
    b = torch.load(ckpt_dir + "multi.ckpt", weights_only=False)
    assert sorted(a) == sorted(b)
    for k in a:
        if k == "trained_embedding_spaces":
            _assert_same_spaces({u: {n: t.numpy() for n, t in m.state_dict().items()} for u, m in a[k].items()},
                                {u: {n: t.numpy() for n, t in m.state_dict().items()} for u, m in b[k].items()})
        elif k in ("entity_id_mappings", "relation_id_mappings", "entity_universes", "relation_universes"):
            assert {u: v for u, v in a[k].items() if v} == {u: v for u, v in b[k].items() if v}, k
        elif k != "embedding_model":
            assert a[k] == b[k], k
    for name in ("single.ckpt", "multi.ckpt"):
        parts = [np.load(os.path.join(ckpt_dir, "%s.rank%d.npy" % (name, r)), allow_pickle=True) for r in range(2)]
        owners = parts[0][3]
        assert owners == parts[1][3] and sorted(owners) == list(range(_CK_N))
        got = {}
        for r, p in enumerate(parts):
            assert p[0] == _CK_N
            assert p[1] == sorted(u for u, o in owners.items() if o == r)
            assert p[4] == {u: dict(m) for u, m in single.entity_id_mappings.items()}   # maps stay complete
            got.update(p[2])
        _assert_same_spaces(got, want)


def test_lpt_loads_carry_across_waves():
    """placement per training wave keeps each rank's cumulative cost. One-universe waves spread
    over every rank (a fresh LPT per wave would give rank 0 all of them), and wave-by-wave placement of
    equal-cost universes is exactly round-robin."""
    rng = np.random.default_rng(2)
    costs = {k: float(rng.integers(1, 100)) for k in range(40)}
    for world in (2, 3, 8):
        loads = [0.0] * world
        owners = {}
        for k in range(40):
            owners.update(place_universes({k: costs[k]}, world, loads))
        assert sorted(set(owners.values())) == list(range(world))
        got = np.zeros(world)
        for k, r in owners.items():
            got[r] += costs[k]
        np.testing.assert_allclose(got, loads)
        assert max(loads) <= sum(loads) / world + max(costs.values()) + 1e-9   # online greedy bound
        loads = [0.0] * world
        eq = {}
        for w0 in range(0, 12, 3):   # waves of 3 equal-cost universes
            eq.update(place_universes({k: 1.0 for k in range(w0, w0 + 3)}, world, loads))
        assert np.bincount(list(eq.values()), minlength=world).max() - \
            np.bincount(list(eq.values()), minlength=world).min() <= 1
    with pytest.raises(ValueError):
        place_universes({0: 1.0}, 2, [0.0])


def _dup_worker(rank, world, port, ckpt_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the one-universe protocol registers every universe on every rank (add_embedding_space has no owner
        # test): the same weights everywhere
        cfg = _ck_config(ckpt_dir)
        for uid in range(_CK_N):
            rng = np.random.default_rng(uid)
            em = np.sort(rng.choice(_CK_E, 10 + 3 * uid, replace=False))
            rm = np.sort(rng.choice(_CK_R, 2 + uid % 3, replace=False))
            torch.manual_seed(100 + uid)
            cfg.add_embedding_space(TransE(len(em), len(rm), **_CK_PARAM))
            cfg._register_maps(uid, em, rm)
            cfg.next_universe_id += 1
        cfg.save_model("dup.ckpt")
    finally:
        dist.destroy_process_group()


def test_multi_rank_checkpoint_with_every_rank_holding_every_universe(tmp_path):
    """universes held by more than one rank are saved once (the owner's copy), not rejected."""
    ckpt_dir = str(tmp_path) + os.sep
    single = _ck_config(ckpt_dir)
    _ck_inject(single)
    mp.spawn(_dup_worker, args=(2, _free_port(), ckpt_dir), nprocs=2, join=True)
    b = torch.load(ckpt_dir + "dup.ckpt", weights_only=False)
    assert b["next_universe_id"] == _CK_N
    _assert_same_spaces(_ck_summary(single),
                        {u: {n: t.numpy() for n, t in m.state_dict().items()}
                         for u, m in b["trained_embedding_spaces"].items()})


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_gpus_ranks(n):
    """`bench.py --gpus N` started without a torch.distributed environment launches N ranks itself
    (torch.distributed.run, 127.0.0.1) and their world size equals --gpus (gloo rehearsal, no GPU work)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["PT_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(n), "--launch-check"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["world_size_env"] == n


def test_bench_rejects_world_size_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero instead of printing a line."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "4", "--launch-check"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and not p.stdout.strip().startswith("{")


def test_lp_pairs_all_edges():
    """The native pair join (pt_lp_pairs): universes without entities or relations, keys whose anchor or relation
    no universe holds (ids beyond every universe's), and a key set of one; the rows are the per-universe
    selection's, ordered by key then universe."""
    em = [np.array([5, 2, 9]), np.zeros(0, np.int64), np.array([2, 40])]
    rm = [np.array([1]), np.array([0, 1]), np.zeros(0, np.int64)]
    ka, kr, ks = np.array([2, 9, 100, 2]), np.array([1, 1, 1, 0]), np.array([0, 1, 1, 0])
    got = [tuple(int(x) for x in row) for row in lp_pairs_all(em, rm, ka, kr, ks)]
    assert got == [(0, 0, 1, 0, 0), (1, 0, 2, 0, 1)]
    assert [tuple(int(x) for x in r) for r in lp_pairs_all(em, rm, np.array([9]), np.array([1]), np.array([1]))] == \
        [(0, 0, 2, 0, 1)]
    assert lp_pairs_all(em, rm, np.zeros(0), np.zeros(0), np.zeros(0)).shape == (0, 5)


def test_lp_pairs_native_rejects_bad_layouts():
    import ctypes
    from openke import _native
    L = _native.lib()
    off = np.array([0, 2], np.int64)
    bad_off = np.array([1, 2], np.int64)       # offsets must start at 0
    ids = np.array([3, -1], np.int64)          # ids must be >= 0
    good = np.array([3, 4], np.int64)
    k = np.array([3], np.int64)
    n = np.zeros(1, np.int64)
    call = lambda eo, ei: L.pt_lp_pairs(1, eo.ctypes.data, ei.ctypes.data, off.ctypes.data, good.ctypes.data, 1,
                                        k.ctypes.data, k.ctypes.data, k.ctypes.data, None, 0, n.ctypes.data)
    assert call(off, good) == 0 and n[0] == 1
    assert call(bad_off, good) == 1
    assert call(off, ids) == 1
    out = np.zeros((1, 5), np.int32)
    rel = np.array([3, 4], np.int64)
    rc = L.pt_lp_pairs(1, off.ctypes.data, good.ctypes.data, off.ctypes.data, rel.ctypes.data, 1, k.ctypes.data,
                       k.ctypes.data, k.ctypes.data, out.ctypes.data, 0, n.ctypes.data)   # no room for the row
    assert rc == 1


def _synthetic_universe(uid, E_glob=40, R_glob=4, D=5):
    """A universe of id uid (a pure function of it, like seed0 + k): local -> global maps and tables."""
    rng = np.random.default_rng(100 + uid)
    E = int(rng.integers(3, 12))
    R = int(rng.integers(1, R_glob + 1))
    em = np.sort(rng.choice(E_glob, E, replace=False)).astype(np.int64)
    rm = np.sort(rng.choice(R_glob, R, replace=False)).astype(np.int64)
    nv = torch.from_numpy(rng.standard_normal((R, D)).astype(np.float32)) if uid % 2 else None
    return {"ent": torch.from_numpy(rng.standard_normal((E, D)).astype(np.float32)),
            "rel": torch.from_numpy(rng.standard_normal((R, D)).astype(np.float32)), "nv": nv, "em": em, "rm": rm,
            "dim": D}


def _toy_rows(unis, keys, E_glob=40):
    """Key rows as the LP fold fills them: per (side, anchor, rel) key the MIN over every universe holding anchor and
    rel of a score of each of its entities (here |anchor + rel - e|_1 over the universe's rows)."""
    rows = torch.full((len(keys), E_glob), float("inf"))
    for u in unis:
        g2l = {int(g): i for i, g in enumerate(u["em"])}
        r2l = {int(g): i for i, g in enumerate(u["rm"])}
        for k, (side, anchor, r) in enumerate(keys):
            if anchor in g2l and r in r2l:
                a = u["ent"][g2l[anchor]] + (u["rel"][r2l[r]] if side else -u["rel"][r2l[r]])
                s = (a[None, :] - u["ent"]).abs().sum(1)
                idx = torch.from_numpy(u["em"])
                rows[k, idx] = torch.minimum(rows[k, idx], s)
    return rows


def _toy_ranks(rows, truths):
    val = rows.gather(1, truths[:, None])
    return [((rows < val).sum(1)).numpy().astype(np.int64)]


def _gather_worker(rank, world, port, n_univ, out_dir):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = [_synthetic_universe(u) for u in range(n_univ) if u % world == rank]
        got = bench.gather_universes(mine, world)
        rng = np.random.default_rng(7)
        keys = [(int(rng.integers(0, 2)), int(rng.integers(0, 40)), int(rng.integers(0, 4))) for _ in range(25)]
        truths = torch.from_numpy(rng.integers(0, 40, 25))
        rows = _toy_rows(mine, keys)
        min_combine([rows])
        d_dist = bench.rank_digest(_toy_ranks(rows, truths))
        d_n1 = bench.rank_digest(_toy_ranks(_toy_rows(got, keys), truths))
        np.save(os.path.join(out_dir, "order%d.npy" % rank),
                np.array([int(u["em"][0]) * 1000 + u["ent"].shape[0] for u in got]))
        with open(os.path.join(out_dir, "digest%d.txt" % rank), "w") as f:
            f.write("%s %s %d" % (d_dist, d_n1, len(got)))
        for u in got:   # every gathered universe equals its source
            src = [v for v in (_synthetic_universe(k) for k in range(n_univ)) if np.array_equal(v["em"], u["em"])
                   and np.array_equal(v["rm"], u["rm"])]
            assert len(src) == 1
            for k in ("ent", "rel", "nv"):
                assert (src[0][k] is None) == (u[k] is None)
                if u[k] is not None:
                    assert torch.equal(src[0][k], u[k])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pu_c4_lp_gather_and_digest(world, tmp_path):
    """bench.py's pu_c4_lp check (N > 1): every rank's universes gathered to every rank (gather_universes, padded
    all_gathers of sizes, tables and remaps), and the ranks from the MIN-combined rows of each rank's own universes
    equal, digest for digest, the ranks an N = 1 recomputation over the gathered universes gives."""
    n_univ = 7
    mp.spawn(_gather_worker, args=(world, _free_port(), n_univ, str(tmp_path)), nprocs=world, join=True)
    digests = [open(os.path.join(tmp_path, "digest%d.txt" % r)).read().split() for r in range(world)]
    for d_dist, d_n1, n in digests:
        assert d_dist == d_n1 and int(n) == n_univ
    assert len({d[0] for d in digests}) == 1
    orders = [np.load(os.path.join(tmp_path, "order%d.npy" % r)) for r in range(world)]
    for o in orders[1:]:
        np.testing.assert_array_equal(o, orders[0])
