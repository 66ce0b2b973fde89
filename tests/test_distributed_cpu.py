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
    assert sorted(tuple(int(x) for x in row) for row in got) == want
    assert len(want) > 0
    assert len(lp_pairs_all([], [], key_anchor, key_rel, key_side)) == 0


def test_lookup_local_absent_and_empty():
    em = np.array([7, 3, 9], dtype=np.int64)
    order = np.argsort(em)
    np.testing.assert_array_equal(lookup_local(em[order], order, [3, 4, 9, 100, -1]), [1, -1, 2, -1, -1])
    np.testing.assert_array_equal(lookup_local(np.zeros(0, np.int64), np.zeros(0, np.int64), [1, 2]), [-1, -1])
