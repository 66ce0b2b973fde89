"""Real-scale pinning, CPU side: the oracle and the library's host code against the reference's own outputs on
the reference's own data (tests/golden/real*.npz, written by tests/golden/make_golden.py from
/root/reference/benchmarks/{WN18,FB15K} and /root/reference/best_models/*.ckpt; see tests/realdata.py).

* sampler: the oracle's sampling() (Base.cpp:266-310) at WN18 scale (E = 40,943, N = 141,442) equal, call by call,
  to the SHA-1 of the reference's batches (bs 1,414 and 100, bern / filter on and off, bs 2,000 x 25 negatives);
* universes: getParallelUniverse (UniverseConstructor.h:327-397) for seeds 4-11 on WN18 - the oracle's and the
  library's host construction (pt_universe_build_many) give the reference's remaps, sizes and batches;
* link prediction: the oracle's scores on the reference-trained TransH WN18 / TransE FB15K tables against the
  reference's own score vectors (torch CPU), its ranks (raw, filtered, type-constrained) against the reference's
  per-query counts, and the reference's float metric accumulation (Test.h:398-454) reproduced from those counts
  by both the oracle and the library (pt_lp_metrics).
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle
import realdata
from helpers import golden, load
from openke import _native

TIE_REL = 1e-6   # candidates within this relative distance of the truth's score are near-ties


def sha1(*arrays):
    m = hashlib.sha1()
    for a in arrays:
        m.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return m.hexdigest()


@pytest.fixture(scope="session")
def real_dirs(tmp_path_factory):
    base = tmp_path_factory.mktemp("real")
    return {name: realdata.write_dataset(golden("real_%s.npz" % name)[0], str(base / name))
            for name in ("wn18", "fb15k")}


def test_real_data_fixture_shapes(real_dirs):
    kg = oracle.KG.load(real_dirs["wn18"])
    assert (kg.ent_total, kg.rel_total, kg.train_total) == (40943, 18, 141442)
    kg = oracle.KG.load(real_dirs["fb15k"])
    assert (kg.ent_total, kg.rel_total) == (14951, 1345)


@pytest.mark.parametrize("path", golden("realsampler_*.npz"), ids=lambda p: p.split("/")[-1])
def test_oracle_sampler_matches_reference_at_wn18_scale(path, real_dirs):
    z = load(path)
    kg = oracle.KG.load(real_dirs["wn18"])
    st = oracle.GlibcRand(int(z["seed"])).rand_reset(8)
    bs, neg = int(z["batch_size"]), int(z["neg_ent"])
    for c, want in enumerate(z["digests"]):
        h, t, r, _ = kg.sample(st, 8, bs, neg, int(z["bern"]), int(z["filter"]))
        if c == 0:
            np.testing.assert_array_equal(np.stack([h, t, r]), z["first"].astype(np.int64))
        assert sha1(h, t, r) == str(want), "call %d" % c


def _universe_golden():
    return load(golden("realuniverses_wn18.npz")[0])


def test_oracle_universes_match_reference_at_wn18_scale(real_dirs):
    z = _universe_golden()
    kg = oracle.KG.load(real_dirs["wn18"])
    for s in z["seeds"]:
        s = int(s)
        rng = oracle.GlibcRand(s)
        st = rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, int(z["s%d_tc" % s]), float(z["s%d_balance" % s]))
        assert ug.train_total == int(z["s%d_train_total" % s])
        np.testing.assert_array_equal(em, z["s%d_ent_remap" % s])
        np.testing.assert_array_equal(rm, z["s%d_rel_remap" % s])
        bs = int(z["s%d_batch_size" % s])
        assert bs == ug.train_total // 20
        for c, want in enumerate(z["s%d_digests" % s]):
            h, t, r, _ = ug.sample(st, 8, bs, 1, 0, 0)
            assert sha1(h, t, r) == str(want), "seed %d call %d" % (s, c)


def test_library_universe_construction_matches_reference_at_wn18_scale(real_dirs):
    """pt_universe_build_many (host C++, 4 threads) on WN18: the reference's remaps and sizes for seeds 4-11."""
    z = _universe_golden()
    L = _native.lib()
    g = ctypes.c_void_p()
    _native.check(L.pt_graph_load(real_dirs["wn18"].encode(), ctypes.byref(g)))
    seeds = np.array(z["seeds"], dtype=np.int64)
    n = len(seeds)
    tcs = np.array([int(z["s%d_tc" % s]) for s in seeds], dtype=np.int64)
    bals = np.array([float(z["s%d_balance" % s]) for s in seeds], dtype=np.float32)
    outs = (ctypes.c_void_p * n)()
    _native.check(L.pt_universe_build_many(g, n, seeds.ctypes.data, 8, tcs.ctypes.data, bals.ctypes.data, 4, outs))
    for i, s in enumerate(seeds):
        U = ctypes.c_void_p(outs[i])
        assert L.pt_universe_train_total(U) == int(z["s%d_train_total" % s])
        E, R = L.pt_universe_ent_total(U), L.pt_universe_rel_total(U)
        em, rm = np.zeros(E, dtype=np.int64), np.zeros(R, dtype=np.int64)
        _native.check(L.pt_universe_remaps(U, em.ctypes.data, rm.ctypes.data))
        np.testing.assert_array_equal(em, z["s%d_ent_remap" % s])
        np.testing.assert_array_equal(rm, z["s%d_rel_remap" % s])
        L.pt_universe_free(U)
    L.pt_graph_free(g)


# ------------------------------------------------------------------------------------------------ link prediction
def lp_cases():
    return golden("reallp_*.npz")


def tables(z):
    return z["ent_embeddings"], z["rel_embeddings"], (z["norm_vector"] if "norm_vector" in z.files else None)


def oracle_rows(z, idx):
    """The oracle's candidate-order score rows (getHeadBatch / getTailBatch order, Test.h:37-107) for queries idx."""
    ent, rel, nv = tables(z)
    E = ent.shape[0]
    model, p = str(z["model"]), int(z["p_norm"])
    q = z["queries"].astype(np.int64)
    heads, tails = np.zeros((len(idx), E), np.float32), np.zeros((len(idx), E), np.float32)
    for i, k in enumerate(idx):
        h, t, r = q[k]
        one = lambda x: np.array([x], dtype=np.int64)   # noqa: E731
        heads[i] = oracle.score(model, p, True, "head_batch", ent, rel, nv, oracle.candidates(E, h), one(t), one(r))
        tails[i] = oracle.score(model, p, True, "tail_batch", ent, rel, nv, one(h), oracle.candidates(E, t), one(r))
    return heads, tails


def tie_counts(rows):
    """Candidates whose score lies within TIE_REL of the truth's (column 0): the only comparisons that a last-ulp
    difference between two correct implementations can flip."""
    s0 = rows[:, :1]
    return (np.abs(rows[:, 1:] - s0) <= TIE_REL * np.maximum(1.0, np.abs(s0))).sum(axis=1)


@pytest.mark.parametrize("path", lp_cases(), ids=lambda p: p.split("/")[-1])
def test_oracle_scores_match_reference_vectors(path):
    """Score vectors of the reference's torch model on its own trained table (TransE.py:46-74, TransH.py:52-93)."""
    z = load(path)
    idx = [int(k) for k in z["vec_queries"]]
    heads, tails = oracle_rows(z, idx)
    np.testing.assert_allclose(heads, z["vec_head"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(tails, z["vec_tail"], rtol=1e-6, atol=1e-6)


def _known(dirname):
    trips = [realdata.read_triples(dirname + f) for f in realdata.SPLITS]
    a = np.concatenate(trips)
    return a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()


@pytest.mark.parametrize("path", lp_cases(), ids=lambda p: p.split("/")[-1])
def test_oracle_ranks_match_reference_counts(path, real_dirs):
    """The oracle's testHead / testTail restatement on its own scores: every query's raw and filtered count (and the
    type-constrained ones) equals the reference's, except by at most the query's near-ties."""
    z = load(path)
    ds = real_dirs[str(z["dataset"])]
    n = min(200, z["queries"].shape[0])
    idx = list(range(n))
    heads, tails = oracle_rows(z, idx)
    q = z["queries"][:n].astype(np.int64)
    test = (q[:, 0], q[:, 1], q[:, 2])
    E = heads.shape[1]
    _, (rh, fh, rt, ft) = oracle.link_prediction(E, _known(ds), test, heads, tails)
    ties = [tie_counts(heads), tie_counts(tails)]
    want = z["ranks"][:, :n].astype(np.int64)
    got = [rh, fh, rt, ft]
    if int(z["type_constrain"]):
        types = oracle.read_types(ds + "type_constrain.txt", int(z["rel_embeddings"].shape[0]))
        _, tc = oracle.rank_constrained(E, _known(ds), test, heads, tails, types)
        got += list(tc)
    exact = 0
    for k, g in enumerate(got):
        d = np.abs(g - want[k])
        tie = ties[(k % 4) // 2]
        assert (d <= tie).all(), (str(z["rank_names"][k]), np.nonzero(d > tie)[0][:10])
        exact += int((d == 0).sum())
    assert exact >= 0.99 * len(got) * n, exact


@pytest.mark.parametrize("path", lp_cases(), ids=lambda p: p.split("/")[-1])
def test_metrics_from_reference_counts(path):
    """Test.h's float accumulation (MRR, MR, Hits@10/3/1 over head and tail, Test.h:398-454) of the reference's
    per-query counts, by the oracle and by the library (pt_lp_metrics), equals the metrics the reference's
    run_link_prediction returned - at the full test split (5,000 WN18 queries)."""
    z = load(path)
    rk = z["ranks"].astype(np.int64)
    n = rk.shape[1]
    met = oracle.metrics_from_ranks(rk[1], rk[3])
    np.testing.assert_array_equal(met.astype(np.float32), z["metrics"].astype(np.float32))
    L = _native.lib()
    out = np.zeros(10, dtype=np.float32)
    r = [np.ascontiguousarray(x) for x in rk[:4]]
    _native.check(L.pt_lp_metrics(r[0].ctypes.data, r[1].ctypes.data, r[2].ctypes.data, r[3].ctypes.data, n,
                                  out.ctypes.data))
    np.testing.assert_array_equal(out[:5], z["metrics"].astype(np.float32))
    if int(z["type_constrain"]):
        c = [np.ascontiguousarray(x) for x in rk[4:8]]
        _native.check(L.pt_lp_metrics(c[0].ctypes.data, c[1].ctypes.data, c[2].ctypes.data, c[3].ctypes.data, n,
                                      out.ctypes.data))
        np.testing.assert_array_equal(out[:5], z["metrics_tc"].astype(np.float32))
