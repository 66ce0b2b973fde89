"""Pin the CPU oracle to the reference: every check compares oracle output with golden vectors the
reference itself produced (tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest

import oracle
from helpers import DATASETS, IllConditioned, assert_tables_close, golden, load, pu_energy, torch_init_tables
from conftest import KG_SMALL


def test_glibc_rand_matches_reference_libc():
    z = load(golden("glibc_rand.npz")[0])
    for seed, vals in zip(z["seeds"], z["values"]):
        g = oracle.GlibcRand(int(seed))
        got = [g.next() for _ in range(len(vals))]
        assert got == vals.tolist(), seed


@pytest.mark.parametrize("path", golden("sampler_*.npz"), ids=lambda p: p.split("/")[-1])
def test_sampler_bit_exact(path):
    z = load(path)
    kg = oracle.KG.load(DATASETS[str(z["dataset"])])
    threads, bs, neg = int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"])
    st = oracle.GlibcRand(int(z["seed"])).rand_reset(threads)
    for c in range(z["batch_h"].shape[0]):
        h, t, r, y = kg.sample(st, threads, bs, neg, int(z["bern"]), int(z["filter"]))
        np.testing.assert_array_equal(h, z["batch_h"][c])
        np.testing.assert_array_equal(t, z["batch_t"][c])
        np.testing.assert_array_equal(r, z["batch_r"][c])
        np.testing.assert_array_equal(y, z["batch_y"][c])


MODE_OF_CALL = {"n": 0, "h": -1, "t": 1}


def call_modes(calls):
    """sampling() mode of each loader call; cross_sampling flips its flag first (TrainDataLoader.py:240-246)."""
    flag, out = 0, []
    for c in calls:
        if c == "c":
            flag = 1 - flag
            out.append(1 if flag else -1)
        else:
            out.append(MODE_OF_CALL[c])
    return out


@pytest.mark.parametrize("path", golden("samplermode_*.npz"), ids=lambda p: p.split("/")[-1])
def test_sampler_modes_bit_exact(path):
    """sampling_head / sampling_tail / cross_sampling and neg_rel relation corruption vs the reference."""
    z = load(path)
    kg = oracle.KG.load(DATASETS[str(z["dataset"])])
    threads, bs = int(z["threads"]), int(z["batch_size"])
    neg, neg_rel = int(z["neg_ent"]), int(z["neg_rel"])
    st = oracle.GlibcRand(int(z["seed"])).rand_reset(threads)
    modes = call_modes(str(z["calls"]))
    assert [{0: "normal", -1: "head_batch", 1: "tail_batch"}[m] for m in modes] == list(z["modes"])
    for c, mode in enumerate(modes):
        h, t, r, y = kg.sample_ex(st, threads, bs, neg, neg_rel, mode, int(z["bern"]), int(z["filter"]))
        np.testing.assert_array_equal(h, z["batch_h"][c])
        np.testing.assert_array_equal(t, z["batch_t"][c])
        np.testing.assert_array_equal(r, z["batch_r"][c])
        np.testing.assert_array_equal(y, z["batch_y"][c])


@pytest.mark.parametrize("path", golden("train_*.npz"), ids=lambda p: p.split("/")[-1])
def test_train_steps_match_reference(path):
    z = load(path)
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    ent, rel, nv = torch_init_tables(model, kg.ent_total, kg.rel_total, dim, int(z["torch_seed"]))
    np.testing.assert_array_equal(ent, z["init_ent_embeddings"])
    np.testing.assert_array_equal(rel, z["init_rel_embeddings"])
    if model == "TransH":
        np.testing.assert_array_equal(nv, z["init_norm_vector"])
    threads, bs, neg = int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"])
    st = oracle.GlibcRand(int(z["seed"])).rand_reset(threads)
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
    ada = str(z["opt"]) == "adagrad"
    ill = IllConditioned()
    for s in range(int(z["steps"])):
        h, t, r, _ = kg.sample(st, threads, bs, neg, int(z["bern"]), int(z["filter"]))
        np.testing.assert_array_equal(h, z["batch_h"][s])
        np.testing.assert_array_equal(t, z["batch_t"][s])
        np.testing.assert_array_equal(r, z["batch_r"][s])
        loss = oracle.train_step(model, p, bool(z["norm_flag"]), str(z["opt"]), float(z["lr"]), float(z["margin"]),
                                 ent, rel, nv, accs, h, t, r, bs, neg)
        assert abs(loss - z["losses"][s]) <= 1e-5 * max(1.0, abs(z["losses"][s])), (s, loss, z["losses"][s])
        if ada:
            for name, a in zip(("ent", "rel", "norm"), accs):
                ill.update(name, a)
        if s == 0:
            assert_tables_close(ent, z["step1_ent_embeddings"], 2e-6, ill.get("ent"))
            assert_tables_close(rel, z["step1_rel_embeddings"], 2e-6, ill.get("rel"))
    assert_tables_close(ent, z["final_ent_embeddings"], 1e-5, ill.get("ent"))
    assert_tables_close(rel, z["final_rel_embeddings"], 1e-5, ill.get("rel"))
    if model == "TransH":
        assert_tables_close(nv, z["final_norm_vector"], 1e-5, ill.get("norm"))


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_universes_match_reference(path):
    z = load(path)
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    seed0, n_univ, epochs = int(z["seed0"]), int(z["n_univ"]), int(z["epochs"])
    universes = []
    noisy_universes = []
    for u in range(n_univ):
        rng = oracle.GlibcRand(seed0 + u)
        st = rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, int(z["u%d_tc" % u]), float(z["u%d_balance" % u]))
        assert ug.train_total == int(z["u%d_train_total" % u])
        np.testing.assert_array_equal(em, z["u%d_ent_remap" % u])
        np.testing.assert_array_equal(rm, z["u%d_rel_remap" % u])
        bs = ug.train_total // 20
        h, t, r, _ = ug.sample(st.copy(), 8, bs, 1, 0, 0)
        np.testing.assert_array_equal(h, z["u%d_b_h" % u])
        np.testing.assert_array_equal(t, z["u%d_b_t" % u])
        np.testing.assert_array_equal(r, z["u%d_b_r" % u])
        # train the universe exactly as Parallel_Universe_Config.train_embedding_space does (:228-258)
        ent, rel, nv = torch_init_tables(model, ug.ent_total, ug.rel_total, dim, seed0 + u)
        accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
        ill = IllConditioned()
        for _ in range(epochs * 20):
            h, t, r, _ = ug.sample(st, 8, bs, 1, 0, 0)
            for name, a in zip(("ent", "rel", "norm"), accs):
                ill.before(name, a)
            oracle.train_step(model, p, True, "adagrad", float(z["u%d_lr" % u]), float(z["u%d_margin" % u]),
                              ent, rel, nv, accs, h, t, r, bs, 1)
            for name, a in zip(("ent", "rel", "norm"), accs):
                ill.after(name, a)
        if ill.events == 0:
            # no noise-decided Adagrad step: the whole trajectory must match
            assert_tables_close(ent, z["u%d_ent" % u], 2e-5)
            assert_tables_close(rel, z["u%d_rel" % u], 2e-5)
            if model == "TransH":
                assert_tables_close(nv, z["u%d_norm" % u], 2e-5)
        else:
            # a gradient component cancelled to rounding level and Adagrad turned its rounding noise
            # into a +-lr step; from there the trajectory depends on summation order (the reference's
            # own CPU and GPU backends differ the same way). Per-step parity is covered elsewhere.
            noisy_universes.append(u)
        universes.append({"ent_remap": em, "rel_remap": rm, "ent": z["u%d_ent" % u], "rel": z["u%d_rel" % u],
                          "norm": z["u%d_norm" % u] if model == "TransH" else None})
    assert len(noisy_universes) <= n_univ // 2, noisy_universes
    # link prediction over the reference's own trained universes
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    test = oracle.sort_test(*oracle.read_triples(KG_SMALL + "test2id.txt"))
    con_h, con_t = pu_energy(kg.ent_total, universes, test, model, p, dim)
    met, _ = oracle.link_prediction(kg.ent_total, all_tr, test, con_h, con_t)
    np.testing.assert_allclose(met, z["lp"].astype(np.float32), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("path", golden("lp_*.npz"), ids=lambda p: p.split("/")[-1])
def test_link_prediction_matches_reference(path):
    z = load(path)
    model, p = str(z["model"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    E = kg.ent_total
    ent, rel = z["ent_embeddings"], z["rel_embeddings"]
    nv = z["norm_vector"] if model == "TransH" else None
    test = oracle.sort_test(*oracle.read_triples(KG_SMALL + "test2id.txt"))
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    n = len(test[0])
    con_h = np.zeros((n, E), dtype=np.float32)
    con_t = np.zeros((n, E), dtype=np.float32)
    for q in range(n):
        h, t, r = (int(x[q]) for x in test)
        con_h[q] = oracle.score(model, p, True, "head_batch", ent, rel, nv, oracle.candidates(E, h), [t], [r])
        con_t[q] = oracle.score(model, p, True, "tail_batch", ent, rel, nv, [h], oracle.candidates(E, t), [r])
    met, _ = oracle.link_prediction(E, all_tr, test, con_h, con_t)
    np.testing.assert_allclose(met, z["metrics"].astype(np.float32), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("path", golden("lpt_*.npz"), ids=lambda p: p.split("/")[-1])
def test_type_constrained_link_prediction_matches_reference(path):
    """Tester.run_link_prediction(type_constrain=True) after importTypeFiles (Test.h:127-502): the
    constrained metrics, and the unconstrained ones of the same run."""
    z = load(path)
    model, p = str(z["model"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    E = kg.ent_total
    ent, rel = z["ent_embeddings"], z["rel_embeddings"]
    nv = z["norm_vector"] if model == "TransH" else None
    test = oracle.sort_test(*oracle.read_triples(KG_SMALL + "test2id.txt"))
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    n = len(test[0])
    con_h = np.zeros((n, E), dtype=np.float32)
    con_t = np.zeros((n, E), dtype=np.float32)
    for q in range(n):
        h, t, r = (int(x[q]) for x in test)
        con_h[q] = oracle.score(model, p, True, "head_batch", ent, rel, nv, oracle.candidates(E, h), [t], [r])
        con_t[q] = oracle.score(model, p, True, "tail_batch", ent, rel, nv, [h], oracle.candidates(E, t), [r])
    types = oracle.read_types(KG_SMALL + "type_constrain.txt", kg.rel_total)
    met_tc, _ = oracle.rank_constrained(E, all_tr, test, con_h, con_t, types)
    np.testing.assert_allclose(met_tc, z["metrics_tc"].astype(np.float32), rtol=1e-6, atol=1e-7)
    met, _ = oracle.link_prediction(E, all_tr, test, con_h, con_t)
    np.testing.assert_allclose(met, z["metrics"].astype(np.float32), rtol=1e-6, atol=1e-7)


def valid_hit10(ranks):
    """getValidHit10 (Valid.h:244-256) from filtered ranks: per side #{rank < 10} / validTotal, then mean."""
    _, fh, _, ft = ranks
    n = np.float32(len(fh))
    return float((np.float32(np.count_nonzero(fh < 10)) / n + np.float32(np.count_nonzero(ft < 10)) / n)
                 / np.float32(2))


@pytest.mark.parametrize("path", golden("val_*.npz"), ids=lambda p: p.split("/")[-1])
def test_validator_hit10_matches_reference(path):
    """Validator.valid() (validHead/validTail + getValidHit10 over the valid split) == the reference."""
    z = load(path)
    model, p = str(z["model"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    E = kg.ent_total
    ent, rel = z["ent_embeddings"], z["rel_embeddings"]
    nv = z["norm_vector"] if model == "TransH" else None
    ev = oracle.sort_test(*oracle.read_triples(KG_SMALL + "valid2id.txt"))
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    n = len(ev[0])
    con_h = np.zeros((n, E), dtype=np.float32)
    con_t = np.zeros((n, E), dtype=np.float32)
    for q in range(n):
        h, t, r = (int(x[q]) for x in ev)
        con_h[q] = oracle.score(model, p, True, "head_batch", ent, rel, nv, oracle.candidates(E, h), [t], [r])
        con_t[q] = oracle.score(model, p, True, "tail_batch", ent, rel, nv, [h], oracle.candidates(E, t), [r])
    _, ranks = oracle.link_prediction(E, all_tr, ev, con_h, con_t)
    assert valid_hit10(ranks) == pytest.approx(float(z["hit10"]), rel=1e-6, abs=1e-7)


@pytest.mark.parametrize("model", ["TransE", "TransH"])
def test_grad_mass_is_the_step_gradient(model):
    """oracle.grad_mass (the tolerance model of helpers.assert_step_close): its gradient is the one the SGD step
    applies (lr 1: w_after == w + (-1) * g bit for bit), and the contributions' magnitude sum bounds it."""
    kg = oracle.KG.load(KG_SMALL)
    rng = np.random.default_rng(5)
    d = 21
    ent = rng.uniform(-0.3, 0.3, (kg.ent_total, d)).astype(np.float32)
    rel = rng.uniform(-0.3, 0.3, (kg.rel_total, d)).astype(np.float32)
    nv = rng.uniform(-0.3, 0.3, (kg.rel_total, d)).astype(np.float32) if model == "TransH" else None
    st = oracle.GlibcRand(9).rand_reset(8)
    h, t, r, _ = kg.sample(st, 8, 40, 3, 1, 1)
    gm = oracle.grad_mass(model, 1, True, 2.0, ent, rel, nv, h, t, r, 40, 3)
    before = {"ent": ent.copy(), "rel": rel.copy(), "norm": None if nv is None else nv.copy()}
    oracle.train_step(model, 1, True, "sgd", 1.0, 2.0, ent, rel, nv, (None, None, None), h, t, r, 40, 3)
    for name, after in (("ent", ent), ("rel", rel), ("norm", nv)):
        if after is None:
            continue
        x = gm[name]
        g, m, a = x["g"], x["mass"], x["abs"]
        np.testing.assert_array_equal(after, before[name] + (-1.0) * g)
        assert (m >= np.abs(g) * (1 - 1e-6)).all() and m.max() > 0
        assert (a >= m * (1 - 1e-5)).all()   # the absolute evaluation bounds the contributions' magnitudes
        touched = (m > 0).any(axis=1)
        assert (x["n"][touched] > 0).all() and (x["n"][~touched] == 0).all()
