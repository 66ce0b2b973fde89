"""GPU parity of the PuTransE / PuTransH path: the persistent multi-universe trainer
(pt_universes_train via Parallel_Universe_Config) and the universe link prediction (pt_lp_min_scores +
pt_rank_rows) against the reference's golden universes and the CPU oracle. pytest -m gpu."""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import KG_SMALL
from helpers import assert_step_close, golden, load, metrics_match_ranks, pu_energy, step_noise, torch_init_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _pu(z, tmp_path, missing="last_rank", valid_steps=10 ** 6):
    from openke.config import Parallel_Universe_Config
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.model import TransE, TransH
    dl = TrainDataLoader(in_path=KG_SMALL, nbatches=20, threads=8, sampling_mode="normal", bern_flag=0,
                         filter_flag=0, neg_ent=1, neg_rel=0, random_seed=int(z["seed"]))
    test_dl = TestDataLoader(dl.in_path, "link")
    cls = TransE if str(z["model"]) == "TransE" else TransH
    return Parallel_Universe_Config(training_identifier="t", train_dataloader=dl, test_dataloader=test_dl,
                                    initial_num_universes=None, min_margin=1, max_margin=4, min_lr=0.001, max_lr=0.1,
                                    min_num_epochs=50, max_num_epochs=200, const_num_epochs=int(z["epochs"]),
                                    min_triple_constraint=int(z["min_tc"]), max_triple_constraint=int(z["max_tc"]),
                                    min_balance=0.25, max_balance=0.5, embedding_model=cls,
                                    embedding_model_param={"dim": int(z["dim"]), "p_norm": int(z["p_norm"]),
                                                           "norm_flag": 1},
                                    missing_embedding_handling=missing, checkpoint_dir=str(tmp_path) + "/",
                                    valid_steps=valid_steps, save_steps=None, training_setting="static",
                                    incremental_strategy=None)


def _universe_case(L, graph, kg, seed, tc, balance, tables, lr, margin, epochs, nbatches, bs=None):
    """One universe built natively and by the oracle from the same (seed, tc, balance), with its initial
    tables (numpy, or a callable (E, R) -> tables) and training hyperparameters."""
    import ctypes
    from openke import _native
    h = ctypes.c_void_p()
    _native.check(L.pt_universe_build(graph, seed, 8, tc, ctypes.c_float(balance), ctypes.byref(h)))
    rng = oracle.GlibcRand(seed)
    st = rng.rand_reset(8)
    ug, em, rm = kg.universe(rng, tc, balance)
    assert L.pt_universe_ent_total(h) == ug.ent_total and L.pt_universe_train_total(h) == ug.train_total
    seeds = np.zeros(8, dtype=np.uint64)
    _native.check(L.pt_universe_seeds(h, seeds.ctypes.data))
    assert (seeds == st).all()
    bs = bs if bs is not None else max(ug.train_total // nbatches, 1)
    if callable(tables):
        tables = tables(ug.ent_total, ug.rel_total)
    assert tables[0].shape[0] == ug.ent_total and tables[1].shape[0] == ug.rel_total
    return {"h": h, "ug": ug, "st": st, "tabs": [None if x is None else x.copy() for x in tables], "bs": bs,
            "lr": lr, "margin": margin, "epochs": epochs, "nbatches": nbatches, "em": em, "rm": rm}


def _teacher_forced_universes(L, cases, model, p, opt, neg, bern, filt, atol=2e-6):
    """The fast universe kernel (pt_universes_train) one step at a time, every universe of `cases` in one
    launch per step, each step starting from the ORACLE's state (tables, Adagrad state, LCG streams) of that
    step: the kernel's step must equal the oracle's step (loss rtol 1e-5, tables atol `atol` + the per-element
    forward-error bound of the step, helpers.kappa_bound / assert_step_close) except on the rows a near-tie
    decision touched and the components whose Adagrad update was noise-decided in either implementation
    (step_noise). Teacher
    forcing keeps one noise-decided +-lr step from spreading into the later steps' comparisons (the
    deterministic mode covers whole trajectories bit for bit: test_gpu_ordered.py)."""
    from openke import _native
    mid = 0 if model == "TransE" else 1
    ada = opt == "adagrad"
    state = []
    for c in cases:
        ent, rel, nv = (None if x is None else x.copy() for x in c["tabs"])
        accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) if ada \
            else (None, None, None)
        state.append({"tabs": [ent, rel, nv], "accs": list(accs), "st": c["st"].copy(),
                      "steps": c["epochs"] * c["nbatches"]})
    masked = 0
    for k in range(max(x["steps"] for x in state)):
        act = [i for i, x in enumerate(state) if k < x["steps"]]
        jobs, keep = [], []
        for i in act:
            c, x = cases[i], state[i]
            dev = [None if a is None else torch.from_numpy(a.copy()).cuda() for a in x["tabs"]]
            dacc = [None if a is None else torch.from_numpy(a.copy()).cuda() for a in x["accs"]]
            seeds = x["st"].copy()
            j = _native.UniverseJob()
            j.graph = L.pt_universe_graph(c["h"])
            j.seeds = seeds.ctypes.data
            j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, c["bs"], 1, 1, neg
            j.lr, j.margin = c["lr"], c["margin"]
            j.ent, j.rel, j.normv = (a.data_ptr() if a is not None else None for a in dev)
            j.ent_acc, j.rel_acc, j.norm_acc = (a.data_ptr() if a is not None else None for a in dacc)
            j.dim = x["tabs"][0].shape[1]
            jobs.append(j)
            keep.append((dev, dacc, seeds))
        arr = (_native.UniverseJob * len(jobs))(*jobs)
        losses = torch.zeros(len(jobs), device="cuda")
        _native.check(L.pt_universes_train(arr, len(jobs), mid, p, 1, _native.PT_ADAGRAD if ada else _native.PT_SGD,
                                           bern, filt, _native.ptr(losses), _native.stream()))
        lh = losses.cpu().numpy()
        for q, i in enumerate(act):
            c, x = cases[i], state[i]
            dev, dacc, _ = keep[q]
            acc0 = [None if a is None else a.copy() for a in x["accs"]]
            tab0 = [None if a is None else a.copy() for a in x["tabs"]]
            hh, tt, rr, _ = c["ug"].sample(x["st"], 8, c["bs"], neg, bern, filt)
            gm = oracle.grad_mass(model, p, True, c["margin"], x["tabs"][0], x["tabs"][1], x["tabs"][2], hh, tt, rr,
                                  c["bs"], neg)
            want = oracle.train_step(model, p, True, opt, c["lr"], c["margin"], x["tabs"][0], x["tabs"][1],
                                     x["tabs"][2], x["accs"] if ada else (None, None, None), hh, tt, rr, c["bs"], neg)
            assert abs(float(lh[q]) - want) <= 1e-5 * max(1.0, abs(want)), (i, k, float(lh[q]), want)
            got_acc = [None if a is None else a.cpu().numpy() for a in dacc]
            for name, g, w, a0, ga, w0 in zip(("ent", "rel", "norm"), dev, x["tabs"], acc0, got_acc, tab0):
                if g is None:
                    continue
                mask = step_noise(a0, x["accs"][("ent", "rel", "norm").index(name)], ga) if ada else None
                masked += 0 if mask is None else int(mask.sum())
                assert_step_close(g.cpu().numpy(), w, atol, mask, what="universe %d step %d %s" % (i, k, name),
                                  before=w0, gm=gm[name], lr=c["lr"], acc_before=a0)
    return masked


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_pu_training_matches_reference(path, tmp_path):
    """train_parallel_universes on the GPU (fast kernel): universes, hyperparameters and remaps equal to the
    reference's goldens; every universe trained (finite per-epoch losses, tables moved); and the fast kernel's
    every step along each golden universe's trajectory equal to the oracle's step from the same state
    (teacher-forced, _teacher_forced_universes). The whole trajectories, bit for bit, are the deterministic
    mode's (test_gpu_ordered.test_deterministic_pu_matches_oracle_and_reference)."""
    from openke import _native
    z = load(path)
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    n_univ = int(z["n_univ"])
    pu = _pu(z, tmp_path)
    assert pu.initial_random_seed == int(z["seed0"])
    pu.train_parallel_universes(n_univ)
    assert pu.next_universe_id == n_univ
    kg = oracle.KG.load(KG_SMALL)
    L = _native.lib()
    import ctypes
    graph = ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(graph)))
    cases = []
    try:
        for u in range(n_univ):
            hp = pu.universe_hparams[u]
            assert hp["tc"] == int(z["u%d_tc" % u])
            assert abs(hp["balance"] - float(z["u%d_balance" % u])) < 1e-9
            assert hp["margin"] == int(z["u%d_margin" % u])
            assert abs(hp["lr"] - float(z["u%d_lr" % u])) < 1e-12
            assert hp["train_total"] == int(z["u%d_train_total" % u])
            em, rm = pu._remaps(u)[:2]
            np.testing.assert_array_equal(em, z["u%d_ent_remap" % u])
            np.testing.assert_array_equal(rm, z["u%d_rel_remap" % u])
            assert np.isfinite(pu.last_universe_losses[u]).all() and len(pu.last_universe_losses[u]) == int(z["epochs"])
            init = torch_init_tables(model, len(em), len(rm), dim, int(z["seed0"]) + u)
            sp = pu.trained_embedding_spaces[u]
            assert not np.array_equal(sp.ent_embeddings.weight.detach().cpu().numpy(), init[0])
            cases.append(_universe_case(L, graph, kg, int(z["seed0"]) + u, int(z["u%d_tc" % u]),
                                        float(z["u%d_balance" % u]), init, float(z["u%d_lr" % u]),
                                        float(z["u%d_margin" % u]), int(z["epochs"]), 20))
        _teacher_forced_universes(L, cases, model, p, "adagrad", 1, 0, 0)
    finally:
        for c in cases:
            L.pt_universe_free(c["h"])
        L.pt_graph_free(graph)


def _inject_reference_universes(pu, z):
    from openke.module.model import TransE, TransH
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    cls = TransE if model == "TransE" else TransH
    universes = []
    for u in range(int(z["n_univ"])):
        em, rm = z["u%d_ent_remap" % u], z["u%d_rel_remap" % u]
        kge = cls(len(em), len(rm), dim=dim, p_norm=p, norm_flag=True)
        kge.ent_embeddings.weight.data.copy_(torch.from_numpy(z["u%d_ent" % u]))
        kge.rel_embeddings.weight.data.copy_(torch.from_numpy(z["u%d_rel" % u]))
        if model == "TransH":
            kge.norm_vector.weight.data.copy_(torch.from_numpy(z["u%d_norm" % u]))
        kge.cuda()
        pu.add_universe(kge, em, rm)
        universes.append({"ent_remap": em, "rel_remap": rm, "ent": z["u%d_ent" % u], "rel": z["u%d_rel" % u],
                          "norm": z["u%d_norm" % u] if model == "TransH" else None})
    return universes


def _assert_ranks_match(ours, ref_ranks, con_h, con_t, rel_tol=1e-6):
    """Per-query ranks equal, except where the truth's score is within float rounding of competing
    candidates' (the reference's own CPU order of summation decides such near-ties): there the rank
    may differ by at most the number of near-tied candidates."""
    mism = 0
    for k, (a, b) in enumerate(zip(ours, ref_ranks)):
        con = con_h if k < 2 else con_t
        for q in np.nonzero(a != b)[0]:
            s0 = con[q][0]
            ties = np.count_nonzero(np.abs(con[q][1:] - s0) <= rel_tol * max(1.0, abs(float(s0))))
            assert abs(int(a[q]) - int(b[q])) <= ties, (k, q, a[q], b[q], ties)
            mism += 1
    return mism


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_pu_link_prediction_matches_reference(path, tmp_path):
    """run_link_prediction over the reference's own trained universes == the reference's metrics
    (ranks equal query by query up to float near-ties, checked against the oracle's score vectors)."""
    z = load(path)
    pu = _pu(z, tmp_path)
    universes = _inject_reference_universes(pu, z)
    mrr, mr, hit10, hit3, hit1 = pu.run_link_prediction()
    met, ranks, (con_h, con_t) = _oracle_metrics(z, universes, "test2id.txt", with_con=True)
    # the oracle ranking restated from the reference reproduces the reference's metrics (test_oracle)
    np.testing.assert_allclose(met, z["lp"].astype(np.float32), rtol=1e-6, atol=1e-7)
    mism = _assert_ranks_match(pu.last_ranks, ranks, con_h, con_t)
    # the metrics are those of our ranks; with no near-tie rank difference, the reference's own numbers
    metrics_match_ranks([mrr, mr, hit10, hit3, hit1], pu.last_ranks)
    if mism == 0:
        np.testing.assert_allclose(np.array([mrr, mr, hit10, hit3, hit1], dtype=np.float32),
                                   z["lp"].astype(np.float32), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("path", golden("universes_*.npz")[:1], ids=lambda p: p.split("/")[-1])
def test_pu_checkpoint_round_trip_on_gpu(path, tmp_path):
    """save_model -> load_parameters (map_location cpu, then onto the GPU) keeps every universe and id map:
    link prediction of the reloaded model equals the original's, rank for rank."""
    z = load(path)
    pu = _pu(z, tmp_path)
    _inject_reference_universes(pu, z)
    want = pu.run_link_prediction()
    want_ranks = [np.array(r).copy() for r in pu.last_ranks]
    pu.save_model("rt.ckpt")
    re = _pu(z, tmp_path)
    re.load_parameters("rt.ckpt")
    assert re.next_universe_id == pu.next_universe_id
    assert all(next(sp.parameters()).is_cuda for sp in re.trained_embedding_spaces.values())
    got = re.run_link_prediction()
    assert list(got) == list(want)
    for a, b in zip(re.last_ranks, want_ranks):
        np.testing.assert_array_equal(np.array(a), b)


def _oracle_metrics(z, universes, split, missing="last_rank", with_con=False):
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    ev = oracle.sort_test(*oracle.read_triples(KG_SMALL + split))
    con_h, con_t = pu_energy(kg.ent_total, universes, ev, model, p, dim)
    if missing == "null_vector":
        _null_vector_fill(con_h, con_t, universes, ev, p, kg.ent_total)
    met, ranks = oracle.link_prediction(kg.ent_total, all_tr, ev, con_h, con_t)
    if with_con:
        return met, ranks, (con_h, con_t)
    return met, ranks


def _null_vector_fill(con_h, con_t, universes, ev, p, E):
    """global_energy_estimation's null_vector replacement (:590-599): +inf candidates get the key's
    minimum over universes of calc_tuple_score (raw anchor, TransE-style _calc against a zero vector)."""
    th, tt, tr = ev
    for q in range(len(th)):
        for side, con in ((0, con_h), (1, con_t)):
            anchor = int(tt[q]) if side == 0 else int(th[q])
            best = np.inf
            for u in universes:
                em, rm = list(u["ent_remap"]), list(u["rel_remap"])
                if anchor not in em or int(tr[q]) not in rm:
                    continue
                la, lr = em.index(anchor), rm.index(int(tr[q]))
                ent = np.vstack([u["ent"], np.zeros((1, u["ent"].shape[1]), dtype=np.float32)])
                zero = ent.shape[0] - 1
                if side == 1:   # tail_batch: _calc(ent, 0, r)
                    s = oracle.score("TransE", p, True, "normal", ent, u["rel"], None, np.array([la]),
                                     np.array([zero]), np.array([lr]))
                else:           # head_batch: _calc(0, ent, r) = 0 + (r - ent)
                    s = oracle.score("TransE", p, True, "normal", ent, u["rel"], None, np.array([zero]),
                                     np.array([la]), np.array([lr]))
                best = min(best, float(s[0]))
            if best != np.inf:
                row = con[q]
                row[row == np.inf] = best


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_pu_valid_hit10_matches_oracle(path, tmp_path):
    """eval_universes('valid') + valid() == validHead/validTail/getValidHit10 on the oracle's vectors."""
    z = load(path)
    pu = _pu(z, tmp_path)
    universes = _inject_reference_universes(pu, z)
    pu.eval_universes(eval_mode='valid')
    hit10 = pu.valid()
    met, _ = _oracle_metrics(z, universes, "valid2id.txt")
    assert abs(hit10 - float(met[2])) < 1e-6, (hit10, met[2])


@pytest.mark.parametrize("path", golden("universes_u*.npz")[:2], ids=lambda p: p.split("/")[-1])
def test_pu_null_vector_ranks_match_oracle(path, tmp_path):
    """missing_embedding_handling='null_vector': per-query raw and filtered ranks == oracle."""
    z = load(path)
    pu = _pu(z, tmp_path, missing="null_vector")
    universes = _inject_reference_universes(pu, z)
    pu.run_link_prediction()
    met, ranks, (con_h, con_t) = _oracle_metrics(z, universes, "test2id.txt", missing="null_vector", with_con=True)
    _assert_ranks_match(pu.last_ranks, ranks, con_h, con_t)


UNIVERSE_DIMS = [8, 20, 50, 100, 20, 64, 69, 23, 44, 85]   # every row-shape class, odd (scalar-chunk) and non-power-of-two chunk counts included


@pytest.mark.parametrize("model,p,neg,bern,filt,opt", [
    ("TransE", 1, 1, 0, 0, "adagrad"),
    ("TransE", 2, 3, 1, 1, "adagrad"),
    ("TransH", 1, 1, 0, 0, "adagrad"),
    ("TransH", 2, 2, 1, 1, "sgd"),
    ("TransE", 1, 1, 1, 0, "sgd"),
])
def test_universe_kernel_matches_oracle(model, p, neg, bern, filt, opt):
    """The fast persistent universe kernel (mixed dims: several shape classes / launches at once):
    (a) teacher-forced, every step of every universe equal to the oracle's step from the same state;
    (b) one uninterrupted run of all epochs: the LCG streams end exactly where `epochs x nbatches`
        sampling() calls leave them (pt_universe_set_states), and under SGD (no noise amplification) the
        tables equal the oracle's whole trajectory within 5e-5."""
    import ctypes
    from openke import _native
    L = _native.lib()
    kg = oracle.KG.load(KG_SMALL)
    graph = ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(graph)))
    rs = np.random.default_rng(7 + neg + bern)
    cases = []
    try:
        for i, dim in enumerate(UNIVERSE_DIMS):
            tc, bal = int(rs.integers(150, 600)), float(rs.uniform(0.25, 0.5))

            def tabs(E, R, dim=dim):
                bound = np.sqrt(6.0 / (E + dim))
                return [rs.uniform(-bound, bound, (E, dim)).astype(np.float32),
                        rs.uniform(-bound, bound, (R, dim)).astype(np.float32),
                        rs.uniform(-bound, bound, (R, dim)).astype(np.float32) if model == "TransH" else None]
            cases.append(_universe_case(L, graph, kg, 1000 + i, tc, bal, tabs, 0.05 if opt == "adagrad" else 0.3,
                                        2.0, 2, 10))
        _teacher_forced_universes(L, cases, model, p, opt, neg, bern, filt)
        # (b) uninterrupted run through a set
        mid = 0 if model == "TransE" else 1
        jobs, keep = [], []
        for c in cases:
            dev = [None if a is None else torch.from_numpy(a.copy()).cuda() for a in c["tabs"]]
            dacc = [None if a is None else torch.zeros_like(a) for a in dev]
            seeds = c["st"].copy()
            j = _native.UniverseJob()
            j.graph = L.pt_universe_graph(c["h"])
            j.seeds = seeds.ctypes.data
            j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, c["bs"], c["epochs"], c["nbatches"], neg
            j.lr, j.margin = c["lr"], c["margin"]
            j.ent, j.rel, j.normv = (a.data_ptr() if a is not None else None for a in dev)
            j.ent_acc, j.rel_acc, j.norm_acc = (a.data_ptr() if a is not None else None for a in dacc)
            j.dim = c["tabs"][0].shape[1]
            jobs.append(j)
            keep.append((dev, dacc, seeds))
        arr = (_native.UniverseJob * len(jobs))(*jobs)
        uset = ctypes.c_void_p()
        _native.check(L.pt_universe_set_create(arr, len(jobs), mid, p, 1,
                                               _native.PT_ADAGRAD if opt == "adagrad" else _native.PT_SGD, bern, filt,
                                               ctypes.byref(uset)))
        try:
            losses = torch.zeros(sum(c["epochs"] for c in cases), device="cuda")
            _native.check(L.pt_universe_set_train(uset, _native.ptr(losses), _native.stream()))
            torch.cuda.synchronize()
            for i, c in enumerate(cases):
                st = c["st"].copy()
                ent, rel, nv = (None if x is None else x.copy() for x in c["tabs"])
                accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) \
                    if opt == "adagrad" else (None, None, None)
                for _ in range(c["epochs"] * c["nbatches"]):
                    hh, tt, rr, _ = c["ug"].sample(st, 8, c["bs"], neg, bern, filt)
                    oracle.train_step(model, p, True, opt, c["lr"], c["margin"], ent, rel, nv, accs, hh, tt, rr,
                                      c["bs"], neg)
                got = np.zeros(8, dtype=np.uint64)
                _native.check(L.pt_universe_set_states(uset, i, got.ctypes.data))
                np.testing.assert_array_equal(got, st)
                if opt == "sgd":
                    for g, w in zip(keep[i][0], (ent, rel, nv)):
                        if w is not None:
                            np.testing.assert_allclose(g.cpu().numpy(), w, rtol=0, atol=5e-5)
        finally:
            L.pt_universe_set_free(uset)
    finally:
        for c in cases:
            L.pt_universe_free(c["h"])
        L.pt_graph_free(graph)


def test_universe_job_validation_errors():
    from openke import _native
    L = _native.lib()
    j = _native.UniverseJob()
    arr = (_native.UniverseJob * 1)(j)
    with pytest.raises(_native.NativeError):
        _native.check(L.pt_universes_train(arr, 1, 0, 1, 1, _native.PT_ADAGRAD, 0, 0, None, _native.stream()))
    assert b"null" in L.pt_last_error()


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_pu_triple_classification_matches_reference(path, tmp_path):
    """run_triple_classification over the reference's trained universes from a fixed C RNG state (the
    negatives come from sampler thread 0): accuracy and threshold == the reference's. The reference
    scores 'normal' triples as (h, relation = batch_t, tail = batch_r) (its test_one_step unpacking,
    Parallel_Universe_Config.py:718), which the drop-in keeps."""
    z = load(path)
    pu = _pu(z, tmp_path)
    _inject_reference_universes(pu, z)
    pu.set_random_seed(4321)
    acc, thr = pu.run_triple_classification()
    assert acc == float(z["tc_acc"]), (acc, float(z["tc_acc"]))
    want = float(z["tc_threshold"])
    if np.isinf(want) or np.isnan(want):
        assert (thr is None and np.isnan(want)) or float(thr) == want, (thr, want)
    else:
        np.testing.assert_allclose(float(thr), want, rtol=1e-5)


@pytest.mark.parametrize("path", golden("universes_u*.npz")[:2], ids=lambda p: p.split("/")[-1])
def test_pu_triple_classification_from_files_matches_reference(path, tmp_path):
    """run_triple_classification_from_files (:802-815): the same positives and negatives written as a
    snapshot's labelled file give the reference's accuracy and threshold (those of the golden run);
    the deleted-triple files are classified at that threshold."""
    import os
    z = load(path)
    pu = _pu(z, tmp_path)
    _inject_reference_universes(pu, z)
    pu.set_random_seed(4321)
    pu.data_loader.set_sampling_mode('classification')
    pos, neg = next(iter(pu.data_loader))
    snap = tmp_path / "incremental" / "0"
    os.makedirs(str(snap))
    with open(str(snap / "triple_classification_prepared_test_examples.txt"), "w") as f:
        for d, truth in ((pos, 1), (neg, 0)):
            for h, t, r in zip(d["batch_h"], d["batch_t"], d["batch_r"]):
                f.write("%d %d %d %d\n" % (h, t, r, truth))
    with open(str(snap / "tc_deleted.txt"), "w") as f:
        for h, t, r in zip(neg["batch_h"][:10], neg["batch_t"][:10], neg["batch_r"][:10]):
            f.write("%d %d %d 0\n" % (h, t, r))
    pu.data_loader.in_path = str(tmp_path) + "/"
    acc, thr = pu.run_triple_classification_from_files(0)
    assert acc == float(z["tc_acc"]), (acc, float(z["tc_acc"]))
    want = float(z["tc_threshold"])
    if np.isinf(want) or np.isnan(want):
        assert (thr is None and np.isnan(want)) or float(thr) == want, (thr, want)
    else:
        np.testing.assert_allclose(float(thr), want, rtol=1e-5)


@pytest.mark.parametrize("path", golden("universes_u*.npz")[:2], ids=lambda p: p.split("/")[-1])
def test_pu_type_constrained_ranks_match_oracle(path, tmp_path):
    """run_link_prediction(type_constrain=True): constrained ranks on the GPU (k_rank_types) == the
    oracle's literal restatement of testHead/testTail's constrained branch (Test.h:127-502, pinned to the
    reference by test_oracle's lpt goldens) on the same universes; the unconstrained ranks unchanged."""
    z = load(path)
    pu = _pu(z, tmp_path)
    universes = _inject_reference_universes(pu, z)
    res = pu.run_link_prediction(type_constrain=True)
    met, ranks, (con_h, con_t) = _oracle_metrics(z, universes, "test2id.txt", with_con=True)
    mism = _assert_ranks_match(pu.last_ranks, ranks, con_h, con_t)
    kg = oracle.KG.load(KG_SMALL)
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]
    ev = oracle.sort_test(*oracle.read_triples(KG_SMALL + "test2id.txt"))
    types = oracle.read_types(KG_SMALL + "type_constrain.txt", kg.rel_total)
    met_tc, ranks_tc = oracle.rank_constrained(kg.ent_total, all_tr, ev, con_h, con_t, types)
    mism += _assert_ranks_match(pu.last_tc_ranks, ranks_tc, con_h, con_t)
    metrics_match_ranks(res, pu.last_tc_ranks)
    if mism == 0:
        np.testing.assert_allclose(np.array(res, dtype=np.float32), met_tc, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("path", golden("universes_u*.npz")[:2], ids=lambda p: p.split("/")[-1])
def test_pu_one_universe_protocol_matches_reference(path, tmp_path):
    """The reference's per-universe protocol driven by hand (Parallel_Universe_Config.py:320-327):
    set_random_seed -> compile_train_datset (getParallelUniverse + process_universe_mappings) ->
    train_embedding_space (Adagrad Trainer on the swapped-in universe, fast fused trainer) ->
    add_embedding_space. Maps and hyperparameters equal the reference's goldens and the universes feed link
    prediction. The tables of this protocol are checked bit for bit in deterministic mode
    (test_gpu_ordered), and the fast trainer's steps teacher-forced in test_gpu_parity."""
    z = load(path)
    dim = int(z["dim"])
    n_univ = int(z["n_univ"])
    pu = _pu(z, tmp_path)
    for _ in range(n_univ):
        pu.set_random_seed(pu.initial_random_seed + pu.next_universe_id)
        pu.compile_train_datset()
        sp = pu.train_embedding_space()
        pu.add_embedding_space(sp)
        pu.next_universe_id += 1
    for u in range(n_univ):
        hp = pu.universe_hparams[u]
        assert hp["margin"] == int(z["u%d_margin" % u])
        assert abs(hp["lr"] - float(z["u%d_lr" % u])) < 1e-12
        assert hp["train_total"] == int(z["u%d_train_total" % u])
        em, rm = pu._remaps(u)[:2]
        np.testing.assert_array_equal(em, z["u%d_ent_remap" % u])
        np.testing.assert_array_equal(rm, z["u%d_rel_remap" % u])
        sp = pu.trained_embedding_spaces[u]
        w = sp.ent_embeddings.weight.detach().cpu().numpy()
        assert w.shape == (len(em), dim) and np.isfinite(w).all()
        init = torch_init_tables(str(z["model"]), len(em), len(rm), dim, int(z["seed0"]) + u)[0]
        assert not np.array_equal(w, init)
    # the universes feed link prediction like train_parallel_universes' do
    mrr, mr, hit10, hit3, hit1 = pu.run_link_prediction()
    metrics_match_ranks([mrr, mr, hit10, hit3, hit1], pu.last_ranks)


@pytest.mark.parametrize("missing", ["last_rank", "null_vector"])
def test_pu_per_key_internals_match_device_rows(missing, tmp_path):
    """The reference's per-(key, universe) steps (obtain_embedding_space_score -> transmit_max_scores /
    transmit_tuple_max_score, :446-540, driven as eval_universes drives them, :556-603) and
    global_energy_estimation2 (:644-701) give the candidate vectors the batched device path gives
    (eval_universes -> k_lp_scan key rows -> global_energy_estimation)."""
    z = load(golden("universes_u1.npz")[0])
    dev_pu = _pu(z, tmp_path, missing=missing)
    _inject_reference_universes(dev_pu, z)
    dev_pu.data_loader.set_sampling_mode('link')
    dev_pu.eval_universes(eval_mode='test')
    man_pu = _pu(z, tmp_path, missing=missing)
    _inject_reference_universes(man_pu, z)
    man_pu.data_loader.set_sampling_mode('link')
    datas = []
    for index, (data_head, data_tail) in enumerate(man_pu.data_loader):
        if index >= 25:
            break
        # the loader hands out views of buffers its next call overwrites (TestDataLoader.sampling_lp)
        data_head, data_tail = ({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in d.items()}
                                for d in (data_head, data_tail))
        datas.append((data_head, data_tail))
        head, rel, tail = int(data_tail['batch_h'][0]), int(data_head['batch_r'][0]), int(data_head['batch_t'][0])
        for u in range(man_pu.next_universe_id):
            if u in man_pu.entity_universes[head] and u in man_pu.relation_universes[rel]:
                man_pu.obtain_embedding_space_score(data_tail, u)
            if u in man_pu.entity_universes[tail] and u in man_pu.relation_universes[rel]:
                man_pu.obtain_embedding_space_score(data_head, u)
    assert man_pu.evaluation_head2tail_triple_score_dict and man_pu.evaluation_tail2head_triple_score_dict
    for data_head, data_tail in datas:
        for d in (data_head, data_tail):
            want = dev_pu.global_energy_estimation(d)
            np.testing.assert_allclose(man_pu.global_energy_estimation(d), want, rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(man_pu.global_energy_estimation2(d), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("smode,neg_rel", [("cross", 0), ("normal", 1), ("cross", 1)])
def test_pu_cross_sampling_and_relation_corruption_match_oracle(smode, neg_rel, tmp_path):
    """train_parallel_universes with a cross-sampling or relation-corrupting loader: the reference trains
    each universe's Trainer over TrainDataLoader.__iter__ (cross_sampling alternates tail/head batches with
    one flag the loader keeps across universes; neg_rel appends corrupt_rel slots, which a head_batch /
    tail_batch view turns into copies of the positive, TransE.py:51-58). Universe by universe here (GPU
    sampler + fused trainer), in deterministic mode: tables equal to the oracle's restatement
    (sampling_ex + the fixed side broadcast + Adagrad steps) bit for bit."""
    from openke.config import Parallel_Universe_Config
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.model import TransE
    z = load(golden("universes_u1.npz")[0])
    dl = TrainDataLoader(in_path=KG_SMALL, nbatches=20, threads=8, sampling_mode=smode, bern_flag=0, filter_flag=1,
                         neg_ent=1, neg_rel=neg_rel, random_seed=int(z["seed"]))
    test_dl = TestDataLoader(dl.in_path, "link")
    dim, p, n_univ, epochs = 8, 1, 3, 2
    pu = Parallel_Universe_Config(training_identifier="x", train_dataloader=dl, test_dataloader=test_dl,
                                  initial_num_universes=None, min_margin=1, max_margin=4, min_lr=0.001, max_lr=0.1,
                                  min_num_epochs=50, max_num_epochs=200, const_num_epochs=epochs,
                                  min_triple_constraint=200, max_triple_constraint=400, min_balance=0.25,
                                  max_balance=0.5, embedding_model=TransE,
                                  embedding_model_param={"dim": dim, "p_norm": p, "norm_flag": 1},
                                  checkpoint_dir=str(tmp_path) + "/", valid_steps=10 ** 6, save_steps=None,
                                  training_setting="static", incremental_strategy=None, deterministic=True)
    pu.train_parallel_universes(n_univ)
    assert pu.next_universe_id == n_univ
    kg = oracle.KG.load(KG_SMALL)
    seed0 = pu.initial_random_seed
    flag = 0
    for u in range(n_univ):
        hp = pu.universe_hparams[u]
        rng = oracle.GlibcRand(seed0 + u)
        st = rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, int(hp["tc"]), float(hp["balance"]))
        np.testing.assert_array_equal(pu._remaps(u)[0], em)
        bs = ug.train_total // 20
        ent, rel, nv = torch_init_tables("TransE", ug.ent_total, ug.rel_total, dim, seed0 + u)
        accs = (np.zeros_like(ent), np.zeros_like(rel), None)
        for _ in range(epochs * 20):
            if smode == "cross":
                flag = 1 - flag
                mode = -1 if flag == 0 else 1
            else:
                mode = 0
            h, t, r, _ = ug.sample_ex(st, 8, bs, 1, neg_rel, mode, 0, 1)
            if mode != 0:   # the head_batch / tail_batch view broadcasts the fixed side and the relation
                fixed = t if mode == -1 else h
                fixed.reshape(-1, bs)[1:] = fixed[:bs]
                r.reshape(-1, bs)[1:] = r[:bs]
            oracle.train_step("TransE", p, True, "adagrad", float(hp["lr"]), float(hp["margin"]), ent, rel, None, accs,
                              h, t, r, bs, 1 + neg_rel)
        sp = pu.trained_embedding_spaces[u]
        np.testing.assert_array_equal(sp.ent_embeddings.weight.detach().cpu().numpy(), ent)
        np.testing.assert_array_equal(sp.rel_embeddings.weight.detach().cpu().numpy(), rel)


def test_multi_rank_pu_flow_matches_single_process(tmp_path):
    """the real sharded flow end to end - two gloo ranks sharing cuda:0 (fresh processes, so
    no GPU-initialised process is re-executed) run Parallel_Universe_Config(deterministic=True) through
    train_parallel_universes (two LPT-placed waves, validation every 4 universes, checkpoints), save_model,
    load_parameters and run_link_prediction (Parallel_Universe_Config.py:316-367, 446-465, 852-935). The
    validation schedule, best_hit10 / bad_counts, the checkpoint's tables and maps, and the ranks and metrics
    equal the one-process run bit for bit."""
    import socket
    import subprocess
    import sys

    def port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return str(p)
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_pu_worker.py")
    out = str(tmp_path)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, worker, "0", "1", port(), out], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    p = port()
    procs = [subprocess.Popen([sys.executable, worker, str(k), "2", p, out], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, env=env) for k in range(2)]
    logs = [pr.communicate(timeout=240)[0] for pr in procs]
    for pr, lg in zip(procs, logs):
        assert pr.returncode == 0, lg[-3000:]
    import json
    one = json.load(open(os.path.join(out, "result_w1.json")))
    two = json.load(open(os.path.join(out, "result_w2.json")))
    assert two["ranks_per_universe"] == [0, 1]   # both ranks trained universes
    for k in ("schedule", "best_hit10", "bad_counts", "next_universe_id", "metrics", "ranks"):
        assert one[k] == two[k], k
    assert len(one["schedule"]) == 3
    a = torch.load(os.path.join(out, "ckpt_w1", "final.ckpt"), weights_only=False)
    b = torch.load(os.path.join(out, "ckpt_w2", "final.ckpt"), weights_only=False)
    assert sorted(a["trained_embedding_spaces"]) == sorted(b["trained_embedding_spaces"]) == list(range(12))
    for u in a["trained_embedding_spaces"]:
        sa = a["trained_embedding_spaces"][u].state_dict()
        sb = b["trained_embedding_spaces"][u].state_dict()
        for k in sa:
            assert torch.equal(sa[k].cpu(), sb[k].cpu()), (u, k)
    for k in ("entity_id_mappings", "relation_id_mappings", "entity_universes", "relation_universes"):
        assert {u: v for u, v in a[k].items() if v} == {u: v for u, v in b[k].items() if v}, k
    for k in ("next_universe_id", "best_hit10", "bad_counts"):
        assert a[k] == b[k], k


def _sgd_set_runs(L, cases, modes):
    """Trains `cases` (from _universe_case, TransE, SGD, p = 2) as one universe set per mode; a mode is
    (configure(), check(set handle)). Returns per mode (tables, per-epoch losses, final LCG states)."""
    import ctypes
    from openke import _native
    runs = []
    for configure, check in modes:
        configure()
        jobs, keep = [], []
        for c in cases:
            dev = [None if a is None else torch.from_numpy(a.copy()).cuda() for a in c["tabs"]]
            seeds = c["st"].copy()
            j = _native.UniverseJob()
            j.graph = L.pt_universe_graph(c["h"])
            j.seeds = seeds.ctypes.data
            j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, c["bs"], c["epochs"], c["nbatches"], 1
            j.lr, j.margin = c["lr"], c["margin"]
            j.ent, j.rel, j.normv = dev[0].data_ptr(), dev[1].data_ptr(), None
            j.dim = c["tabs"][0].shape[1]
            jobs.append(j)
            keep.append((dev, seeds))
        arr = (_native.UniverseJob * len(jobs))(*jobs)
        uset = ctypes.c_void_p()
        _native.check(L.pt_universe_set_create(arr, len(jobs), 0, 2, 1, _native.PT_SGD, 0, 0, ctypes.byref(uset)))
        try:
            check(uset)
            losses = torch.zeros(sum(c["epochs"] for c in cases), device="cuda")
            _native.check(L.pt_universe_set_train(uset, _native.ptr(losses), _native.stream()))
            torch.cuda.synchronize()
            states = []
            for i in range(len(cases)):
                got = np.zeros(8, dtype=np.uint64)
                _native.check(L.pt_universe_set_states(uset, i, got.ctypes.data))
                states.append(got)
        finally:
            L.pt_universe_set_free(uset)
        runs.append(([[t.cpu().numpy() for t in k[0][:2]] for k in keep], losses.cpu().numpy(), states))
    return runs


def _check_sgd_runs(cases, runs):
    """Two runs of _sgd_set_runs against each other and the oracle's trajectory: tables within 5e-5, losses within
    1e-5, the sampler streams ending where the oracle's do."""
    (tab_t, loss_t, st_t), (tab_1, loss_1, st_1) = runs
    np.testing.assert_allclose(loss_t, loss_1, rtol=1e-5, atol=1e-6)
    for i, c in enumerate(cases):
        st = c["st"].copy()
        ent, rel = c["tabs"][0].copy(), c["tabs"][1].copy()
        for _ in range(c["epochs"] * c["nbatches"]):
            hh, tt, rr, _ = c["ug"].sample(st, 8, c["bs"], 1, 0, 0)
            oracle.train_step("TransE", 2, True, "sgd", c["lr"], c["margin"], ent, rel, None, (None, None, None),
                              hh, tt, rr, c["bs"], 1)
        np.testing.assert_array_equal(st_t[i], st)
        np.testing.assert_array_equal(st_1[i], st)
        for g_t, g_1, want in zip(tab_t[i], tab_1[i], (ent, rel)):
            np.testing.assert_allclose(g_t, g_1, rtol=0, atol=5e-5)
            np.testing.assert_allclose(g_t, want, rtol=0, atol=5e-5)


def _small_set_cases(L, graph, kg, seed):
    rs = np.random.default_rng(seed)
    cases = []
    for i, dim in enumerate([200, 69, 20, 200, 12, 69]):
        tc, bal = int(rs.integers(300, 900)), float(rs.uniform(0.25, 0.5))

        def tabs(E, R, dim=dim):
            bound = np.sqrt(6.0 / (E + dim))
            return [rs.uniform(-bound, bound, (E, dim)).astype(np.float32),
                    rs.uniform(-bound, bound, (R, dim)).astype(np.float32), None]
        cases.append(_universe_case(L, graph, kg, 2000 + i, tc, bal, tabs, 0.3, 2.0, 3, 10))
    return cases


@pytest.mark.parametrize("width", [2, 4])
def test_universe_teams_equal_one_workgroup_and_oracle(width):
    """Team universes (universes_team.h; off by default since round 6 - measured slower than one workgroup): a set of
    fewer universes than CUs trains its longest TransE universes with teams of `width` workgroups
    (pt_universe_set_teams > 0). Under SGD with p = 2 (no noise amplification, no sign decisions), over whole runs of
    3 epochs x 10 steps: the team-trained tables equal the one-workgroup tables and the oracle's trajectory within
    5e-5, the sampler streams end where the oracle's do, the per-epoch losses agree within 1e-5; and under Adagrad
    each team step equals the oracle's step from the same state (teacher forcing, test_universe_kernel_matches_oracle's
    bound)."""
    import ctypes
    from openke import _native
    L = _native.lib()
    kg = oracle.KG.load(KG_SMALL)
    graph = ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(graph)))
    default_w = L.pt_get_universe_team_width()
    cases = _small_set_cases(L, graph, kg, 31 + width)
    try:
        def teams(w):
            def check(uset):
                nt, nw = ctypes.c_int64(), ctypes.c_int64()
                _native.check(L.pt_universe_set_teams(uset, ctypes.byref(nt), ctypes.byref(nw)))
                if w > 1:
                    assert nt.value > 0 and nw.value >= 2 * nt.value, (nt.value, nw.value)
                else:
                    assert nt.value == 0
            return (lambda: _native.check(L.pt_set_universe_team_width(w))), check
        _check_sgd_runs(cases, _sgd_set_runs(L, cases, [teams(width), teams(1)]))
        # Adagrad, teacher-forced step by step with teams of `width`
        _native.check(L.pt_set_universe_team_width(width))
        for c in cases:
            c["lr"], c["epochs"], c["nbatches"] = 0.05, 1, 6
        _teacher_forced_universes(L, cases, "TransE", 1, "adagrad", 1, 0, 0)
    finally:
        _native.check(L.pt_set_universe_team_width(default_w))
        for c in cases:
            L.pt_universe_free(c["h"])
        L.pt_graph_free(graph)
