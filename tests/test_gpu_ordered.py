"""Reference-order (deterministic) mode on the GPU: bit-identical to the CPU oracle.

The oracle (oracle/oracle.c) restates one training step in the order torch's autograd sums it
(embedding_dense_backward per lookup in slot order, the two entity lookups added, Trainer.py:44-56) with
sequential dot products and IEEE arithmetic. The deterministic mode of the HIP path (ordered.hip, set with
Trainer(deterministic=True), Parallel_Universe_Config(deterministic=True), pt_trainer_set_deterministic,
pt_universes_train_ex(PT_DETERMINISTIC)) performs the same operations in the same order, so tables,
Adagrad state and every step's loss must be EQUAL to the oracle's, over whole Adagrad trajectories - no
tolerance, no noise mask. The oracle itself is pinned to the reference's goldens in test_oracle.py (where
Adagrad's amplification of rounding noise is handled with the IllConditioned masks), so this mode
separates "rounding noise" from "bug" for the fast kernels (their step-level parity: test_gpu_pu.py,
test_gpu_parity.py). pytest -m gpu."""
import numpy as np
import pytest
import torch

import oracle
from conftest import KG_SMALL
from helpers import IllConditioned, assert_tables_close, golden, load, torch_init_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _tables(kge):
    out = [kge.ent_embeddings.weight.detach().cpu().numpy(), kge.rel_embeddings.weight.detach().cpu().numpy()]
    out.append(kge.norm_vector.weight.detach().cpu().numpy() if hasattr(kge, "norm_vector") else None)
    return out


def _equal(got, want, what):
    for name, g, w in zip(("ent", "rel", "norm"), got, want):
        if w is None:
            continue
        g = np.asarray(g)
        bad = g != w
        assert not bad.any(), "%s %s: %d entries differ (max %g)" % (what, name, int(bad.sum()),
                                                                      float(np.abs(g - w).max()))


RUN_CASES = [
    # model, dim, p, norm_flag, opt, bs, neg, bern, filter, steps
    ("TransE", 20, 1, True, "adagrad", 50, 1, 0, 0, 40),      # C3's universe step shape
    ("TransE", 69, 1, True, "adagrad", 64, 3, 1, 1, 30),
    ("TransE", 23, 2, True, "sgd", 40, 2, 0, 1, 30),
    ("TransE", 50, 1, True, "sgd", 100, 1, 0, 0, 20),        # C1 (WN18 config: dim 50, batch 100, 1 neg)
    ("TransE", 200, 2, True, "sgd", 80, 25, 1, 1, 5),        # C2's step shape
    ("TransE", 32, 2, False, "adagrad", 60, 4, 1, 0, 20),
    ("TransH", 23, 1, True, "adagrad", 48, 1, 0, 0, 30),
    ("TransH", 69, 2, False, "adagrad", 32, 2, 1, 1, 20),
    ("TransH", 20, 2, True, "sgd", 70, 3, 1, 1, 20),
]


@pytest.mark.parametrize("case", RUN_CASES, ids=lambda c: "%s-d%d-p%d-nf%d-%s-bs%d-neg%d" % (c[0], c[1], c[2], c[3],
                                                                                          c[4], c[5], c[6]))
def test_deterministic_trainer_run_bit_exact(case):
    """Trainer(deterministic=True).run(): GPU-sampled batches + reference-order steps == the oracle's
    sampling + steps, bit for bit (tables, Adagrad state, every step's loss), and the same twice."""
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    model, dim, p, nf, opt, bs, neg, bern, filt, steps = case
    lr, margin, seed = (0.5 if opt == "sgd" else 0.05), 3.0, 17
    runs = []
    for _ in range(2):
        dl = TrainDataLoader(in_path=KG_SMALL, batch_size=bs, threads=8, sampling_mode="normal", bern_flag=bern,
                             filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)
        dl.nbatches = steps
        torch.manual_seed(dim + neg)
        cls = TransE if model == "TransE" else TransH
        kge = cls(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=nf)
        t0 = [None if x is None else x.copy() for x in _tables(kge)]
        ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
        tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt,
                     deterministic=True)
        tr.run()
        accs = [None if a is None else a.cpu().numpy() for a in tr.optimizer.state_sum]
        runs.append((_tables(kge), accs, tr.last_step_losses.copy()))
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(seed).rand_reset(8)
    ent, rel, nv = t0
    oaccs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) \
        if opt == "adagrad" else (None, None, None)
    losses = []
    for _ in range(steps):
        h, t, r, _ = kg.sample(st, 8, bs, neg, bern, filt)
        losses.append(oracle.train_step(model, p, nf, opt, lr, margin, ent, rel, nv, oaccs, h, t, r, bs, neg))
    for tabs, accs, step_losses in runs:
        np.testing.assert_array_equal(step_losses, np.array(losses, dtype=np.float32))
        _equal(tabs, (ent, rel, nv), "tables")
        if opt == "adagrad":
            _equal(accs, oaccs, "state_sum")


@pytest.mark.parametrize("path", golden("train_*.npz"), ids=lambda p: p.split("/")[-1])
def test_deterministic_train_one_step_on_reference_batches(path):
    """Trainer(deterministic=True).train_one_step on the reference's own golden batches: equal to the
    oracle at every step; against the reference's tables within the oracle's own tolerance (test_oracle)."""
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    z = load(path)
    model, dim, p, nf = str(z["model"]), int(z["dim"]), int(z["p_norm"]), bool(z["norm_flag"])
    bs, neg, opt = int(z["batch_size"]), int(z["neg_ent"]), str(z["opt"])
    dl = TrainDataLoader(in_path=KG_SMALL, batch_size=bs, threads=int(z["threads"]), sampling_mode="normal",
                         bern_flag=int(z["bern"]), filter_flag=int(z["filter"]), neg_ent=neg, neg_rel=0,
                         random_seed=int(z["seed"]))
    torch.manual_seed(int(z["torch_seed"]))
    cls = TransE if model == "TransE" else TransH
    kge = cls(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=nf)
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=float(z["margin"])), batch_size=bs)
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=float(z["lr"]), use_gpu=True, opt_method=opt,
                 deterministic=True)
    tr.run()
    ent, rel = z["init_ent_embeddings"].copy(), z["init_rel_embeddings"].copy()
    nv = z["init_norm_vector"].copy() if model == "TransH" else None
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) \
        if opt == "adagrad" else (None, None, None)
    ill = IllConditioned()
    for s in range(int(z["steps"])):
        d = {"batch_h": z["batch_h"][s], "batch_t": z["batch_t"][s], "batch_r": z["batch_r"][s], "mode": "normal"}
        loss = tr.train_one_step(d)
        for k, a in zip(("ent", "rel", "norm"), accs):
            ill.before(k, a)
        want = oracle.train_step(model, p, nf, opt, float(z["lr"]), float(z["margin"]), ent, rel, nv, accs,
                                 d["batch_h"], d["batch_t"], d["batch_r"], bs, neg)
        for k, a in zip(("ent", "rel", "norm"), accs):
            ill.after(k, a)
        assert np.float32(loss) == np.float32(want), (s, loss, want)
        _equal(_tables(kge), (ent, rel, nv), "step %d" % s)
    keys = {"ent": "final_ent_embeddings", "rel": "final_rel_embeddings", "norm": "final_norm_vector"}
    for name, got in zip(("ent", "rel", "norm"), _tables(kge)):
        if got is not None:
            assert_tables_close(got, z[keys[name]], 1e-5, ill.get(name))


def _universe_jobs(model, dims, neg, bern, filt, seed, opt, epochs=2, nbatches=10):
    """Universes of kg_small built natively and by the oracle (same seeds), random init tables."""
    import ctypes
    from openke import _native
    L = _native.lib()
    g = ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(g)))
    kg = oracle.KG.load(KG_SMALL)
    jobs, cases = [], []
    rs = np.random.default_rng(seed)
    for i, dim in enumerate(dims):
        s = seed * 100 + i
        tc = int(rs.integers(150, 600))
        bal = float(rs.uniform(0.25, 0.5))
        h = ctypes.c_void_p()
        _native.check(L.pt_universe_build(g, s, 8, tc, ctypes.c_float(bal), ctypes.byref(h)))
        rng = oracle.GlibcRand(s)
        st = rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, tc, bal)
        E, R = ug.ent_total, ug.rel_total
        bound = np.sqrt(6.0 / (E + dim))
        tabs = [rs.uniform(-bound, bound, (E, dim)).astype(np.float32),
                rs.uniform(-bound, bound, (R, dim)).astype(np.float32),
                rs.uniform(-bound, bound, (R, dim)).astype(np.float32) if model == "TransH" else None]
        dev = [torch.from_numpy(x).cuda() if x is not None else None for x in tabs]
        accs = [torch.zeros_like(x) if x is not None else None for x in dev]
        seeds = np.zeros(8, dtype=np.uint64)
        _native.check(L.pt_universe_seeds(h, seeds.ctypes.data))
        bs = max(ug.train_total // nbatches, 1)
        j = _native.UniverseJob()
        j.graph = L.pt_universe_graph(h)
        j.seeds = seeds.ctypes.data
        j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, bs, epochs, nbatches, neg
        j.lr, j.margin = (0.05 if opt == "adagrad" else 0.3), 2.0
        j.ent, j.rel, j.normv = (x.data_ptr() if x is not None else None for x in dev)
        j.ent_acc, j.rel_acc, j.norm_acc = (x.data_ptr() if x is not None else None for x in accs)
        j.dim = dim
        jobs.append(j)
        cases.append({"h": h, "seeds": seeds, "ug": ug, "st": st.copy(), "tabs": tabs, "dev": dev, "accs": accs,
                      "bs": bs, "epochs": epochs, "nbatches": nbatches, "lr": float(j.lr), "margin": 2.0})
    return g, jobs, cases


def _oracle_universe_run(c, model, p, opt, neg, bern, filt):
    ent, rel, nv = (x.copy() if x is not None else None for x in c["tabs"])
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) \
        if opt == "adagrad" else (None, None, None)
    st = c["st"].copy()
    ep_loss = []
    for _ in range(c["epochs"]):
        tot = 0.0
        for _ in range(c["nbatches"]):
            h, t, r, _ = c["ug"].sample(st, 8, c["bs"], neg, bern, filt)
            tot += oracle.train_step(model, p, True, opt, c["lr"], c["margin"], ent, rel, nv, accs, h, t, r, c["bs"],
                                     neg)
        ep_loss.append(tot)
    return (ent, rel, nv), accs, ep_loss, st


@pytest.mark.parametrize("model,p,neg,bern,filt,opt", [
    ("TransE", 1, 1, 0, 0, "adagrad"),
    ("TransE", 2, 3, 1, 1, "adagrad"),
    ("TransH", 1, 1, 0, 0, "adagrad"),
    ("TransH", 2, 2, 1, 1, "sgd"),
    ("TransE", 1, 1, 1, 0, "sgd"),
])
def test_deterministic_universes_bit_exact(model, p, neg, bern, filt, opt):
    """pt_universes_train_ex(PT_DETERMINISTIC): every universe (mixed dims, odd ones included) equal to the
    oracle's training of the same universe - tables, Adagrad state, per-epoch loss sums."""
    from openke import _native
    L = _native.lib()
    dims = [8, 20, 50, 100, 20, 64, 69, 23]
    g, jobs, cases = _universe_jobs(model, dims, neg, bern, filt, 7 + neg + bern, opt)
    try:
        arr = (_native.UniverseJob * len(jobs))(*jobs)
        losses = torch.zeros(sum(c["epochs"] for c in cases), device="cuda")
        _native.check(L.pt_universes_train_ex(arr, len(jobs), 0 if model == "TransE" else 1, p, 1,
                                              _native.PT_ADAGRAD if opt == "adagrad" else _native.PT_SGD, bern, filt,
                                              _native.PT_DETERMINISTIC, _native.ptr(losses), _native.stream()))
        lh = losses.cpu().numpy()
        off = 0
        for c in cases:
            tabs, accs, ep_loss, _ = _oracle_universe_run(c, model, p, opt, neg, bern, filt)
            np.testing.assert_array_equal(lh[off:off + c["epochs"]], np.array(ep_loss, dtype=np.float32))
            off += c["epochs"]
            _equal([x.cpu().numpy() if x is not None else None for x in c["dev"]], tabs, "universe tables")
            if opt == "adagrad":
                _equal([x.cpu().numpy() if x is not None else None for x in c["accs"]], accs, "universe state_sum")
    finally:
        for c in cases:
            L.pt_universe_free(c["h"])
        L.pt_graph_free(g)


def _pu(z, tmp_path, deterministic):
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
                                    checkpoint_dir=str(tmp_path) + "/", valid_steps=10 ** 6, save_steps=None,
                                    training_setting="static", incremental_strategy=None,
                                    deterministic=deterministic)


def _oracle_golden_universe(kg, z, u):
    model, dim, p = str(z["model"]), int(z["dim"]), int(z["p_norm"])
    seed0 = int(z["seed0"])
    rng = oracle.GlibcRand(seed0 + u)
    st = rng.rand_reset(8)
    ug, em, rm = kg.universe(rng, int(z["u%d_tc" % u]), float(z["u%d_balance" % u]))
    bs = ug.train_total // 20
    ent, rel, nv = torch_init_tables(model, ug.ent_total, ug.rel_total, dim, seed0 + u)
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
    ill = IllConditioned()
    losses = []
    for _ in range(int(z["epochs"])):
        tot = 0.0
        for _ in range(20):
            h, t, r, _ = ug.sample(st, 8, bs, 1, 0, 0)
            for name, a in zip(("ent", "rel", "norm"), accs):
                ill.before(name, a)
            tot += oracle.train_step(model, p, True, "adagrad", float(z["u%d_lr" % u]), float(z["u%d_margin" % u]),
                                     ent, rel, nv, accs, h, t, r, bs, 1)
            for name, a in zip(("ent", "rel", "norm"), accs):
                ill.after(name, a)
        losses.append(tot)
    return (ent, rel, nv), ill, losses


@pytest.mark.parametrize("protocol", ["batched", "one_universe"])
@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_deterministic_pu_matches_oracle_and_reference(path, protocol, tmp_path):
    """Parallel_Universe_Config(deterministic=True) on the reference's golden PU runs, through the batched
    universe kernel (train_parallel_universes) and through the reference's one-universe protocol
    (set_random_seed -> compile_train_datset -> train_embedding_space on the fused trainer): every universe
    bit-identical to the oracle's Adagrad training; against the reference's own tables within 2e-5 wherever
    the oracle's trajectory had no noise-decided Adagrad step (the oracle-vs-reference relation of
    test_oracle.test_universes_match_reference, inherited exactly)."""
    z = load(path)
    model = str(z["model"])
    n_univ = int(z["n_univ"])
    pu = _pu(z, tmp_path, True)
    if protocol == "batched":
        pu.train_parallel_universes(n_univ)
    else:
        for _ in range(n_univ):
            pu.set_random_seed(pu.initial_random_seed + pu.next_universe_id)
            pu.compile_train_datset()
            pu.add_embedding_space(pu.train_embedding_space())
            pu.next_universe_id += 1
    kg = oracle.KG.load(KG_SMALL)
    for u in range(n_univ):
        sp = pu.trained_embedding_spaces[u]
        got = _tables(sp)
        want, ill, losses = _oracle_golden_universe(kg, z, u)
        _equal(got, want, "universe %d" % u)
        if protocol == "batched":
            np.testing.assert_array_equal(pu.last_universe_losses[u], np.array(losses, dtype=np.float32))
        if ill.events == 0:
            for name, g_ in zip(("ent", "rel", "norm"), got):
                if g_ is not None:
                    assert_tables_close(g_, z["u%d_%s" % (u, name)], 2e-5)


def test_deterministic_mode_switches_per_trainer():
    """The mode is per trainer handle: a deterministic and a fast trainer side by side, and pt_trainer_run_timed
    (the fast path's measurement hook) refuses a deterministic trainer."""
    import ctypes
    from openke import _native
    from openke.module.model import TransE
    L = _native.lib()
    torch.manual_seed(0)
    kge = TransE(50, 4, dim=8, p_norm=1, norm_flag=True).cuda()
    desc = kge.native_desc(_native.PT_SGD, 0.1, 1.0)
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    _native.check(L.pt_trainer_create(ctypes.byref(desc), ctypes.byref(a)))
    _native.check(L.pt_trainer_create(ctypes.byref(desc), ctypes.byref(b)))
    try:
        _native.check(L.pt_trainer_set_deterministic(a, 1))
        assert L.pt_trainer_get_deterministic(a) == 1 and L.pt_trainer_get_deterministic(b) == 0
        ms = (ctypes.c_float * 4)()
        losses = torch.zeros(2, device="cuda")
        assert L.pt_trainer_run_timed(a, None, 4, 1, 0, 0, 2, _native.ptr(losses), ms, _native.stream()) != 0
        assert b"fast path" in L.pt_last_error()
        _native.check(L.pt_trainer_set_deterministic(a, 0))
        assert L.pt_trainer_get_deterministic(a) == 0
    finally:
        L.pt_trainer_free(a)
        L.pt_trainer_free(b)


def test_failed_deterministic_enable_leaves_fast_mode():
    """a universe set whose batch is too large for the reference-order LDS plan refuses
    pt_universe_set_deterministic (PT_ENOTSUP) and stays in the fast mode - a later train call runs the fast
    kernel (finite losses, trained tables) instead of launching the ordered kernel without its workspace."""
    import ctypes
    from openke import _native
    L = _native.lib()
    g, jobs, cases = _universe_jobs("TransE", [20], 1, 0, 0, 3, "adagrad", epochs=1, nbatches=2)
    try:
        jobs[0].batch_size = cases[0]["bs"] = 1100   # 2,200 slots: 202 KB of ordered-mode LDS (> 160 KB)
        arr = (_native.UniverseJob * 1)(*jobs)
        uset = ctypes.c_void_p()
        _native.check(L.pt_universe_set_create(arr, 1, 0, 1, 1, _native.PT_ADAGRAD, 0, 0, ctypes.byref(uset)))
        try:
            before = cases[0]["dev"][0].clone()
            assert L.pt_universe_set_deterministic(uset, 1) != 0
            assert b"too large" in L.pt_last_error()
            losses = torch.zeros(1, device="cuda")
            _native.check(L.pt_universe_set_train(uset, _native.ptr(losses), _native.stream()))
            torch.cuda.synchronize()
            assert torch.isfinite(losses).all() and float(losses[0]) > 0
            assert not torch.equal(before, cases[0]["dev"][0])
        finally:
            L.pt_universe_set_free(uset)
    finally:
        for c in cases:
            L.pt_universe_free(c["h"])
        L.pt_graph_free(g)
