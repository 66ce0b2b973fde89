"""GPU parity tests: the HIP path (through the C-ABI and the drop-in openke API) against the
reference's golden vectors and the CPU oracle. Run on an MI355X: pytest -m gpu."""
import ctypes
import os
import tempfile

import numpy as np
import pytest
import torch

import oracle
from conftest import KG_SMALL, KG_TINY, PKG
from helpers import (DATASETS, IllConditioned, assert_close_vs_oracle, assert_ranks_match, assert_step_close,
                     assert_tables_close, golden, load, metrics_match_ranks, step_noise, torch_init_tables)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _loader(ds, threads, bs, neg, bern, filt, seed):
    from openke.data import TrainDataLoader
    return TrainDataLoader(in_path=DATASETS[ds], batch_size=bs, threads=threads, sampling_mode="normal",
                           bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)


@pytest.mark.parametrize("path", golden("sampler_*.npz"), ids=lambda p: p.split("/")[-1])
def test_sampler_bit_exact_on_gpu(path):
    """TrainDataLoader.sampling() (GPU sampler behind the Base.so-compatible ABI) == reference."""
    z = load(path)
    dl = _loader(str(z["dataset"]), int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"]), int(z["bern"]),
                 int(z["filter"]), int(z["seed"]))
    for c in range(z["batch_h"].shape[0]):
        d = dl.sampling()
        np.testing.assert_array_equal(d["batch_h"], z["batch_h"][c])
        np.testing.assert_array_equal(d["batch_t"], z["batch_t"][c])
        np.testing.assert_array_equal(d["batch_r"], z["batch_r"][c])
        np.testing.assert_array_equal(d["batch_y"], z["batch_y"][c])


def _model(z, dl):
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    torch.manual_seed(int(z["torch_seed"]))
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=int(z["dim"]), p_norm=int(z["p_norm"]),
              norm_flag=bool(z["norm_flag"]))
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=float(z["margin"])), batch_size=dl.get_batch_size())
    return kge, ns


def _tables(kge):
    out = {"ent": kge.ent_embeddings.weight.detach().cpu().numpy(),
           "rel": kge.rel_embeddings.weight.detach().cpu().numpy()}
    if hasattr(kge, "norm_vector"):
        out["norm"] = kge.norm_vector.weight.detach().cpu().numpy()
    return out


GOLD_KEYS = {"ent": "ent_embeddings", "rel": "rel_embeddings", "norm": "norm_vector"}


@pytest.mark.parametrize("path", golden("train_*.npz"), ids=lambda p: p.split("/")[-1])
def test_train_one_step_matches_reference(path):
    """Trainer.train_one_step on the reference's own batches: loss and updated tables."""
    from openke.config import Trainer
    z = load(path)
    dl = _loader("small", int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"]), int(z["bern"]),
                 int(z["filter"]), int(z["seed"]))
    kge, ns = _model(z, dl)
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=float(z["lr"]), use_gpu=True,
                 opt_method=str(z["opt"]))
    tr.run()
    ada = str(z["opt"]) == "adagrad"
    ill = IllConditioned()
    for s in range(int(z["steps"])):
        d = dl.sampling()
        np.testing.assert_array_equal(d["batch_h"], z["batch_h"][s])
        np.testing.assert_array_equal(d["batch_t"], z["batch_t"][s])
        np.testing.assert_array_equal(d["batch_r"], z["batch_r"][s])
        if ada:
            for name, a in zip(("ent", "rel", "norm"), tr.optimizer.state_sum):
                ill.before(name, None if a is None else a.cpu().numpy())
        loss = tr.train_one_step(d)
        assert abs(loss - z["losses"][s]) <= 1e-5 * max(1.0, abs(z["losses"][s])), (s, loss, z["losses"][s])
        if ada:
            for name, a in zip(("ent", "rel", "norm"), tr.optimizer.state_sum):
                ill.after(name, None if a is None else a.cpu().numpy())
        if s == 0:
            for k, v in _tables(kge).items():
                assert_tables_close(v, z["step1_" + GOLD_KEYS[k]], 2e-6, ill.get(k))
    for k, v in _tables(kge).items():
        assert_tables_close(v, z["final_" + GOLD_KEYS[k]], 1e-5, ill.get(k))


@pytest.mark.parametrize("path", golden("train_*.npz"), ids=lambda p: p.split("/")[-1])
def test_fused_epoch_matches_reference(path):
    """Trainer.run(): in-kernel sampling + fused steps replayed as one hipGraph == reference."""
    from openke.config import Trainer
    z = load(path)
    steps = int(z["steps"])
    dl = _loader("small", int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"]), int(z["bern"]),
                 int(z["filter"]), int(z["seed"]))
    dl.nbatches = steps
    kge, ns = _model(z, dl)
    tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=float(z["lr"]), use_gpu=True,
                 opt_method=str(z["opt"]))
    tr.run()
    ada = str(z["opt"]) == "adagrad"
    np.testing.assert_allclose(tr.last_epoch_loss, float(np.sum(z["losses"])), rtol=1e-5)
    # the oracle's independent float32 trajectory on the same (golden) batches
    ent, rel = z["init_ent_embeddings"].copy(), z["init_rel_embeddings"].copy()
    nv = z["init_norm_vector"].copy() if str(z["model"]) == "TransH" else None
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
    for s_ in range(steps):
        oracle.train_step(str(z["model"]), int(z["p_norm"]), bool(z["norm_flag"]), str(z["opt"]), float(z["lr"]),
                          float(z["margin"]), ent, rel, nv, accs, z["batch_h"][s_], z["batch_t"][s_], z["batch_r"][s_],
                          int(z["batch_size"]), int(z["neg_ent"]))
    orc = {"ent": ent, "rel": rel, "norm": nv}
    for k, v in _tables(kge).items():
        if ada:
            assert_close_vs_oracle(v, z["final_" + GOLD_KEYS[k]], orc[k])
        else:
            assert_tables_close(v, z["final_" + GOLD_KEYS[k]], 1e-5)
    # the stream advanced exactly like `steps` sampling() calls: the next batch matches the oracle's
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(int(z["seed"])).rand_reset(int(z["threads"]))
    for _ in range(steps + 1):
        h, t, r, _ = kg.sample(st, int(z["threads"]), int(z["batch_size"]), int(z["neg_ent"]), int(z["bern"]),
                               int(z["filter"]))
    d = dl.sampling()
    np.testing.assert_array_equal(d["batch_h"], h)
    np.testing.assert_array_equal(d["batch_t"], t)


@pytest.mark.parametrize("path", golden("lp_*.npz"), ids=lambda p: p.split("/")[-1])
def test_link_prediction_matches_reference(path):
    """Tester.run_link_prediction over the HIP scoring kernel == the reference's metrics."""
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    z = load(path)
    test_dl = TestDataLoader(KG_SMALL, "link")
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=int(z["dim"]),
              p_norm=int(z["p_norm"]), norm_flag=True)
    with torch.no_grad():
        kge.ent_embeddings.weight.copy_(torch.from_numpy(z["ent_embeddings"]))
        kge.rel_embeddings.weight.copy_(torch.from_numpy(z["rel_embeddings"]))
        if str(z["model"]) == "TransH":
            kge.norm_vector.weight.copy_(torch.from_numpy(z["norm_vector"]))
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=True)
    res = tester.run_link_prediction(type_constrain=False)
    np.testing.assert_allclose(np.array(res, dtype=np.float32), z["metrics"].astype(np.float32), rtol=1e-6)


@pytest.mark.parametrize("path", golden("lpt_*.npz"), ids=lambda p: p.split("/")[-1])
def test_type_constrained_link_prediction_matches_reference(path):
    """Tester.run_link_prediction(type_constrain=True) (k_rank_types on the GPU rows) == the reference's
    constrained metrics; the legacy testHead/testTail symbols with type_constrain on candidate-order
    vectors give the same (host ranking, Test.h:118-504)."""
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    z = load(path)
    test_dl = TestDataLoader(KG_SMALL, "link")
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=int(z["dim"]),
              p_norm=int(z["p_norm"]), norm_flag=True)
    with torch.no_grad():
        kge.ent_embeddings.weight.copy_(torch.from_numpy(z["ent_embeddings"]))
        kge.rel_embeddings.weight.copy_(torch.from_numpy(z["rel_embeddings"]))
        if str(z["model"]) == "TransH":
            kge.norm_vector.weight.copy_(torch.from_numpy(z["norm_vector"]))
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=True)
    res = tester.run_link_prediction(type_constrain=True)
    np.testing.assert_allclose(np.array(res, dtype=np.float32), z["metrics_tc"].astype(np.float32), rtol=1e-6)
    np.testing.assert_allclose(np.array(tester.last_metrics, dtype=np.float32), z["metrics"].astype(np.float32),
                               rtol=1e-6)
    # the reference's own loop over the Base.so-compatible symbols (Tester.py:70-93)
    L = tester.lib
    L.initTest()
    E = test_dl.get_ent_tot()
    for index, (dh, dt) in enumerate(test_dl):
        con = np.ascontiguousarray(tester.test_one_step(dh), dtype=np.float32)
        L.testHead(con.ctypes.data, index, 1)
        con = np.ascontiguousarray(tester.test_one_step(dt), dtype=np.float32)
        L.testTail(con.ctypes.data, index, 1)
        assert len(con) == E
    L.test_link_prediction(1)
    got = [L.getTestLinkMRR(1), L.getTestLinkMR(1), L.getTestLinkHit10(1), L.getTestLinkHit3(1), L.getTestLinkHit1(1)]
    np.testing.assert_allclose(np.array(got, dtype=np.float32), z["metrics_tc"].astype(np.float32), rtol=1e-6)
    got = [L.getTestLinkMRR(0), L.getTestLinkMR(0), L.getTestLinkHit10(0), L.getTestLinkHit3(0), L.getTestLinkHit1(0)]
    np.testing.assert_allclose(np.array(got, dtype=np.float32), z["metrics"].astype(np.float32), rtol=1e-6)


@pytest.mark.parametrize("path", golden("val_*.npz"), ids=lambda p: p.split("/")[-1])
def test_validator_matches_reference(path):
    """openke.config.Validator.valid() (the static experiments' early-stopping check, Validator.py:35-44)
    on the GPU == the reference's hit@10; the legacy validHead/validTail/getValidHit10 symbols agree."""
    from openke.config import Validator
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    z = load(path)
    valid_dl = TestDataLoader(KG_SMALL, "link", mode='valid')
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=valid_dl.get_ent_tot(), rel_tot=valid_dl.get_rel_tot(), dim=int(z["dim"]),
              p_norm=int(z["p_norm"]), norm_flag=True)
    with torch.no_grad():
        kge.ent_embeddings.weight.copy_(torch.from_numpy(z["ent_embeddings"]))
        kge.rel_embeddings.weight.copy_(torch.from_numpy(z["rel_embeddings"]))
        if str(z["model"]) == "TransH":
            kge.norm_vector.weight.copy_(torch.from_numpy(z["norm_vector"]))
    validator = Validator(model=kge, data_loader=valid_dl)
    assert validator.valid() == pytest.approx(float(z["hit10"]), rel=1e-6, abs=1e-7)
    L = validator.lib
    L.validInit()
    for index, (dh, dt) in enumerate(valid_dl):
        con = np.ascontiguousarray(validator.valid_one_step(dh), dtype=np.float32)
        L.validHead(con.ctypes.data, index)
        con = np.ascontiguousarray(validator.valid_one_step(dt), dtype=np.float32)
        L.validTail(con.ctypes.data, index)
    assert L.getValidHit10() == pytest.approx(float(z["hit10"]), rel=1e-6, abs=1e-7)


@pytest.mark.parametrize("model,p,norm_flag", [("TransE", 1, True), ("TransE", 2, True), ("TransE", 2, False),
                                               ("TransH", 1, True), ("TransH", 2, True)])
@pytest.mark.parametrize("dim", [8, 20, 50, 200, 300])
def test_scores_match_oracle(model, p, norm_flag, dim):
    """pt_score (model.predict) in all three modes against the oracle's restatement."""
    from openke.module.model import TransE, TransH
    E, R = 300, 9
    torch.manual_seed(dim + p)
    cls = TransE if model == "TransE" else TransH
    kge = cls(E, R, dim=dim, p_norm=p, norm_flag=norm_flag).cuda()
    T = _tables(kge)
    rng = np.random.default_rng(dim)
    n = 1000
    h, t, r = rng.integers(0, E, n), rng.integers(0, E, n), rng.integers(0, R, n)
    for mode, hh, tt, rr in (("normal", h, t, r), ("head_batch", h, t[:1], r[:1]), ("tail_batch", h[:1], t, r[:1])):
        got = kge.predict({"batch_h": hh, "batch_t": tt, "batch_r": rr, "mode": mode})
        ref = oracle.score(model, p, norm_flag, mode, T["ent"], T["rel"], T.get("norm"), hh, tt, rr)
        np.testing.assert_allclose(got, ref, rtol=2e-6, atol=2e-6)


def test_full_size_fb15k237_step_matches_oracle(tmp_path):
    """C2 shape (FB15K237-shaped synthetic: E=14,541, R=237, D=200, bs=2000, neg=25, L2, bern, filter):
    the GPU sampler is bit-exact with the oracle at full size and one fused SGD step matches the
    oracle's step from the same state within fp32 tolerance."""
    import sys
    sys.path.insert(0, os.path.join(PKG, "tools"))
    import synth_kg
    from openke.config import Trainer
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    path = synth_kg.ensure_dataset(str(tmp_path), "fb15k237")
    bs, neg = 2000, 25
    dl = _loader_path(path, 8, bs, neg, 1, 1, 4)
    kg = oracle.KG.load(path)
    st = oracle.GlibcRand(4).rand_reset(8)
    h, t, r, _ = kg.sample(st, 8, bs, neg, 1, 1)
    d = dl.sampling()
    np.testing.assert_array_equal(d["batch_h"], h)
    np.testing.assert_array_equal(d["batch_t"], t)
    np.testing.assert_array_equal(d["batch_r"], r)
    torch.manual_seed(0)
    kge = TransE(dl.get_ent_tot(), dl.get_rel_tot(), dim=200, p_norm=2, norm_flag=True)
    ent0 = kge.ent_embeddings.weight.detach().numpy().copy()
    rel0 = kge.rel_embeddings.weight.detach().numpy().copy()
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=5.0), batch_size=bs)
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=1.0, use_gpu=True)
    tr.run()
    # fused in-kernel-sampled step (the bench's step) vs oracle on the next batch
    dl.nbatches = 1
    tr.train_times = 1
    tr.run()
    h2, t2, r2, _ = kg.sample(st, 8, bs, neg, 1, 1)
    ent, rel = ent0.copy(), rel0.copy()
    loss = oracle.train_step("TransE", 2, True, "sgd", 1.0, 5.0, ent, rel, None, (None, None, None), h2, t2, r2, bs, neg)
    np.testing.assert_allclose(tr.last_epoch_loss, loss, rtol=1e-5)
    got = _tables(kge)
    assert_tables_close(got["ent"], ent, 1e-5)
    assert_tables_close(got["rel"], rel, 1e-5)


def _loader_path(path, threads, bs, neg, bern, filt, seed):
    from openke.data import TrainDataLoader
    return TrainDataLoader(in_path=path, batch_size=bs, threads=threads, sampling_mode="normal",
                           bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)


def test_missing_library_fails_loudly(monkeypatch):
    from openke import _native
    monkeypatch.setattr(_native, "_LIB", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libputranse_hip.so")
    with pytest.raises(_native.NativeError):
        _native.lib()


@pytest.mark.parametrize("dup", [False, True])
def test_gpu_ranking_matches_host_ranking(dup):
    """pt_score_rows + pt_rank_rows (GPU, entity order) == pt_score_queries + pt_rank_queries (host rules
    of testHead/testTail on the candidate-order rows), including exact ties (duplicated entity rows)."""
    from openke import _native
    from openke.data import TestDataLoader
    from openke.module.model import TransE
    L = _native.lib()
    tdl = TestDataLoader(KG_SMALL, "link")
    E, R = tdl.get_ent_tot(), tdl.get_rel_tot()
    torch.manual_seed(5)
    kge = TransE(E, R, dim=16, p_norm=1, norm_flag=True).cuda()
    if dup:   # many exact ties: every 4th entity copies its predecessor
        w = kge.ent_embeddings.weight.data
        w[1::4] = w[0::4][:w[1::4].shape[0]]
    h, t, r = tdl.eval_triples()
    known = L.pt_legacy_known()
    desc = kge.native_desc()
    n = len(h)
    dev = torch.device("cuda")
    qh, qt, qr = (torch.from_numpy(x).to(dev) for x in (h, t, r))
    for side, anchor, truth in ((0, t, qh), (1, h, qt)):
        cand = torch.empty((n, E), device=dev)
        _native.check(L.pt_score_queries(ctypes.byref(desc), side, _native.ptr(qh), _native.ptr(qt), _native.ptr(qr),
                                         n, _native.ptr(cand), _native.stream()))
        con = cand.cpu().numpy()
        raw_h, filt_h = np.zeros(n, np.int64), np.zeros(n, np.int64)
        _native.check(L.pt_rank_queries(known, E, h.ctypes.data, t.ctypes.data, r.ctypes.data, n, side,
                                        con.ctypes.data, raw_h.ctypes.data, filt_h.ctypes.data, 0))
        rows = torch.empty((n, E), device=dev)
        _native.check(L.pt_score_rows(ctypes.byref(desc), side, _native.ptr(qh), _native.ptr(qt), _native.ptr(qr), n,
                                      _native.ptr(rows), _native.stream()))
        a = np.ascontiguousarray(anchor)
        rr = np.ascontiguousarray(r)
        off = np.zeros(n + 1, np.int64)
        _native.check(L.pt_known_partners(known, side, n, a.ctypes.data, rr.ctypes.data, off.ctypes.data, None))
        part = np.zeros(max(int(off[-1]), 1), np.int64)
        _native.check(L.pt_known_partners(known, side, n, a.ctypes.data, rr.ctypes.data, off.ctypes.data,
                                          part.ctypes.data))
        raw = torch.zeros(n, dtype=torch.int64, device=dev)
        filt = torch.zeros(n, dtype=torch.int64, device=dev)
        # device arguments held by names until the kernel has run (a temporary would be freed and its
        # memory reused by the next argument's allocation before the launch)
        row_of = torch.arange(n, device=dev)
        d_off, d_part = torch.from_numpy(off).to(dev), torch.from_numpy(part).to(dev)
        _native.check(L.pt_rank_rows(_native.ptr(rows), E, _native.ptr(row_of), _native.ptr(truth), None,
                                     _native.ptr(d_off), _native.ptr(d_part), n, _native.ptr(raw), _native.ptr(filt),
                                     _native.stream()))
        np.testing.assert_array_equal(raw.cpu().numpy(), raw_h)
        np.testing.assert_array_equal(filt.cpu().numpy(), filt_h)
        # the two kernels score every (query, entity) identically
        gl = rows.cpu().numpy()
        for q in range(0, n, 17):
            cidx = oracle.candidates(E, int(h[q] if side == 0 else t[q]))
            np.testing.assert_array_equal(con[q], gl[q][cidx])


# Counting-sort (neg >= 4) step / apply kernels across their shapes: float4 rows at every lane-group
# width (D = 20 -> 8 lanes, 100 -> 32, 200 -> 64, 300 -> 64 x 2 chunks), negatives split over 1, 2 or 4
# lane groups and over several record windows (neg > G), the VEC=1 kernel (D % 4 != 0), TransH, p in
# {1, 2}, norm_flag on/off, SGD and Adagrad. Reference: the oracle's float32 steps on the same batches
# (the GPU sampler is bit-exact with the oracle's), tolerance 2e-5 absolute on the tables (Adagrad:
# noise-dominated components excluded, see assert_tables_close) and 1e-5 relative on the loss.
CSR_CASES = [
    # model, dim, p, norm_flag, opt, bs, neg
    ("TransE", 20, 1, True, "sgd", 64, 5),
    ("TransE", 100, 2, False, "adagrad", 48, 12),
    ("TransE", 200, 2, True, "sgd", 128, 25),
    ("TransE", 300, 1, True, "adagrad", 40, 30),
    ("TransE", 64, 2, True, "sgd", 24, 150),
    ("TransE", 18, 2, True, "sgd", 50, 8),
    ("TransH", 24, 2, True, "adagrad", 40, 6),
    ("TransE", 136, 2, False, "sgd", 60, 7),     # fused step + apply with one wave per positive
    ("TransE", 200, 1, True, "sgd", 6, 300),     # fused step + apply, two record windows per wave
]


@pytest.mark.parametrize("case", CSR_CASES, ids=lambda c: "%s-d%d-p%d-nf%d-%s-neg%d" % (c[0], c[1], c[2], c[3], c[4], c[6]))
def test_counting_sort_step_matches_oracle(case):
    from openke.config import Trainer
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    model, dim, p, nf, opt, bs, neg = case
    steps, lr, margin, seed = 3, (0.5 if opt == "sgd" else 0.1), 4.0, 7
    dl = _loader_path(KG_SMALL, 8, bs, neg, 1, 1, seed)
    dl.nbatches = steps
    torch.manual_seed(dim + neg)
    cls = TransE if model == "TransE" else TransH
    kge = cls(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=nf)
    t0 = _tables(kge)
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
    tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt)
    tr.run()
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(seed).rand_reset(8)
    ent, rel = t0["ent"].copy(), t0["rel"].copy()
    nv = t0["norm"].copy() if model == "TransH" else None
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)) if opt == "adagrad" \
        else (None, None, None)
    ill = IllConditioned()
    loss = 0.0
    for _ in range(steps):
        h, t, r, _ = kg.sample(st, 8, bs, neg, 1, 1)
        for k, a in zip(("ent", "rel", "norm"), accs):
            ill.before(k, a)
        loss += oracle.train_step(model, p, nf, opt, lr, margin, ent, rel, nv, accs, h, t, r, bs, neg)
        for k, a in zip(("ent", "rel", "norm"), accs):
            ill.after(k, a)
    np.testing.assert_allclose(tr.last_epoch_loss, loss, rtol=1e-5)
    got = _tables(kge)
    orc = {"ent": ent, "rel": rel, "norm": nv}
    for k, v in got.items():
        assert_tables_close(v, orc[k], 2e-5, ill.get(k) if opt == "adagrad" else None)


# The fused step + apply (step_apply.hip: each table row updated inside the step kernel by the wave whose
# gradient contribution arrives last, pt_trainer_set_step_apply) against the step + apply pair on the same
# batches and initial tables: the same operations in the same order per row, so the two differ only by the
# order of the positives' float atomics - per-step losses within 1e-5 relative, tables within 1e-5 absolute
# after 12 steps. Shapes: one float4 chunk per lane (D = 200), two (D = 300, Adagrad, p = 1), one wave per
# positive (neg 7, no normalization), two record windows per wave (neg 300).
SA_CASES = [
    # dim, p, norm_flag, opt, bs, neg
    (200, 2, True, "sgd", 128, 25),
    (300, 1, True, "adagrad", 40, 30),
    (136, 2, False, "sgd", 60, 7),
    (200, 1, True, "sgd", 6, 300),
]


@pytest.mark.parametrize("case", SA_CASES, ids=lambda c: "d%d-p%d-nf%d-%s-bs%d-neg%d" % c)
def test_step_apply_matches_step_and_apply_pair(case):
    from openke import _native
    from openke.config import Trainer
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    dim, p, nf, opt, bs, neg = case
    steps, lr, margin, seed = 12, (0.5 if opt == "sgd" else 0.1), 4.0, 11
    runs = {}
    for fused in (1, 0):
        dl = _loader_path(KG_SMALL, 8, bs, neg, 1, 1, seed)
        dl.nbatches = steps
        torch.manual_seed(dim + neg)
        kge = TransE(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=nf)
        ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
        tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt)
        tr._setup()
        _native.check(_native.lib().pt_trainer_set_step_apply(tr._native, fused))
        tr.run()
        assert _native.lib().pt_trainer_step_apply(tr._native) == fused
        runs[fused] = (tr.last_epoch_loss, _tables(kge))
    (l1, t1), (l0, t0) = runs[1], runs[0]
    np.testing.assert_allclose(l1, l0, rtol=1e-5)
    for k in t1:
        np.testing.assert_allclose(t1[k], t0[k], atol=1e-5, rtol=0)


@pytest.mark.parametrize("path", golden("tc_*.npz"), ids=lambda p: p.split("/")[-1])
def test_triple_classification_matches_reference(path):
    """Tester.run_triple_classification (Tester.py:142-191) with the classification loader: the GPU
    scores, the reference's threshold sweep and accuracy; then the next getTestBatch negatives
    (filtered corruption on sampler thread 0, Test.h:576-599) bit-exact with the reference's."""
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    z = load(path)
    dl = TestDataLoader(KG_SMALL, "classification")
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=int(z["dim"]), p_norm=int(z["p_norm"]),
              norm_flag=True)
    with torch.no_grad():
        kge.ent_embeddings.weight.copy_(torch.from_numpy(z["ent_embeddings"]))
        kge.rel_embeddings.weight.copy_(torch.from_numpy(z["rel_embeddings"]))
        if hasattr(kge, "norm_vector"):
            kge.norm_vector.weight.copy_(torch.from_numpy(z["norm_vector"]))
    tester = Tester(model=kge, data_loader=dl, use_gpu=True)
    acc, thr = tester.run_triple_classification()
    assert abs(acc - float(z["acc"])) < 1e-12, (acc, float(z["acc"]))
    np.testing.assert_allclose(float(thr), float(z["threshold"]), rtol=1e-5)
    pos, neg = next(iter(dl))
    for k in ("h", "t", "r"):
        np.testing.assert_array_equal(pos["batch_" + k], z["pos_" + k])
        np.testing.assert_array_equal(neg["batch_" + k], z["neg_" + k])


# The fused LDS sampling + counting-sort kernel (k_sample_sort, taken once a run pre-samples >= 96 steps
# in one chunk) against the two-pass form (k_sample_csr + k_scan_counts, pt_trainer_set_sampling) and the
# oracle over 120 steps: both forms draw the same batches (the per-step losses agree to float rounding:
# only the order of the gradient sums inside an entity's bucket may differ) and land on the oracle's
# tables. Tolerance: 1e-5 relative on every step's loss, 1e-4 absolute on the tables after 120 SGD steps.
@pytest.mark.parametrize("model", ["TransE", "TransH"])
def test_fused_sample_sort_matches_two_pass_and_oracle(model):
    from openke.config import Trainer
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    dim, p, bs, neg, steps, lr, margin, seed = 20, 1, 64, 5, 120, 0.05, 4.0, 5
    cls = TransE if model == "TransE" else TransH
    runs = {}
    from openke import _native
    for two_pass in ("0", "1"):
        dl = _loader_path(KG_SMALL, 8, bs, neg, 1, 1, seed)
        dl.nbatches = steps
        torch.manual_seed(19)
        kge = cls(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
        t0 = _tables(kge)
        ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
        tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method="sgd")
        tr._setup()
        _native.check(_native.lib().pt_trainer_set_sampling(tr._native, _native.PT_PATH_TWO_PASS if two_pass == "1"
                                                            else -1, 0))
        tr.run()
        assert _native.lib().pt_trainer_last_path(tr._native) == (_native.PT_PATH_TWO_PASS if two_pass == "1"
                                                                 else _native.PT_PATH_FUSED)
        runs[two_pass] = (tr.last_epoch_loss, _tables(kge), t0)
    (lf, tf, t0), (lt, tt, _) = runs["0"], runs["1"]
    np.testing.assert_allclose(lf, lt, rtol=1e-5)
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(seed).rand_reset(8)
    ent, rel = t0["ent"].copy(), t0["rel"].copy()
    nv = t0["norm"].copy() if model == "TransH" else None
    loss = 0.0
    for _ in range(steps):
        h, t, r, _ = kg.sample(st, 8, bs, neg, 1, 1)
        loss += oracle.train_step(model, p, True, "sgd", lr, margin, ent, rel, nv, (None, None, None), h, t, r,
                                  bs, neg)
    np.testing.assert_allclose(lf, loss, rtol=1e-5)
    orc = {"ent": ent, "rel": rel, "norm": nv}
    for k in tf:
        np.testing.assert_allclose(tf[k], tt[k], atol=1e-4, rtol=0)
        np.testing.assert_allclose(tf[k], orc[k], atol=1e-4, rtol=0)


def test_static_experiment_flow(tmp_path):
    """The control flow of the reference's static experiments (experiments/static_experiment_TransE_on_WN18.py
    :53-162) through the drop-in API: TrainDataLoader(nbatches=100) -> TransE -> NegativeSampling ->
    Validator on the valid split -> Trainer.run() in rounds of valid_steps epochs with early stopping,
    save_checkpoint + deepcopy of the best model -> Tester.run_link_prediction. Validation hit@10 and the
    test metrics must equal the oracle's ranking of the GPU-trained tables."""
    from copy import deepcopy

    from openke.config import Tester, Trainer, Validator
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    sys_test = __import__("test_oracle")
    dl = TrainDataLoader(in_path=KG_SMALL, nbatches=100, threads=8, sampling_mode="normal", bern_flag=0,
                         filter_flag=0, neg_ent=1, neg_rel=0, random_seed=12345)
    torch.manual_seed(5)
    transe = TransE(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=16, p_norm=1, norm_flag=True)
    model = NegativeSampling(model=transe, loss=MarginLoss(margin=4.0), batch_size=dl.get_batch_size())
    valid_dl = TestDataLoader(dl.in_path, "link", mode='valid')
    validator = Validator(model=transe, data_loader=valid_dl)
    trainer = Trainer(model=model, data_loader=dl, alpha=0.01, train_times=2, use_gpu=True)
    best, best_model, bad, hits, losses = 0, None, 0, [], []
    for _ in range(3):
        trainer.run()
        losses.append(trainer.last_epoch_loss)
        hit10 = validator.valid()
        hits.append(hit10)
        if hit10 > best:
            best, bad = hit10, 0
            best_model = deepcopy(transe)
            transe.save_checkpoint(str(tmp_path / "transe.ckpt"))
        else:
            bad += 1
    assert losses[-1] < losses[0], losses
    # the last validation == the oracle's ranking of the same (GPU-trained) tables
    kg = oracle.KG.load(KG_SMALL)
    E = kg.ent_total
    ent = transe.ent_embeddings.weight.detach().cpu().numpy()
    rel = transe.rel_embeddings.weight.detach().cpu().numpy()
    all_tr = [np.concatenate(x) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                              for f in ("test2id.txt", "train2id.txt", "valid2id.txt")))]

    def oracle_ranks(split):
        ev = oracle.sort_test(*oracle.read_triples(KG_SMALL + split))
        n = len(ev[0])
        con_h = np.zeros((n, E), dtype=np.float32)
        con_t = np.zeros((n, E), dtype=np.float32)
        for q in range(n):
            h, t, r = (int(x[q]) for x in ev)
            con_h[q] = oracle.score("TransE", 1, True, "head_batch", ent, rel, None, oracle.candidates(E, h), [t],
                                    [r])
            con_t[q] = oracle.score("TransE", 1, True, "tail_batch", ent, rel, None, [h], oracle.candidates(E, t),
                                    [r])
        met, ranks = oracle.link_prediction(E, all_tr, ev, con_h, con_t)
        return met, ranks, con_h, con_t

    # GPU and oracle scores of the same tables differ in summation order: ranks must agree up to
    # near-ties (the tables come from float-atomic training, so ties differ from run to run)
    _, vr, vch, vct = oracle_ranks("valid2id.txt")
    mism = assert_ranks_match(validator.last_ranks, vr, vch, vct)
    # hit@10 is the one of our ranks, which equal the oracle's up to float near-ties of the truth's score
    assert hits[-1] == pytest.approx(sys_test.valid_hit10(validator.last_ranks), rel=1e-6, abs=1e-7)
    if mism == 0:
        assert hits[-1] == pytest.approx(sys_test.valid_hit10(vr), rel=1e-6, abs=1e-7)
    # checkpoint round trip and the test metrics of the final model
    again = TransE(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=16, p_norm=1, norm_flag=True)
    again.load_checkpoint(str(tmp_path / "transe.ckpt"))
    np.testing.assert_array_equal(again.ent_embeddings.weight.detach().cpu().numpy(),
                                  best_model.ent_embeddings.weight.detach().cpu().numpy())
    tester = Tester(model=transe, data_loader=TestDataLoader(KG_SMALL, "link", mode='test'), use_gpu=True)
    res = tester.run_link_prediction(type_constrain=False)
    met, tr_, tch, tct = oracle_ranks("test2id.txt")
    metrics_match_ranks(res, tester.last_ranks)
    if assert_ranks_match(tester.last_ranks, tr_, tch, tct) == 0:
        np.testing.assert_allclose(np.array(res, dtype=np.float32), met, rtol=1e-5, atol=1e-6)


# The fast single-model trainer teacher-forced: every step starts from the oracle's state (tables, Adagrad
# state, sampler streams) and must equal the oracle's step - loss within 1e-5 relative, tables within 2e-6
# absolute + the forward-error bound of the step per element (helpers.kappa_bound: 2 k eps A |d update / d g|, A the
# oracle's absolute-value evaluation of the element's gradient, k = contributions + 2D + 16), except on the rows a
# near-tie decision touched (margin or p = 1 sign within rounding) and the components whose
# Adagrad update was noise-decided in either implementation
# (helpers.step_noise). Covers the small-neg in-step sampler path and the counting-sort path (neg >= 4)
# with its split sampler, TransE / TransH, p 1 / 2, SGD / Adagrad, the odd dims. Whole trajectories are
# compared bit for bit in deterministic mode (test_gpu_ordered.py).
TF_CASES = [
    # model, dim, p, norm_flag, opt, bs, neg, bern, filter, steps
    ("TransE", 20, 1, True, "adagrad", 50, 1, 0, 0, 25),
    ("TransE", 69, 1, True, "adagrad", 64, 3, 1, 1, 15),
    ("TransE", 23, 2, True, "adagrad", 40, 6, 0, 1, 15),
    ("TransE", 200, 2, True, "sgd", 120, 25, 1, 1, 6),
    ("TransE", 100, 2, False, "adagrad", 48, 12, 1, 1, 10),
    ("TransH", 23, 1, True, "adagrad", 48, 1, 0, 0, 20),
    ("TransH", 69, 2, True, "adagrad", 32, 5, 1, 1, 10),
    ("TransH", 20, 2, False, "sgd", 70, 2, 1, 0, 10),
]


@pytest.mark.parametrize("case", TF_CASES, ids=lambda c: "%s-d%d-p%d-nf%d-%s-bs%d-neg%d" % (c[0], c[1], c[2], c[3],
                                                                                         c[4], c[5], c[6]))
def test_fast_trainer_steps_teacher_forced(case):
    _teacher_forced_trainer(case)


# the slot-scale mode (pt_trainer_set_slot_scale) teacher-forced the same way: TransE float4 rows on the
# counting-sort path (neg >= 4), SGD and Adagrad, p 1 and 2, with and without normalization
TF_SC_CASES = [
    ("TransE", 200, 2, True, "sgd", 120, 25, 1, 1, 6),
    ("TransE", 100, 2, False, "adagrad", 48, 12, 1, 1, 10),
    ("TransE", 200, 1, True, "adagrad", 48, 9, 1, 1, 8),
    ("TransE", 12, 1, True, "sgd", 40, 6, 0, 1, 10),
]


@pytest.mark.parametrize("case", TF_SC_CASES, ids=lambda c: "%s-d%d-p%d-nf%d-%s-bs%d-neg%d" % (c[0], c[1], c[2], c[3],
                                                                                            c[4], c[5], c[6]))
def test_slot_scale_steps_teacher_forced(case):
    _teacher_forced_trainer(case, slot_scale=1)


def _teacher_forced_trainer(case, slot_scale=0):
    from openke import _native
    from openke.module.model import TransE, TransH
    model, dim, p, nf, opt, bs, neg, bern, filt, steps = case
    lr, margin, seed = (0.5 if opt == "sgd" else 0.05), 3.0, 23
    L = _native.lib()
    kg = oracle.KG.load(KG_SMALL)
    E, R = kg.ent_total, kg.rel_total
    torch.manual_seed(dim + neg)
    kge = (TransE if model == "TransE" else TransH)(E, R, dim=dim, p_norm=p, norm_flag=nf).cuda()
    ada = opt == "adagrad"
    devt = [t for t in kge.tables()]
    dacc = [None if t is None else torch.zeros_like(t) for t in devt] if ada else [None, None, None]
    ent, rel, nv = (None if t is None else t.detach().cpu().numpy().copy() for t in devt)
    accs = [np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv)] if ada else [None] * 3
    desc = kge.native_desc(_native.PT_ADAGRAD if ada else _native.PT_SGD, lr, margin, tuple(dacc))
    g, smp, tr = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(g)))
    st = oracle.GlibcRand(seed).rand_reset(8)
    _native.check(L.pt_sampler_create(g, 8, st.ctypes.data, ctypes.byref(smp)))
    _native.check(L.pt_trainer_create(ctypes.byref(desc), ctypes.byref(tr)))
    if slot_scale:
        _native.check(L.pt_trainer_set_slot_scale(tr, 1))
    try:
        loss = torch.zeros(1, device="cuda")
        for k in range(steps):
            with torch.no_grad():
                for d_, h_ in zip(devt, (ent, rel, nv)):
                    if h_ is not None:
                        d_.copy_(torch.from_numpy(h_))
                for d_, h_ in zip(dacc, accs):
                    if h_ is not None:
                        d_.copy_(torch.from_numpy(h_))
            _native.check(L.pt_sampler_set_seeds(smp, st.ctypes.data))
            loss.zero_()
            _native.check(L.pt_trainer_step(tr, smp, bs, neg, bern, filt, None, None, None, _native.ptr(loss),
                                            _native.stream()))
            got = [None if t is None else t.detach().cpu().numpy() for t in devt]
            got_acc = [None if t is None else t.cpu().numpy() for t in dacc]
            acc0 = [None if a is None else a.copy() for a in accs]
            tab0 = [None if a is None else a.copy() for a in (ent, rel, nv)]
            h, t, r, _ = kg.sample(st, 8, bs, neg, bern, filt)
            gm = oracle.grad_mass(model, p, nf, margin, ent, rel, nv, h, t, r, bs, neg)
            want = oracle.train_step(model, p, nf, opt, lr, margin, ent, rel, nv, accs, h, t, r, bs, neg)
            assert abs(float(loss.item()) - want) <= 1e-5 * max(1.0, abs(want)), (k, float(loss.item()), want)
            for i, name in enumerate(("ent", "rel", "norm")):
                w = (ent, rel, nv)[i]
                if w is None:
                    continue
                mask = step_noise(acc0[i], accs[i], got_acc[i]) if ada else None
                assert_step_close(got[i], w, 2e-6, mask, what="step %d %s" % (k, name), before=tab0[i],
                                  gm=gm[name], lr=lr, acc_before=acc0[i])
        if slot_scale:
            assert L.pt_trainer_slot_scale(tr) == 1
        # the streams advanced exactly like one sampling() call per step
        nxt = np.zeros(8, dtype=np.uint64)
        _native.check(L.pt_sampler_get_seeds(smp, nxt.ctypes.data))
        np.testing.assert_array_equal(nxt, st)
    finally:
        torch.cuda.synchronize()
        L.pt_trainer_free(tr)
        L.pt_sampler_free(smp)
        L.pt_graph_free(g)


# The slot-scale mode (pt_trainer_set_slot_scale: per-slot records and per-positive base rows instead of the
# corrupted entities' gradient rows; the apply pass re-forms every slot's row with the step kernel's own
# operations) against the contribution-row pair, from the same tables over 12 SGD steps (p 1 and 2). The re-formed
# rows are the stored rows' operations; the runs differ only by the order of the positive rows' float atomics,
# which SGD passes on at rounding level (tolerance 1e-6). Adagrad turns such noise into +-lr steps: the mode is
# teacher-forced against the oracle instead (test_slot_scale_steps_teacher_forced).
@pytest.mark.parametrize("case", [(200, 2, True, "sgd", 64, 25), (200, 1, True, "sgd", 48, 9),
                                  (12, 2, True, "sgd", 40, 6), (64, 1, False, "sgd", 32, 7)],
                         ids=lambda c: "d%d_p%d_%s_neg%d" % (c[0], c[1], c[3], c[5]))
def test_slot_scale_matches_contribution_rows(case):
    from openke import _native
    from openke.config import Trainer
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    dim, p, nf, opt, bs, neg = case
    steps, lr, margin, seed = 12, (0.5 if opt == "sgd" else 0.1), 4.0, 11
    runs = {}
    for sc in (1, 0):
        dl = _loader_path(KG_SMALL, 8, bs, neg, 1, 1, seed)
        dl.nbatches = steps
        torch.manual_seed(dim + neg)
        kge = TransE(dl.get_ent_tot(), dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=nf)
        ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
        tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt)
        tr._setup()
        _native.check(_native.lib().pt_trainer_set_slot_scale(tr._native, sc))
        tr.run()
        assert _native.lib().pt_trainer_slot_scale(tr._native) == sc
        runs[sc] = (tr.last_epoch_loss, _tables(kge))
    (l1, t1), (l0, t0) = runs[1], runs[0]
    np.testing.assert_allclose(l1, l0, rtol=1e-6)
    for k in t1:
        np.testing.assert_allclose(t1[k], t0[k], atol=1e-6, rtol=0)
