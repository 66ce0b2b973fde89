"""Cross sampling and relation corruption on the GPU, against the reference's goldens and the oracle.

sampling() takes a mode and a relation-corruption rate besides the normal form (Base.cpp:185-264):
mode -1 (TrainDataLoader.sampling_head) replaces every negative's head through corrupt_tail, mode 1
(sampling_tail) its tail through corrupt_head, both with corrupt_*'s default filter (Corrupt.h:9, :59),
and cross_sampling alternates them (TrainDataLoader.py:198-246); neg_rel appends relation corruptions
(corrupt_rel, Corrupt.h:108-189). The GPU sampler (k_sample) must reproduce the reference's batches
bit for bit (goldens samplermode_*.npz, made by tests/golden/make_golden.py from the reference), and
Trainer.run / train_one_step must train on them like the oracle's float32 restatement (1e-5).
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import KG_SMALL
from helpers import DATASETS, golden, load
from test_oracle import call_modes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _loader(ds, threads, bs, neg, neg_rel, bern, filt, seed, mode="cross", nbatches=None):
    from openke.data import TrainDataLoader
    return TrainDataLoader(in_path=DATASETS[ds], batch_size=bs, nbatches=nbatches, threads=threads,
                           sampling_mode=mode, bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=neg_rel,
                           random_seed=seed)


@pytest.mark.parametrize("path", golden("samplermode_*.npz"), ids=lambda p: p.split("/")[-1])
def test_sampler_modes_bit_exact_on_gpu(path):
    """sampling_head / sampling_tail / cross_sampling / neg_rel through the drop-in loader == reference."""
    z = load(path)
    bs = int(z["batch_size"])
    dl = _loader(str(z["dataset"]), int(z["threads"]), bs, int(z["neg_ent"]), int(z["neg_rel"]), int(z["bern"]),
                 int(z["filter"]), int(z["seed"]))
    fn = {"n": dl.sampling, "h": dl.sampling_head, "t": dl.sampling_tail, "c": dl.cross_sampling}
    for c, call in enumerate(str(z["calls"])):
        d = fn[call]()
        assert d["mode"] == str(z["modes"][c])
        np.testing.assert_array_equal(dl.batch_h, z["batch_h"][c])
        np.testing.assert_array_equal(dl.batch_t, z["batch_t"][c])
        np.testing.assert_array_equal(dl.batch_r, z["batch_r"][c])
        np.testing.assert_array_equal(dl.batch_y, z["batch_y"][c])
        # the returned views are the reference's slices (TrainDataLoader.py:212-217, :231-236)
        if d["mode"] == "head_batch":
            assert len(d["batch_t"]) == bs and len(d["batch_r"]) == bs and len(d["batch_h"]) == len(dl.batch_h)
        if d["mode"] == "tail_batch":
            assert len(d["batch_h"]) == bs and len(d["batch_r"]) == bs and len(d["batch_t"]) == len(dl.batch_t)


def _model(model, dl, dim, p, seed, margin):
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    torch.manual_seed(seed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    init = [kge.ent_embeddings.weight.detach().numpy().copy(), kge.rel_embeddings.weight.detach().numpy().copy(),
            kge.norm_vector.weight.detach().numpy().copy() if model == "TransH" else None]
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=dl.get_batch_size())
    return kge, ns, init


def _tables(kge):
    out = [kge.ent_embeddings.weight.detach().cpu().numpy(), kge.rel_embeddings.weight.detach().cpu().numpy()]
    out.append(kge.norm_vector.weight.detach().cpu().numpy() if hasattr(kge, "norm_vector") else None)
    return out


RUN_CASES = [
    # model, dim, p, opt, lr, sampling_mode, threads, bs, neg_ent, neg_rel, bern, filter, seed, steps
    ("TransE", 16, 1, "sgd", 0.5, "cross", 8, 120, 2, 0, 1, 1, 41, 4),
    ("TransE", 24, 2, "sgd", 0.3, "normal", 8, 100, 2, 1, 0, 1, 42, 3),
    ("TransH", 12, 2, "sgd", 0.2, "cross", 5, 77, 1, 2, 1, 0, 43, 3),
    ("TransE", 20, 1, "sgd", 0.05, "cross", 8, 150, 3, 1, 0, 1, 44, 2),
]


@pytest.mark.parametrize("case", RUN_CASES, ids=lambda c: "%s-%s-neg%d-rel%d-%s" % (c[0], c[5], c[8], c[9], c[3]))
def test_cross_and_relation_training_matches_oracle(case):
    """Trainer.run() over cross-sampled / relation-corrupted batches (TrainDataLoader.__iter__ ->
    cross_sampling, Trainer.py:91-100) == the oracle's sampling + float32 training restatement."""
    from openke.config import Trainer
    model, dim, p, opt, lr, smode, threads, bs, neg, neg_rel, bern, filt, seed, steps = case
    margin = 4.0
    dl = _loader("small", threads, bs, neg, neg_rel, bern, filt, seed, mode=smode)
    dl.nbatches = steps
    kge, ns, init = _model(model, dl, dim, p, seed + 100, margin)
    tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt)
    tr.run()
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(seed).rand_reset(threads)
    ent, rel, nv = (None if a is None else a.copy() for a in init)
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
    modes = call_modes("c" * steps) if smode == "cross" else [0] * steps
    total = 0.0
    for mode in modes:
        h, t, r, _ = kg.sample_ex(st, threads, bs, neg, neg_rel, mode, bern, filt)
        if mode != 0:
            # sampling_head / sampling_tail return the first bs relations and fixed-side entities, which the
            # model broadcasts over every negative (TransE.py:51-58): relation-corruption slots become
            # copies of their positive
            fixed = t if mode == -1 else h
            fixed.reshape(-1, bs)[1:] = fixed[:bs]
            r.reshape(-1, bs)[1:] = r[:bs]
        total += oracle.train_step(model, p, True, opt, lr, margin, ent, rel, nv, accs, h, t, r, bs, neg + neg_rel)
    np.testing.assert_allclose(tr.last_epoch_loss, total, rtol=1e-5, atol=1e-6)
    for got, want in zip(_tables(kge), (ent, rel, nv)):
        if want is not None:
            np.testing.assert_allclose(got, want, rtol=0, atol=2e-5)
    # the loader's cross flag and the sampler streams advanced like `steps` loader calls
    nxt = call_modes("c" * (steps + 1))[-1] if smode == "cross" else 0
    h, t, r, _ = kg.sample_ex(st, threads, bs, neg, neg_rel, nxt, bern, filt)
    d = dl.cross_sampling() if smode == "cross" else dl.sampling()
    np.testing.assert_array_equal(dl.batch_h, h)
    np.testing.assert_array_equal(dl.batch_t, t)
    np.testing.assert_array_equal(dl.batch_r, r)
    assert d["mode"] == {0: "normal", -1: "head_batch", 1: "tail_batch"}[nxt]


@pytest.mark.parametrize("mode", ["head_batch", "tail_batch"])
def test_train_one_step_on_cross_batch(mode):
    """Trainer.train_one_step on a head_batch / tail_batch dict (the broadcast form TransE._calc reshapes,
    TransE.py:51-58) == the oracle on the expanded batch."""
    from openke.config import Trainer
    threads, bs, neg, seed = 8, 90, 3, 45
    dl = _loader("small", threads, bs, neg, 0, 1, 1, seed)
    kge, ns, init = _model("TransE", dl, 16, 2, 7, 3.0)
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=0.4, use_gpu=True, opt_method="sgd")
    tr.run()
    d = dl.sampling_head() if mode == "head_batch" else dl.sampling_tail()
    loss = tr.train_one_step(d)
    ent, rel = init[0].copy(), init[1].copy()
    want = oracle.train_step("TransE", 2, True, "sgd", 0.4, 3.0, ent, rel, None, (None, None, None), dl.batch_h,
                             dl.batch_t, dl.batch_r, bs, neg)
    assert abs(loss - want) <= 1e-5 * max(1.0, abs(want)), (loss, want)
    got = _tables(kge)
    np.testing.assert_allclose(got[0], ent, rtol=0, atol=2e-6)
    np.testing.assert_allclose(got[1], rel, rtol=0, atol=2e-6)


@pytest.mark.parametrize("path", golden("nbr_*.npz"), ids=lambda p: p.split("/")[-1])
def test_neighbourhood_getters_match_reference(path):
    """TrainDataLoader.get_positive_entities / get_negative_entities / get_entity_relations (Base.cpp:312-466)
    on the full graph and on a swapped-in universe == the reference's outputs."""
    z = load(path)
    dl = _loader("small", 8, 50, 1, 0, 0, 0, int(z["seed"]), mode="normal")
    uni = z["universe"]
    if len(uni):
        dl.compile_universe_dataset(int(uni[0]), float(uni[1]))
        dl.swap_helpers()
    assert dl.lib.getEntityTotal() == int(z["ent_total"]) and dl.lib.getRelationTotal() == int(z["rel_total"])
    for i, (e, r, f) in enumerate(z["queries"]):
        np.testing.assert_array_equal(dl.get_positive_entities(int(e), int(r), int(f)), z["pos_%d" % i])
        np.testing.assert_array_equal(dl.get_negative_entities(int(e), int(r), int(f)), z["neg_%d" % i])
        np.testing.assert_array_equal(dl.get_entity_relations(int(e), int(f)), z["rels_%d" % i])
    if len(uni):
        dl.reset_universe()
