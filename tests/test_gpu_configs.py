"""Every BASELINE.json configuration under -m gpu, at its real shape (synthetic graphs of the named datasets'
shapes, tools/synth_kg.py; the same universe draws, dims and init as bench.py):

  C1  TransE on WN18, dim 50, batch 100, 1 negative, SGD       fast steps teacher-forced + reference order
  C3  PuTransE on WN18, 512 universes, dim ~ U{20..100}        whole set (fast) + longest universes vs oracle
  C4  PuTransE on Wikidata, 1024 universes, dim 200            whole set (fast) + longest universes + LP ranks
  C5  PuTransH on FB15K (1,345 relations: the LDS-fallback      whole set (fast) + longest universes vs oracle
      relation lists), 256 universes, dim 20

(C2 runs at full size in test_gpu_parity.test_full_size_fb15k237_step_matches_oracle.)

Whole-set checks (every universe of the workload, its full epochs): per-epoch losses finite, the last epoch's
loss below the first, every table moved, and the LCG streams advanced by exactly epochs x nbatches sampling()
calls (Python affine jump of the seeds). Longest universes (largest epochs x batch x dim) at 2 epochs: the
deterministic mode equal to the oracle bit for bit, and the fast kernel's every step teacher-forced against the
oracle (test_gpu_pu._teacher_forced_universes). pytest -m gpu."""
import ctypes
import os
import sys

import numpy as np
import pytest
import torch

import oracle
from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(PKG, "tools"))
sys.path.insert(0, REPO)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("synth"))


M64 = (1 << 64) - 1
LCG_A, LCG_C = 25214903917, 11


def lcg_jump(s, n):
    """State of the reference's per-thread LCG (Random.h:18-21) after n draws."""
    a, c = 1, 0                       # accumulated affine map x -> a x + c
    pa, pc = LCG_A, LCG_C             # the map of 2^k draws
    while n:
        if n & 1:
            a, c = (pa * a) & M64, (pa * c + pc) & M64
        pa, pc = (pa * pa) & M64, (pa * pc + pc) & M64
        n >>= 1
    return (a * int(s) + c) & M64


def advanced_states(seeds, threads, bs, dpp, calls):
    """LCG states after `calls` sampling() calls of bs positives (Base.cpp:200-207 thread split)."""
    per = bs // threads if bs % threads == 0 else bs // threads + 1
    out = np.zeros(threads, dtype=np.uint64)
    for i in range(threads):
        ln = min(max(bs - i * per, 0), per)
        out[i] = lcg_jump(seeds[i], calls * ln * dpp)
    return out


class Workload:
    """The universes of a bench.py PU workload (bench.PU_WORKLOADS: same seeds, draws, dims and tables)."""

    def __init__(self, name, data_dir):
        import bench
        import synth_kg
        from openke import _native
        self.L = _native.lib()
        self.n = _native
        shape, n_univ, model, dim_spec, p, tc_range, margin_range, _ = bench.PU_WORKLOADS[name]
        self.model, self.p, self.n_univ = model, p, n_univ
        self.path = synth_kg.ensure_dataset(data_dir, shape)
        self.g = ctypes.c_void_p()
        _native.check(self.L.pt_graph_load(self.path.encode(), ctypes.byref(self.g)))
        self.draws = [bench.universe_draws(k, tc_range, margin_range) for k in range(n_univ)]
        if isinstance(dim_spec, tuple):
            self.dims = [int(np.random.default_rng(1000 + k).integers(dim_spec[0], dim_spec[1] + 1))
                         for k in range(n_univ)]
        else:
            self.dims = [dim_spec] * n_univ
        seeds = np.array([4 + k for k in range(n_univ)], dtype=np.int64)
        tcs = np.array([d[0] for d in self.draws], dtype=np.int64)
        bals = np.array([d[1] for d in self.draws], dtype=np.float32)
        self.h = (ctypes.c_void_p * n_univ)()
        _native.check(self.L.pt_universe_build_many(self.g, n_univ, seeds.ctypes.data, 8, tcs.ctypes.data,
                                                    bals.ctypes.data, 0, self.h))
        self.E = [self.L.pt_universe_ent_total(self.h[k]) for k in range(n_univ)]
        self.R = [self.L.pt_universe_rel_total(self.h[k]) for k in range(n_univ)]
        self.bs = [self.L.pt_universe_train_total(self.h[k]) // 20 for k in range(n_univ)]
        self.xavier = bench._xavier

    def init_tables(self, k):
        rng = np.random.default_rng(k)
        D = self.dims[k]
        ent = self.xavier(rng, self.E[k], D)
        rel = self.xavier(rng, self.R[k], D)
        nv = self.xavier(rng, self.R[k], D) if self.model == "TransH" else None
        return [ent, rel, nv]

    def seeds(self, k):
        st = np.zeros(8, dtype=np.uint64)
        self.n.check(self.L.pt_universe_seeds(self.h[k], st.ctypes.data))
        return st

    def jobs(self, ks, epochs=None, tables=None):
        """UniverseJob array for universes ks (device tables kept alive in the returned list)."""
        jobs, keep = [], []
        for i, k in enumerate(ks):
            tabs = tables[i] if tables is not None else self.init_tables(k)
            dev = [None if a is None else torch.from_numpy(a.copy()).cuda() for a in tabs]
            acc = [None if a is None else torch.zeros_like(a) for a in dev]
            st = self.seeds(k)
            tc, bal, margin, ep, lr = self.draws[k]
            j = self.n.UniverseJob()
            j.graph = self.L.pt_universe_graph(self.h[k])
            j.seeds = st.ctypes.data
            j.threads, j.batch_size, j.nbatches, j.neg = 8, self.bs[k], 20, 1
            j.epochs = ep if epochs is None else epochs
            j.lr, j.margin = lr, margin
            j.ent, j.rel, j.normv = (a.data_ptr() if a is not None else None for a in dev)
            j.ent_acc, j.rel_acc, j.norm_acc = (a.data_ptr() if a is not None else None for a in acc)
            j.dim = self.dims[k]
            jobs.append(j)
            keep.append((dev, acc, st, tabs))
        return (self.n.UniverseJob * len(jobs))(*jobs), keep

    def longest(self, count):
        work = [self.draws[k][3] * self.bs[k] * self.dims[k] for k in range(self.n_univ)]
        return [int(k) for k in np.argsort(work)[::-1][:count]]

    def close(self):
        for k in range(self.n_univ):
            self.L.pt_universe_free(self.h[k])
        self.L.pt_graph_free(self.g)


def _whole_set(w):
    """Every universe of the workload through the fast kernel (pt_universe_set_*), full epochs."""
    L, n = w.L, w.n
    ks = list(range(w.n_univ))
    arr, keep = w.jobs(ks)
    uset = ctypes.c_void_p()
    mid = 0 if w.model == "TransE" else 1
    n.check(L.pt_universe_set_create(arr, len(ks), mid, w.p, 1, n.PT_ADAGRAD, 0, 0, ctypes.byref(uset)))
    try:
        epochs = [int(arr[i].epochs) for i in range(len(ks))]
        losses = torch.zeros(sum(epochs), device="cuda")
        n.check(L.pt_universe_set_train(uset, n.ptr(losses), n.stream()))
        torch.cuda.synchronize()
        lh = losses.cpu().numpy()
        assert np.isfinite(lh).all()
        off = 0
        for i, k in enumerate(ks):
            ls = lh[off:off + epochs[i]]
            off += epochs[i]
            assert ls[-1] < ls[0], (k, ls[0], ls[-1])
            got = np.zeros(8, dtype=np.uint64)
            n.check(L.pt_universe_set_states(uset, i, got.ctypes.data))
            np.testing.assert_array_equal(got, advanced_states(keep[i][2], 8, w.bs[k], 3, epochs[i] * 20))
            for dv, t0 in zip(keep[i][0], keep[i][3]):
                if dv is None:
                    continue
                x = dv.cpu().numpy()
                assert np.isfinite(x).all() and not np.array_equal(x, t0), k
    finally:
        L.pt_universe_set_free(uset)
    return keep


def _longest_vs_oracle(w, count=3, epochs=2):
    """The longest universes at `epochs` epochs: deterministic mode == oracle bit for bit; the fast kernel
    teacher-forced step by step against the oracle."""
    from test_gpu_pu import _teacher_forced_universes
    L, n = w.L, w.n
    kg = oracle.KG.load(w.path)
    ks = w.longest(count)
    arr, keep = w.jobs(ks, epochs=epochs)
    mid = 0 if w.model == "TransE" else 1
    losses = torch.zeros(count * epochs, device="cuda")
    n.check(L.pt_universes_train_ex(arr, count, mid, w.p, 1, n.PT_ADAGRAD, 0, 0, n.PT_DETERMINISTIC, n.ptr(losses),
                                    n.stream()))
    lh = losses.cpu().numpy()
    cases = []
    for i, k in enumerate(ks):
        tc, bal, margin, _, lr = w.draws[k]
        rng = oracle.GlibcRand(4 + k)
        st = rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, tc, bal)
        assert ug.ent_total == w.E[k] and ug.train_total // 20 == w.bs[k]
        ent, rel, nv = (None if a is None else a.copy() for a in keep[i][3])
        accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
        st0 = st.copy()
        for e in range(epochs):
            tot = 0.0
            for _ in range(20):
                hh, tt, rr, _ = ug.sample(st, 8, w.bs[k], 1, 0, 0)
                tot += oracle.train_step(w.model, w.p, True, "adagrad", lr, float(margin), ent, rel, nv, accs, hh, tt,
                                         rr, w.bs[k], 1)
            assert np.float32(tot) == lh[i * epochs + e], (k, e, tot, lh[i * epochs + e])
        for dv, want in zip(keep[i][0], (ent, rel, nv)):
            if want is not None:
                np.testing.assert_array_equal(dv.cpu().numpy(), want)
        for dv, want in zip(keep[i][1], accs):
            if want is not None:
                np.testing.assert_array_equal(dv.cpu().numpy(), want)
        cases.append({"h": w.h[k], "ug": ug, "st": st0, "tabs": keep[i][3], "bs": w.bs[k], "lr": lr,
                      "margin": float(margin), "epochs": epochs, "nbatches": 20})
    _teacher_forced_universes(L, cases, w.model, w.p, "adagrad", 1, 0, 0)


@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_pu_workload_whole_set_and_longest_universes(name, data_dir):
    w = Workload(name, data_dir)
    try:
        _whole_set(w)
        _longest_vs_oracle(w)
    finally:
        w.close()


C4_LP_QUERIES = 240   # test queries of C4's link-prediction parity (of 6,000), every key against 1024 universes


def test_c4_link_prediction_ranks_match_oracle(data_dir):
    """C4's link prediction (global energy estimation over 1024 trained universes, Parallel_Universe_Config.py
    :446-642): the device path (pt_lp_min_scores key rows -> pt_rank_rows) on a subset of test queries ranks
    every query as the oracle does on the same trained tables (equal up to float near-ties of the truth's
    score), and the metrics are those of the ranks."""
    from helpers import assert_ranks_match, metrics_match_ranks
    from openke.config.Parallel_Universe_Config import lookup_local, lp_pair_array, lp_pairs_all
    w = Workload("c4", data_dir)
    L, n = w.L, w.n
    try:
        keep = _whole_set(w)
        E = sum(1 for _ in open(os.path.join(w.path, "entity2id.txt")))
        trip = {f: np.loadtxt(os.path.join(w.path, f), dtype=np.int64, ndmin=2)
                for f in ("train2id.txt", "valid2id.txt", "test2id.txt")}
        allt = np.concatenate(list(trip.values()))
        test = trip["test2id.txt"][:C4_LP_QUERIES]
        th, tt, tr = (np.ascontiguousarray(test[:, c]) for c in range(3))
        nq = len(th)
        ems, rms = [], []
        for k in range(w.n_univ):
            em = np.zeros(max(w.E[k], 1), np.int64)
            rm = np.zeros(max(w.R[k], 1), np.int64)
            n.check(L.pt_universe_remaps(w.h[k], em.ctypes.data, rm.ctypes.data))
            ems.append(em[:w.E[k]])
            rms.append(rm[:w.R[k]])
        keys = {}
        q_row = [np.zeros(nq, np.int64), np.zeros(nq, np.int64)]
        for q in range(nq):
            for side, anchor in ((0, int(tt[q])), (1, int(th[q]))):
                q_row[side][q] = keys.setdefault((side, anchor, int(tr[q])), len(keys))
        ks = np.array([k[0] for k in keys], np.int64)
        ka = np.array([k[1] for k in keys], np.int64)
        kr = np.array([k[2] for k in keys], np.int64)
        dev = torch.device("cuda")
        rows = torch.full((len(keys), E), float("inf"), device=dev)
        moff = np.cumsum([0] + [len(e) for e in ems])
        dremaps = torch.from_numpy(np.concatenate(ems)).to(dev)
        lp_us = []
        for k in range(w.n_univ):
            U = n.LpUniverse()
            ent, rel, _ = keep[k][0]
            U.ent, U.rel, U.normv = ent.data_ptr(), rel.data_ptr(), None
            U.ent_total, U.rel_total, U.dim = w.E[k], w.R[k], w.dims[k]
            U.d_ent_remap = dremaps.data_ptr() + 8 * int(moff[k])
            lp_us.append(U)
        pair_arr, arr_p = lp_pair_array([lp_pairs_all(ems, rms, ka, kr, ks)])
        arr_u = (n.LpUniverse * len(lp_us))(*lp_us)
        n.check(L.pt_lp_min_scores(arr_u, len(lp_us), 0, w.p, 1, arr_p, len(pair_arr), E, n.ptr(rows), None,
                                   n.stream()))
        known = ctypes.c_void_p()
        ah, at, ar = (np.ascontiguousarray(allt[:, c]) for c in range(3))
        n.check(L.pt_known_create(ah.ctypes.data, at.ctypes.data, ar.ctypes.data, len(ah), ctypes.byref(known)))
        ranks = []
        for side, anchor, truth in ((0, tt, th), (1, th, tt)):
            off = np.zeros(nq + 1, np.int64)
            n.check(L.pt_known_partners(known, side, nq, anchor.ctypes.data, tr.ctypes.data, off.ctypes.data, None))
            part = np.zeros(max(int(off[-1]), 1), np.int64)
            n.check(L.pt_known_partners(known, side, nq, anchor.ctypes.data, tr.ctypes.data, off.ctypes.data,
                                        part.ctypes.data))
            d_row = torch.from_numpy(q_row[side]).to(dev)
            d_truth = torch.from_numpy(truth).to(dev)
            d_off, d_part = torch.from_numpy(off).to(dev), torch.from_numpy(part).to(dev)
            raw = torch.zeros(nq, dtype=torch.int64, device=dev)
            filt = torch.zeros(nq, dtype=torch.int64, device=dev)
            n.check(L.pt_rank_rows(n.ptr(rows), E, n.ptr(d_row), n.ptr(d_truth), None, n.ptr(d_off), n.ptr(d_part),
                                   nq, n.ptr(raw), n.ptr(filt), n.stream()))
            ranks += [raw.cpu().numpy(), filt.cpu().numpy()]
        L.pt_known_free(known)
        met = np.zeros(10, dtype=np.float32)
        n.check(L.pt_lp_metrics(ranks[0].ctypes.data, ranks[1].ctypes.data, ranks[2].ctypes.data,
                                ranks[3].ctypes.data, nq, met.ctypes.data))
        metrics_match_ranks(met[:5], tuple(ranks))
        # the oracle: per key the MIN over every universe holding the anchor and the relation of its scores
        # of every local entity, in candidate order (getHeadBatch / getTailBatch); one oracle.score call per
        # (universe, side) over all the queries the universe holds, universes on a thread pool
        tabs = [[x.cpu().numpy() for x in keep[k][0][:2]] for k in range(w.n_univ)]
        head_vec = np.full((nq, E), np.inf, dtype=np.float32)
        tail_vec = np.full((nq, E), np.inf, dtype=np.float32)

        def universe_scores(k):
            eo = np.argsort(ems[k], kind="stable")
            ro = np.argsort(rms[k], kind="stable")
            lh = lookup_local(ems[k][eo], eo, th)
            lt = lookup_local(ems[k][eo], eo, tt)
            lr = lookup_local(rms[k][ro], ro, tr)
            out = []
            Ek = w.E[k]
            loc = np.arange(Ek, dtype=np.int64)
            for mode, anchor in (("tail_batch", lh), ("head_batch", lt)):
                qs = np.nonzero((lr >= 0) & (anchor >= 0))[0]
                if len(qs) == 0:
                    continue
                a = np.repeat(anchor[qs], Ek)
                c = np.tile(loc, len(qs))
                rr = np.repeat(lr[qs], Ek)
                sc = oracle.score("TransE", w.p, True, mode, tabs[k][0], tabs[k][1], None,
                                  a if mode == "tail_batch" else c, c if mode == "tail_batch" else a, rr)
                out.append((mode, qs, sc.reshape(len(qs), Ek)))
            return k, out

        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=16) as ex:
            for k, out in ex.map(universe_scores, range(w.n_univ)):
                for mode, qs, sc in out:
                    vec = tail_vec if mode == "tail_batch" else head_vec
                    sub = vec[np.ix_(qs, ems[k])]
                    vec[np.ix_(qs, ems[k])] = np.minimum(sub, sc)
        con_h = np.stack([head_vec[q][oracle.candidates(E, int(th[q]))] for q in range(nq)])
        con_t = np.stack([tail_vec[q][oracle.candidates(E, int(tt[q]))] for q in range(nq)])
        _, want = oracle.link_prediction(E, [allt[:, 0], allt[:, 1], allt[:, 2]], (th, tt, tr), con_h, con_t)
        assert_ranks_match(tuple(ranks), want, con_h, con_t)
    finally:
        w.close()


@pytest.mark.parametrize("bs", [100, 1414])   # the config's batch 100, and nbatches = 100 of the WN18 experiment
def test_c1_wn18_steps_match_oracle(bs, data_dir):
    """C1: TransE on a WN18-shaped graph (40,943 entities), dim 50, 1 negative, L1, SGD (bench.py c1): the
    fast trainer's steps teacher-forced against the oracle, and 10 steps of the deterministic mode equal to the
    oracle's bit for bit."""
    import bench
    import synth_kg
    from helpers import assert_step_close
    from openke import _native
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    shape, model, dim, p, opt, lr, margin, _, neg, bern, filt = bench.WORKLOADS["c1"]
    path = synth_kg.ensure_dataset(data_dir, shape)
    L = _native.lib()
    kg = oracle.KG.load(path)
    torch.manual_seed(1)
    kge = TransE(kg.ent_total, kg.rel_total, dim=dim, p_norm=p, norm_flag=True).cuda()
    ent, rel = (t.detach().cpu().numpy().copy() for t in kge.tables()[:2])
    init = (ent.copy(), rel.copy())
    desc = kge.native_desc(_native.PT_SGD, lr, margin)
    g, smp, tr = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    _native.check(L.pt_graph_load(path.encode(), ctypes.byref(g)))
    st = oracle.GlibcRand(4).rand_reset(8)
    _native.check(L.pt_sampler_create(g, 8, st.ctypes.data, ctypes.byref(smp)))
    _native.check(L.pt_trainer_create(ctypes.byref(desc), ctypes.byref(tr)))
    try:
        loss = torch.zeros(1, device="cuda")
        for k in range(5):
            with torch.no_grad():
                kge.ent_embeddings.weight.copy_(torch.from_numpy(ent))
                kge.rel_embeddings.weight.copy_(torch.from_numpy(rel))
            _native.check(L.pt_sampler_set_seeds(smp, st.ctypes.data))
            loss.zero_()
            _native.check(L.pt_trainer_step(tr, smp, bs, neg, bern, filt, None, None, None, _native.ptr(loss),
                                            _native.stream()))
            got = [t.detach().cpu().numpy() for t in kge.tables()[:2]]
            before = (ent.copy(), rel.copy())
            h, t, r, _ = kg.sample(st, 8, bs, neg, bern, filt)
            gm = oracle.grad_mass(model, p, True, margin, ent, rel, None, h, t, r, bs, neg)
            want = oracle.train_step(model, p, True, opt, lr, margin, ent, rel, None, (None, None, None), h, t, r, bs,
                                     neg)
            assert abs(float(loss.item()) - want) <= 1e-5 * max(1.0, abs(want)), (k, float(loss.item()), want)
            for gg, ww, b0, nm in zip(got, (ent, rel), before, ("ent", "rel")):
                assert_step_close(gg, ww, 2e-6, what="step %d %s" % (k, nm), before=b0, gm=gm[nm], lr=lr)
    finally:
        torch.cuda.synchronize()
        L.pt_trainer_free(tr)
        L.pt_sampler_free(smp)
        L.pt_graph_free(g)
    # reference order: Trainer(deterministic=True) through the drop-in loader, 10 steps
    dl = TrainDataLoader(in_path=path, batch_size=bs, threads=8, sampling_mode="normal", bern_flag=bern,
                         filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=4)
    dl.nbatches = 10
    with torch.no_grad():
        kge.ent_embeddings.weight.copy_(torch.from_numpy(init[0]))
        kge.rel_embeddings.weight.copy_(torch.from_numpy(init[1]))
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
    trn = Trainer(model=ns, data_loader=dl, train_times=1, alpha=lr, use_gpu=True, opt_method=opt, deterministic=True)
    trn.run()
    ent, rel = init[0].copy(), init[1].copy()
    st = oracle.GlibcRand(4).rand_reset(8)
    losses = []
    for _ in range(10):
        h, t, r, _ = kg.sample(st, 8, bs, neg, bern, filt)
        losses.append(oracle.train_step(model, p, True, opt, lr, margin, ent, rel, None, (None, None, None), h, t, r,
                                        bs, neg))
    np.testing.assert_array_equal(trn.last_step_losses, np.array(losses, dtype=np.float32))
    np.testing.assert_array_equal(kge.ent_embeddings.weight.detach().cpu().numpy(), ent)
    np.testing.assert_array_equal(kge.rel_embeddings.weight.detach().cpu().numpy(), rel)
