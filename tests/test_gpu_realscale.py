"""Real-scale parity of the HIP path against the reference's own outputs on the reference's own data
(tests/golden/real*.npz; see tests/realdata.py and tests/test_realscale_cpu.py, which pins the oracle to the same
fixtures).

* Tester.run_link_prediction on the GPU (pt_score_rows + k_rank_rows, k_rank_types for type_constrain) with the
  reference-trained TransH WN18 table (E = 40,943, 5,000 test triples, both sides) and TransE FB15K table
  (E = 14,951): every query's raw / filtered / type-constrained count equal to the reference's (Test.h:118-359)
  except by at most its near-ties, metrics equal when the counts are; GPU scores within 1e-5 of the reference's
  score vectors (TransE.py:46-74, TransH.py:52-93) and of the oracle's;
* the device sampler behind TrainDataLoader.sampling() at WN18 scale: SHA-1 of every call equal to the
  reference's (Base.cpp:266-310), and C2's counting-sort sampler (pt_trainer_sample_csr) on WN18 equal to the
  reference's first bs 2,000 x 25 batch;
* the drop-in universe protocol on WN18 (setRandomSeed / randReset, getParallelUniverse, swapHelpers, sampling,
  resetUniverse) for seeds 4-11: the reference's remaps and the SHA-1 of its universe batches.
"""
import ctypes
import hashlib
import random

import numpy as np
import pytest
import torch

import oracle
import realdata
from helpers import golden, load

pytestmark = pytest.mark.gpu

# near-tie band, relative to max(1, |truth score|): twice the largest GPU-vs-reference score difference measured on
# these tables, for both operands of a comparison (test_gpu_scores_match_reference_vectors holds them to it)
TIE_REL = 4e-6
SCORE_ATOL = 1e-5   # north_star's fp32 tolerance


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


@pytest.fixture(scope="module")
def real_dirs(tmp_path_factory):
    base = tmp_path_factory.mktemp("real")
    return {name: realdata.write_dataset(golden("real_%s.npz" % name)[0], str(base / name))
            for name in ("wn18", "fb15k")}


def sha1(*arrays):
    m = hashlib.sha1()
    for a in arrays:
        m.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return m.hexdigest()


def _model(z, test_dl):
    from openke.module.model import TransE, TransH
    cls = TransE if str(z["model"]) == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=int(z["dim"]),
              p_norm=int(z["p_norm"]), norm_flag=True)
    sd = {"ent_embeddings.weight": torch.from_numpy(z["ent_embeddings"]),
          "rel_embeddings.weight": torch.from_numpy(z["rel_embeddings"])}
    if "norm_vector" in z.files:
        sd["norm_vector.weight"] = torch.from_numpy(z["norm_vector"])
    kge.load_state_dict(sd, strict=False)
    return kge


def _entity_rows(tester, side, q):
    """[n][E] GPU scores in entity order (pt_score_rows, the rows k_rank_rows reads) of queries q (h, t, r)."""
    from openke import _native
    kge = tester.model
    dev = kge.ent_embeddings.weight.device
    E = kge.ent_embeddings.weight.shape[0]
    qh, qt, qr = (torch.from_numpy(np.ascontiguousarray(q[:, c], dtype=np.int64)).to(dev) for c in range(3))
    rows = torch.empty((len(q), E), dtype=torch.float32, device=dev)
    desc = kge.native_desc()
    _native.check(tester.lib.pt_score_rows(ctypes.byref(desc), side, _native.ptr(qh), _native.ptr(qt),
                                           _native.ptr(qr), len(q), _native.ptr(rows), _native.stream()))
    return rows


def _tie_counts(tester, q):
    """Per query and side, the candidates whose GPU score lies within TIE_REL of the truth's: the comparisons a
    last-ulp difference from the reference's torch arithmetic can flip."""
    out = []
    for side, col in ((0, 0), (1, 1)):   # head queries rank the true head, tail queries the true tail
        ties = np.zeros(len(q), dtype=np.int64)
        for s in range(0, len(q), 1024):
            rows = _entity_rows(tester, side, q[s:s + 1024])
            truth = torch.from_numpy(q[s:s + 1024, col].astype(np.int64)).to(rows.device)
            s0 = rows.gather(1, truth[:, None])
            band = TIE_REL * torch.clamp(s0.abs(), min=1.0)
            ties[s:s + 1024] = ((rows - s0).abs() <= band).sum(dim=1).cpu().numpy() - 1
        out.append(ties)
    return out


@pytest.mark.parametrize("path", golden("reallp_*.npz"), ids=lambda p: p.split("/")[-1])
def test_gpu_link_prediction_matches_reference_counts(path, real_dirs):
    from openke import _native
    from openke.config import Tester
    from openke.data import TestDataLoader
    z = load(path)
    tc = bool(int(z["type_constrain"]))
    test_dl = TestDataLoader(real_dirs[str(z["dataset"])], "link")
    tester = Tester(model=_model(z, test_dl), data_loader=test_dl, use_gpu=True)
    res = tester.run_link_prediction(type_constrain=tc)
    q = z["queries"].astype(np.int64)
    h, t, r = test_dl.eval_triples()
    np.testing.assert_array_equal(np.stack([h, t, r], 1), q)   # the reference's sorted test order (Reader.h:311)
    got = list(tester.last_ranks) + (list(tester.last_tc_ranks) if tc else [])
    want = z["ranks"].astype(np.int64)
    assert len(got) == want.shape[0]
    ties = _tie_counts(tester, q)
    differ = 0
    for k, g in enumerate(got):
        d = np.abs(np.asarray(g, dtype=np.int64) - want[k])
        tie = ties[(k % 4) // 2]
        bad = np.nonzero(d > tie)[0]
        assert len(bad) == 0, (str(z["rank_names"][k]), bad[:10], g[bad[:10]], want[k][bad[:10]], tie[bad[:10]])
        differ += int((d != 0).sum())
    n = q.shape[0]
    assert differ <= max(2, 0.01 * len(got) * n), differ
    met = np.zeros(10, dtype=np.float32)
    rk = [np.ascontiguousarray(x, dtype=np.int64) for x in tester.last_ranks]
    _native.check(tester.lib.pt_lp_metrics(*(x.ctypes.data for x in rk), n, met.ctypes.data))
    if differ == 0:   # the same counts through the reference's float accumulation: the same metrics, bit for bit
        np.testing.assert_array_equal(np.array(tester.last_metrics, dtype=np.float32),
                                      z["metrics"].astype(np.float32))
        np.testing.assert_array_equal(np.array(res, dtype=np.float32), z["metrics_tc" if tc else "metrics"]
                                      .astype(np.float32))
    else:
        np.testing.assert_array_equal(np.array(tester.last_metrics, dtype=np.float32), met[:5])
        np.testing.assert_allclose(np.array(tester.last_metrics, dtype=np.float32), z["metrics"].astype(np.float32),
                                   rtol=2e-3)


@pytest.mark.parametrize("path", golden("reallp_*.npz"), ids=lambda p: p.split("/")[-1])
def test_gpu_scores_match_reference_vectors(path, real_dirs):
    """GPU score rows against the reference's own torch score vectors (candidate order [truth, 0..E-1 \\ truth],
    Test.h:37-107) within 1e-5 and 1e-6 relative, and against the oracle for 64 more queries."""
    from openke.config import Tester
    from openke.data import TestDataLoader
    z = load(path)
    test_dl = TestDataLoader(real_dirs[str(z["dataset"])], "link")
    tester = Tester(model=_model(z, test_dl), data_loader=test_dl, use_gpu=True)
    q = z["queries"].astype(np.int64)
    E = test_dl.get_ent_tot()
    for i, k in enumerate(z["vec_queries"]):
        for side, ref in ((0, z["vec_head"][i]), (1, z["vec_tail"][i])):
            row = _entity_rows(tester, side, q[k:k + 1])[0].cpu().numpy()
            cand = oracle.candidates(E, int(q[k, side]))
            np.testing.assert_allclose(row[cand], ref, rtol=1e-6, atol=SCORE_ATOL)
            assert float(np.abs(row[cand] - ref).max()) <= TIE_REL / 2 * max(1.0, float(np.abs(ref).max()))
    ent, rel = z["ent_embeddings"], z["rel_embeddings"]
    nv = z["norm_vector"] if "norm_vector" in z.files else None
    pick = np.linspace(0, len(q) - 1, 64).astype(np.int64)
    for side, mode in ((0, "head_batch"), (1, "tail_batch")):
        rows = _entity_rows(tester, side, q[pick]).cpu().numpy()
        for i, k in enumerate(pick):
            h, t, r = (np.array([x], dtype=np.int64) for x in q[k])
            allc = np.arange(E, dtype=np.int64)
            want = oracle.score(str(z["model"]), int(z["p_norm"]), True, mode, ent, rel, nv,
                                allc if side == 0 else h, allc if side == 1 else t, r)
            np.testing.assert_allclose(rows[i], want, rtol=1e-6, atol=SCORE_ATOL)


@pytest.mark.parametrize("path", golden("realsampler_*.npz"), ids=lambda p: p.split("/")[-1])
def test_gpu_sampler_matches_reference_at_wn18_scale(path, real_dirs):
    from openke.data import TrainDataLoader
    z = load(path)
    dl = TrainDataLoader(in_path=real_dirs["wn18"], batch_size=int(z["batch_size"]), threads=8,
                         sampling_mode="normal", bern_flag=int(z["bern"]), filter_flag=int(z["filter"]),
                         neg_ent=int(z["neg_ent"]), neg_rel=0, random_seed=int(z["seed"]))
    for c, want in enumerate(z["digests"]):
        d = dl.sampling()
        if c == 0:
            np.testing.assert_array_equal(np.stack([d["batch_h"], d["batch_t"], d["batch_r"]]),
                                          z["first"].astype(np.int64))
        assert sha1(d["batch_h"], d["batch_t"], d["batch_r"]) == str(want), "call %d" % c


@pytest.mark.parametrize("path_name", ["fused", "part", "twopass"])
def test_gpu_counting_sort_sampler_matches_reference_at_wn18_scale(path_name, real_dirs):
    """C2's in-kernel samplers (k_sample_part / k_sample_csr) on WN18 with bs 2,000 x 25 negatives, bern + filter:
    the positives and every (positive, negative) record of the first call equal the reference's batch; bucket starts
    and destinations consistent with it. The all-LDS k_sample_sort holds a bucket count per entity: at E = 40,943
    its plan does not fit the LDS, and asking for it is refused with an error, not run."""
    from openke._native import NativeError
    from test_gpu_sampling import PATHS, _check_batches, _Ctx
    z = load(golden("realsampler_w5.npz")[0])
    bs, neg = int(z["batch_size"]), int(z["neg_ent"])
    h, t, r = (z["first"][i].astype(np.int64) for i in range(3))
    ph, pt_, pr = h[:bs], t[:bs], r[:bs]
    nh = h[bs:].reshape(neg, bs).T
    nt = t[bs:].reshape(neg, bs).T
    tail = (nt != pt_[:, None]).astype(np.int64)   # corrupt_head replaces the tail (Corrupt.h:9-56)
    assert ((tail == 1) | (nh != ph[:, None])).all()
    ent = np.where(tail == 1, nt, nh)
    want = [(np.stack([ph, pr, pt_], 1), ((ent << 1) | tail).astype(np.int32).reshape(-1))]
    ctx = _Ctx(int(z["seed"]), path=real_dirs["wn18"])
    try:
        if path_name == "fused":
            with pytest.raises(NativeError, match="does not fit LDS"):
                ctx.sample(bs, neg, int(z["bern"]), int(z["filter"]), 1, PATHS[path_name])
            return
        got = ctx.sample(bs, neg, int(z["bern"]), int(z["filter"]), 1, PATHS[path_name])
        _check_batches(got, want, ctx.E, bs, neg)
    finally:
        ctx.close()


def test_gpu_dropin_universes_match_reference_at_wn18_scale(real_dirs):
    """The reference's per-universe protocol through the drop-in loader on WN18 (Parallel_Universe_Config.py:
    157-161, 209-226): remaps, sizes, batch size and the SHA-1 of two GPU-sampled universe batches for seeds 4-11."""
    from openke.data import TrainDataLoader
    z = load(golden("realuniverses_wn18.npz")[0])
    tc_range = tuple(int(x) for x in z["tc_range"])
    bal_range = tuple(float(x) for x in z["bal_range"])
    dl = TrainDataLoader(in_path=real_dirs["wn18"], nbatches=20, threads=8, sampling_mode="normal", bern_flag=0,
                         filter_flag=0, neg_ent=1, neg_rel=0, random_seed=4)
    for s in z["seeds"]:
        s = int(s)
        dl.lib.setRandomSeed(s)
        dl.lib.randReset()
        random.seed(s)
        tc = random.randrange(*tc_range)
        bal = round(random.uniform(*bal_range), 2)
        assert (tc, bal) == (int(z["s%d_tc" % s]), float(z["s%d_balance" % s]))
        dl.compile_universe_dataset(tc, bal)
        em, rm = dl.get_universe_mappings()
        np.testing.assert_array_equal(em, z["s%d_ent_remap" % s])
        np.testing.assert_array_equal(rm, z["s%d_rel_remap" % s])
        assert dl.batch_size == int(z["s%d_batch_size" % s])
        dl.swap_helpers()
        for c, want in enumerate(z["s%d_digests" % s]):
            d = dl.sampling()
            assert sha1(d["batch_h"], d["batch_t"], d["batch_r"]) == str(want), "seed %d call %d" % (s, c)
        dl.reset_universe()
