"""CPU-side checks of the product library: it loads, exports every symbol include/putranse.h
declares, and its host-side parts (graph ingest, universe construction, ranking, metrics) match the
oracle / the reference's golden vectors. No GPU compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from conftest import KG_SMALL, REPO
from helpers import golden, load
from openke import _native


def header_symbols():
    src = open(os.path.join(REPO, "include", "putranse.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\([^;]*\)\s*;", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "sizeof")))


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    names = header_symbols()
    assert len(names) > 60, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert not [n for n in names if n not in _native.SIGNATURES], [n for n in names if n not in _native.SIGNATURES]
    assert L.pt_version() == 1


def _graph(path):
    h = ctypes.c_void_p()
    _native.check(_native.lib().pt_graph_load(path.encode(), ctypes.byref(h)))
    return h


def test_graph_ingest_matches_oracle():
    L = _native.lib()
    g = _graph(KG_SMALL)
    kg = oracle.KG.load(KG_SMALL)
    assert L.pt_graph_ent_total(g) == kg.ent_total
    assert L.pt_graph_rel_total(g) == kg.rel_total
    n = L.pt_graph_train_total(g)
    assert n == kg.train_total
    h, t, r = (np.zeros(n, dtype=np.int64) for _ in range(3))
    _native.check(L.pt_graph_triples(g, h.ctypes.data, t.ctypes.data, r.ctypes.data))
    oh, ot, orr = kg.train()
    np.testing.assert_array_equal(h, oh)
    np.testing.assert_array_equal(t, ot)
    np.testing.assert_array_equal(r, orr)
    L.pt_graph_free(g)


def test_graph_load_errors_are_reported_not_fatal():
    L = _native.lib()
    h = ctypes.c_void_p()
    rc = L.pt_graph_load(b"/nonexistent/dir/", ctypes.byref(h))
    assert rc == 2
    assert b"cannot open" in L.pt_last_error()


@pytest.mark.parametrize("path", golden("universes_*.npz"), ids=lambda p: p.split("/")[-1])
def test_universe_construction_matches_reference(path):
    z = load(path)
    L = _native.lib()
    g = _graph(KG_SMALL)
    seed0, n = int(z["seed0"]), int(z["n_univ"])
    seeds = np.array([seed0 + u for u in range(n)], dtype=np.int64)
    tcs = np.array([int(z["u%d_tc" % u]) for u in range(n)], dtype=np.int64)
    bals = np.array([float(z["u%d_balance" % u]) for u in range(n)], dtype=np.float32)
    outs = (ctypes.c_void_p * n)()
    _native.check(L.pt_universe_build_many(g, n, seeds.ctypes.data, 8, tcs.ctypes.data, bals.ctypes.data, 4, outs))
    for u in range(n):
        U = ctypes.c_void_p(outs[u])
        assert L.pt_universe_train_total(U) == int(z["u%d_train_total" % u])
        E, R = L.pt_universe_ent_total(U), L.pt_universe_rel_total(U)
        em, rm = np.zeros(E, dtype=np.int64), np.zeros(R, dtype=np.int64)
        _native.check(L.pt_universe_remaps(U, em.ctypes.data, rm.ctypes.data))
        np.testing.assert_array_equal(em, z["u%d_ent_remap" % u])
        np.testing.assert_array_equal(rm, z["u%d_rel_remap" % u])
        # the universe graph's helper-sorted triples equal the oracle's restatement
        rng = oracle.GlibcRand(seed0 + u)
        st = rng.rand_reset(8)
        seeds_out = np.zeros(8, dtype=np.uint64)
        _native.check(L.pt_universe_seeds(U, seeds_out.ctypes.data))
        np.testing.assert_array_equal(seeds_out, st)
        L.pt_universe_free(U)
    L.pt_graph_free(g)


def test_universe_construction_matches_oracle_on_many_seeds():
    """Bit-exact universes for 40 seeds and a range of sizes/balances on the small KG."""
    L = _native.lib()
    g = _graph(KG_SMALL)
    kg = oracle.KG.load(KG_SMALL)
    for k in range(40):
        tc = 100 + 37 * k
        bal = 0.25 + 0.006 * k
        U = ctypes.c_void_p()
        _native.check(L.pt_universe_build(g, 1000 + k, 8, tc, ctypes.c_float(bal), ctypes.byref(U)))
        rng = oracle.GlibcRand(1000 + k)
        rng.rand_reset(8)
        ug, em, rm = kg.universe(rng, tc, bal)
        assert L.pt_universe_train_total(U) == ug.train_total
        E = L.pt_universe_ent_total(U)
        pem = np.zeros(E, dtype=np.int64)
        _native.check(L.pt_universe_remaps(U, pem.ctypes.data, None))
        np.testing.assert_array_equal(pem, em)
        G = L.pt_universe_graph(U)
        n = L.pt_graph_train_total(G)
        h, t, r = (np.zeros(n, dtype=np.int64) for _ in range(3))
        _native.check(L.pt_graph_triples(G, h.ctypes.data, t.ctypes.data, r.ctypes.data))
        oh, ot, orr = ug.train()
        np.testing.assert_array_equal(h, oh)
        np.testing.assert_array_equal(t, ot)
        np.testing.assert_array_equal(r, orr)
        L.pt_universe_free(U)
    L.pt_graph_free(g)


@pytest.mark.parametrize("path", golden("lp_*.npz"), ids=lambda p: p.split("/")[-1])
def test_ranking_and_metrics_match_reference(path):
    """Host ranking (pt_rank_queries) + float metric accumulation (pt_lp_metrics) on oracle scores
    reproduce the reference's link-prediction numbers."""
    z = load(path)
    L = _native.lib()
    model, p = str(z["model"]), int(z["p_norm"])
    kg = oracle.KG.load(KG_SMALL)
    E = kg.ent_total
    ent, rel = z["ent_embeddings"], z["rel_embeddings"]
    nv = z["norm_vector"] if model == "TransH" else None
    th, tt, tr = oracle.sort_test(*oracle.read_triples(KG_SMALL + "test2id.txt"))
    all_tr = [np.ascontiguousarray(np.concatenate(x)) for x in zip(*(oracle.read_triples(KG_SMALL + f)
                                                                  for f in ("test2id.txt", "train2id.txt",
                                                                            "valid2id.txt")))]
    n = len(th)
    con_h = np.zeros((n, E), dtype=np.float32)
    con_t = np.zeros((n, E), dtype=np.float32)
    for q in range(n):
        con_h[q] = oracle.score(model, p, True, "head_batch", ent, rel, nv, oracle.candidates(E, th[q]), [tt[q]], [tr[q]])
        con_t[q] = oracle.score(model, p, True, "tail_batch", ent, rel, nv, [th[q]], oracle.candidates(E, tt[q]), [tr[q]])
    known = ctypes.c_void_p()
    _native.check(L.pt_known_create(all_tr[0].ctypes.data, all_tr[1].ctypes.data, all_tr[2].ctypes.data,
                                    len(all_tr[0]), ctypes.byref(known)))
    ranks = []
    for side, con in ((0, con_h), (1, con_t)):
        raw, filt = np.zeros(n, dtype=np.int64), np.zeros(n, dtype=np.int64)
        _native.check(L.pt_rank_queries(known, E, th.ctypes.data, tt.ctypes.data, tr.ctypes.data, n, side,
                                        con.ctypes.data, raw.ctypes.data, filt.ctypes.data, 4))
        ranks += [raw, filt]
    _, (orh, ofh, ort, oft) = oracle.link_prediction(E, all_tr, (th, tt, tr), con_h, con_t)
    np.testing.assert_array_equal(ranks[0], orh)
    np.testing.assert_array_equal(ranks[1], ofh)
    np.testing.assert_array_equal(ranks[2], ort)
    np.testing.assert_array_equal(ranks[3], oft)
    met = np.zeros(10, dtype=np.float32)
    _native.check(L.pt_lp_metrics(ranks[0].ctypes.data, ranks[1].ctypes.data, ranks[2].ctypes.data,
                                  ranks[3].ctypes.data, n, met.ctypes.data))
    np.testing.assert_array_equal(met[:5], z["metrics"].astype(np.float32))
    L.pt_known_free(known)


def _reference_best_threshold(score, ans):
    """Literal restatement of the reference's get_best_threshlod loop (Tester.py:120-139)."""
    res = np.concatenate([ans.reshape(-1, 1), score.reshape(-1, 1)], axis=-1)[np.argsort(score)]
    total_all = float(len(score))
    total_false = total_all - np.sum(ans)
    cur, mx, thr = 0.0, 0.0, None
    for index, (a, s) in enumerate(res):
        if a == 1:
            cur += 1.0
        v = (2 * cur + total_false - index - 1) / total_all
        if v > mx:
            mx, thr = v, s
    return thr, mx


def test_best_threshold_matches_reference_loop():
    """Tester.get_best_threshlod (vectorized) equals the reference loop on random and tied scores."""
    from openke.config import Tester
    t = Tester()
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 100, 1000):
        for ties in (False, True):
            score = rng.integers(0, 5, n).astype(np.float32) if ties else rng.standard_normal(n).astype(np.float32)
            ans = rng.integers(0, 2, n)
            assert t.get_best_threshlod(score, ans) == _reference_best_threshold(score, ans)


def test_classification_without_threshold_raises_like_reference():
    """No threshold with a positive accuracy (a lone negative score): the reference's loop raises TypeError
    at `score > None` (Tester.py:183-184); the drop-in raises the same error instead of returning 0."""
    from openke.config import Tester

    class _Scores(Tester):
        def test_one_step(self, data):
            return np.asarray(data, dtype=np.float32)

    t = _Scores()
    assert t.get_best_threshlod(np.array([0.5], np.float32), np.array([0]))[0] is None
    with pytest.raises(TypeError):
        t.run_triple_classification(data_iterator=[([], [0.5])])
    # a usable threshold: the reference's accuracy formula (Tester.py:182-190)
    acc, thr = t.run_triple_classification(data_iterator=[([0.1, 0.2], [0.9, 0.3])])
    assert thr == np.float32(0.2) and acc == 1.0


def test_import_type_files_matches_oracle_reader():
    """importTypeFiles (Reader.h:352-396) in the library's global context: per-relation [lef, rig) and
    the sorted type lists == the oracle's reading of the same type_constrain.txt (host code only)."""
    L = _native.lib()
    L.setInPath(ctypes.create_string_buffer(KG_SMALL.encode(), len(KG_SMALL) * 2))
    L.importTrainFiles()   # sets relationTotal (its device upload is irrelevant here)
    R = L.getRelationTotal()
    L.importTypeFiles()
    want = oracle.read_types(KG_SMALL + "type_constrain.txt", R)
    for side in (0, 1):
        n = L.pt_legacy_types(side, None, None, None)
        assert n >= 0
        lef, rig = np.zeros(R, dtype=np.int64), np.zeros(R, dtype=np.int64)
        lst = np.zeros(max(n, 1), dtype=np.int64)
        assert L.pt_legacy_types(side, lef.ctypes.data, rig.ctypes.data, lst.ctypes.data) == n
        np.testing.assert_array_equal(lef, want[3 * side])
        np.testing.assert_array_equal(rig, want[3 * side + 1])
        np.testing.assert_array_equal(lst[:n], want[3 * side + 2][:n])


def _header_copy(tmp_path, header_text=None):
    """kg_small with a count line prepended to every *2id.txt file (the upstream OpenKE format)."""
    d = tmp_path / "kg_small_header"
    d.mkdir()
    for name in ("entity2id.txt", "relation2id.txt", "train2id.txt", "test2id.txt", "valid2id.txt",
                 "type_constrain.txt"):
        body = open(KG_SMALL + name).read()
        if name == "type_constrain.txt":
            (d / name).write_text(body)
            continue
        head = header_text if header_text is not None and name == "train2id.txt" else "%d\n" % body.count("\n")
        (d / name).write_text(head + body)
    return str(d) + os.sep


def _graph_arrays(L, g):
    n = L.pt_graph_train_total(g)
    arrs = [np.zeros(n, dtype=np.int64) for _ in range(3)]
    _native.check(L.pt_graph_triples(g, *(a.ctypes.data for a in arrs)))
    return (L.pt_graph_ent_total(g), L.pt_graph_rel_total(g)), arrs


def test_count_header_reader_is_opt_in(tmp_path):
    """Opt-in count-header format (pt_set_count_header): a header-prefixed copy of kg_small reads back the
    same graph as the headerless original; the default line-count contract (Reader.h:176-196) rejects it."""
    L = _native.lib()
    hdr = _header_copy(tmp_path)
    assert L.pt_get_count_header() == 0
    g0 = _graph(KG_SMALL)
    want_tot, want = _graph_arrays(L, g0)
    L.pt_graph_free(g0)
    # default: the header line is taken as a record and the ids go out of range -> a reported error
    h = ctypes.c_void_p()
    assert L.pt_graph_load(hdr.encode(), ctypes.byref(h)) == 2
    assert b"count-header" in L.pt_last_error()
    try:
        _native.check(L.pt_set_count_header(1))
        g1 = _graph(hdr)
        got_tot, got = _graph_arrays(L, g1)
        L.pt_graph_free(g1)
        assert got_tot == want_tot
        for a, b in zip(got, want):
            np.testing.assert_array_equal(a, b)
        # and a headerless folder under the header format is a reported error, never a silent misread
        assert L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(h)) == 2
    finally:
        L.pt_set_count_header(0)


def test_count_header_legacy_loaders(tmp_path):
    """The Base.so-compatible importTrainFiles / importTestFiles under the opt-in format: same totals and
    ranking-order test/valid triples as the headerless folder; a malformed header is reported through
    pt_legacy_import_status and leaves the format's error message."""
    L = _native.lib()
    hdr = _header_copy(tmp_path)
    (tmp_path / "bad").mkdir()
    bad = _header_copy(tmp_path / "bad", header_text="three thousand\n")

    def load(path):
        L.setInPath(ctypes.create_string_buffer(path.encode(), len(path) * 2))
        L.importTrainFiles()
        _native.check(L.pt_legacy_import_status())
        L.importTestFiles()
        _native.check(L.pt_legacy_import_status())
        out = [L.getEntityTotal(), L.getRelationTotal(), L.getTrainTotal(), L.getTestTotal(), L.getValidTotal()]
        for valid in (0, 1):
            n = L.pt_legacy_eval_triples(valid, None, None, None)
            arrs = [np.zeros(n, dtype=np.int64) for _ in range(3)]
            L.pt_legacy_eval_triples(valid, *(a.ctypes.data for a in arrs))
            out.append(np.stack(arrs))
        return out

    want = load(KG_SMALL)
    try:
        L.pt_set_count_header(1)
        got = load(hdr)
        assert got[:5] == want[:5] and want[:5] == [500, 7, 3000, 100, 100]
        np.testing.assert_array_equal(got[5], want[5])
        np.testing.assert_array_equal(got[6], want[6])
        L.setInPath(ctypes.create_string_buffer(bad.encode(), len(bad) * 2))
        L.importTrainFiles()
        assert L.pt_legacy_import_status() == 2
        assert b"not a record count" in L.pt_last_error()
    finally:
        L.pt_set_count_header(0)
        load(KG_SMALL)   # leave the global context as other tests expect it


def test_test_loader_inherits_count_header(tmp_path):
    """A default TestDataLoader after TrainDataLoader(count_header=True) reads with the train loader's format
    (it does not switch the process back to the line-count reader, which would re-read train2id.txt and fail)."""
    from openke.data import TestDataLoader, TrainDataLoader
    L = _native.lib()
    hdr = _header_copy(tmp_path)
    try:
        tr = TrainDataLoader(in_path=hdr, nbatches=10, threads=8, count_header=True)
        te = TestDataLoader(tr.in_path, "link")
        assert te.count_header is True and L.pt_get_count_header() == 1
        assert (te.entTotal, te.relTotal, L.getTrainTotal(), L.getTestTotal()) == (500, 7, 3000, 100)
        # an explicit choice still wins
        assert TestDataLoader(tr.in_path, "link", count_header=True).count_header is True
    finally:
        L.pt_set_count_header(0)
        L.setInPath(ctypes.create_string_buffer(KG_SMALL.encode(), len(KG_SMALL) * 2))
        L.importTrainFiles()
        L.importTestFiles()


@pytest.mark.parametrize("san", ["address", "thread"])
def test_host_sanitizers(san):
    """the host side under ASan + UBSan and under TSan (make san: the reader, universe construction
    single and pt_universe_build_many on 8 threads, host ranking on 8 workers, the Base.so-compatible context,
    the oracle's multi-threaded loop; each multi-threaded result equal to its one-thread form). Any sanitizer
    report fails the driver (ASan / UBSan abort, TSan exits non-zero)."""
    import subprocess
    pkg = os.path.join(REPO, "openke-putranse_amd")
    if not os.path.exists(os.path.join(pkg, "build", "kernels.hip.o")):
        pytest.skip("product build objects absent (make -C openke-putranse_amd first)")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    r = subprocess.run(["make", "-C", pkg, "san", "SAN=" + san, "-j8"], capture_output=True, text=True, env=env,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "san_driver: ok (0 failed checks)" in out
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]


def test_universe_dims_supported():
    """Every universe dim the fast kernels accept has its row shape compiled into its class kernel (the host's
    shape choice and the kernels' shape_reachable agree; a mismatch would leave a universe untrained, so the
    library reports the dim unsupported instead): TransE and TransH 1-512, TransE float4 rows up to 1,024."""
    from openke import _native
    L = _native.lib()
    for d in range(1, 513):
        assert L.pt_universe_dim_supported(d, _native.PT_TRANSE) == 1, d
        assert L.pt_universe_dim_supported(d, _native.PT_TRANSH) == 1, d
    for d in range(516, 1025, 4):
        assert L.pt_universe_dim_supported(d, _native.PT_TRANSE) == 1, d
    assert L.pt_universe_dim_supported(0, _native.PT_TRANSE) == 0
