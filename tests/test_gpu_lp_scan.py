"""The TransE link-prediction scan rounds every pair's score the same way on each of its paths (pytest -m gpu).

pt_lp_min_scores (global energy estimation, Parallel_Universe_Config.py:446-642) scores every local entity of a
universe against each of its (key, universe) pairs and MINs the score into the key's row. k_lp_scan_t's waves
take a universe's pairs two at a time (one pass over the row feeds both sums) and the remainder one at a time.
Until round 6 the compiler's fp contraction fused some of those loops' products into fmas and not others, so the
same pair's score could differ by an ulp between the two paths. Every rounding is now explicit (x-hat = x * inv
from the sum8 tree of fma squares; y = fma(sg, x-hat, b); |y| added, or fma(y, y, a); dim d into partial d mod 8),
and a pair's score must not depend on the path: the rows of one call over all pairs equal, bit for bit, those of
one call per pair (a universe with one pair takes the one-pair path). The rows of both are checked against the
oracle's scores elsewhere (test_gpu_pu, test_gpu_configs C4, test_gpu_realscale)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _rows(n, unis, pairs, p, nf, E, n_keys):
    L = n.lib()
    dev = torch.device("cuda")
    rows = torch.full((n_keys, E), float("inf"), device=dev)
    tup = torch.full((n_keys,), float("inf"), device=dev)
    lp_us = []
    for u in unis:
        U = n.LpUniverse()
        U.ent, U.rel, U.normv = u["ent"].data_ptr(), u["rel"].data_ptr(), None
        U.ent_total, U.rel_total, U.dim = u["ent"].shape[0], u["rel"].shape[0], u["ent"].shape[1]
        U.d_ent_remap = u["remap"].data_ptr()
        lp_us.append(U)
    arr_u = (n.LpUniverse * len(lp_us))(*lp_us)
    arr = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 5)
    arr_p = arr.ctypes.data_as(ctypes.POINTER(n.LpPair))
    n.check(L.pt_lp_min_scores(arr_u, len(lp_us), 0, p, nf, arr_p, len(arr), E, n.ptr(rows), n.ptr(tup), n.stream()))
    torch.cuda.synchronize()
    return rows.cpu(), tup.cpu()


def _diff(a, b):
    ai, bi = a.view(torch.int32), b.view(torch.int32)
    bad = ai != bi
    if not bad.any():
        return None
    ulp = (ai.long() - bi.long()).abs()[bad & torch.isfinite(a) & torch.isfinite(b)]
    return "%d of %d cells differ, ulps max %d; e.g. %s vs %s" % (
        int(bad.sum()), bad.numel(), int(ulp.max()) if len(ulp) else -1, a[bad][:4].tolist(), b[bad][:4].tolist())


@pytest.mark.parametrize("p,nf", [(1, 1), (2, 1), (1, 0), (2, 0)])
@pytest.mark.parametrize("D", [20, 50, 64, 100, 200])
def test_scan_paths_round_alike(D, p, nf):
    from openke import _native as n
    g = torch.Generator().manual_seed(D * 7 + p + 3 * nf)
    rng = np.random.default_rng(D + 11 * p + nf)
    dev = torch.device("cuda")
    E, n_keys = 2000, 29
    Eu, Ru = int(rng.integers(100, 700)), 5   # not a multiple of the 64-row tile: a partial last tile
    uni = {"ent": (torch.rand(Eu, D, generator=g) * 2 - 1).to(dev),
           "rel": (torch.rand(Ru, D, generator=g) * 2 - 1).to(dev),
           "remap": torch.from_numpy(np.sort(rng.choice(E, Eu, replace=False)).astype(np.int64)).to(dev)}
    # 29 keys, one pair each: the 8 waves take pairs (w, w + 8) through the two-pair pass, the rest one at a time
    pairs = [(k, 0, int(rng.integers(Eu)), int(rng.integers(Ru)), k % 2) for k in range(n_keys)]
    together, t_tog = _rows(n, [uni], pairs, p, nf, E, n_keys)
    alone = torch.full((n_keys, E), float("inf"))
    t_alone = torch.full((n_keys,), float("inf"))
    for pr in pairs:   # one pair per call: the one-pair path
        r1, t1 = _rows(n, [uni], [pr], p, nf, E, n_keys)
        alone = torch.minimum(alone, r1)
        t_alone = torch.minimum(t_alone, t1)
    assert torch.isfinite(together).sum() == n_keys * Eu
    d = _diff(together, alone)
    assert d is None, "D %d p %d nf %d: %s" % (D, p, nf, d)
    assert torch.equal(t_tog.view(torch.int32), t_alone.view(torch.int32))
