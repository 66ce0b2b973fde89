"""The two TransE link-prediction scan kernels give bit-identical key rows (pytest -m gpu).

pt_lp_min_scores (global energy estimation, Parallel_Universe_Config.py:446-642) scores every local entity of a
universe against each of its (key, universe) pairs and MINs the score into the key's row. Round 6 added
k_lp_scan_v (entity row in registers, the pairs' base rows in LDS, two dims per v_pk_fma_f32) beside
k_lp_scan_t (entity rows in LDS, base rows through scalar loads). Both keep the score's expression and its
summation order (8 interleaved partial sums, dim d into partial d mod 8), so the rows must be equal bit for bit,
for p 1 and 2, with and without normalization, at every register tier (dims up to 32 / 64 / 128 / 200), for a
universe whose dim is below its launch's tier (zero-padded dims), and where k_lp_scan_v does not apply (dims
not a multiple of 4, or above 200) - there both settings take k_lp_scan_t. The rows of both are checked
against the oracle's scores elsewhere (test_gpu_pu, test_gpu_configs C4, test_gpu_realscale)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible HIP device"


def _rows(L, n, unis, pairs, model, p, nf, E, n_keys, kernel):
    dev = torch.device("cuda")
    rows = torch.full((n_keys, E), float("inf"), device=dev)
    tup = torch.full((n_keys,), float("inf"), device=dev)
    lp_us = []
    for u in unis:
        U = n.LpUniverse()
        U.ent, U.rel = u["ent"].data_ptr(), u["rel"].data_ptr()
        U.normv = u["nv"].data_ptr() if u["nv"] is not None else None
        U.ent_total, U.rel_total, U.dim = u["ent"].shape[0], u["rel"].shape[0], u["ent"].shape[1]
        U.d_ent_remap = u["remap"].data_ptr()
        lp_us.append(U)
    arr_u = (n.LpUniverse * len(lp_us))(*lp_us)
    arr = np.ascontiguousarray(pairs, dtype=np.int32)
    arr_p = arr.ctypes.data_as(__import__("ctypes").POINTER(n.LpPair))
    old = L.pt_get_lp_scan_kernel()
    n.check(L.pt_set_lp_scan_kernel(kernel))
    try:
        n.check(L.pt_lp_min_scores(arr_u, len(lp_us), model, p, nf, arr_p, len(arr), E, n.ptr(rows), n.ptr(tup),
                                   n.stream()))
        torch.cuda.synchronize()
    finally:
        n.check(L.pt_set_lp_scan_kernel(old))
    return rows.cpu(), tup.cpu()


def _case(dims, E, n_keys, seed, model=0):
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    dev = torch.device("cuda")
    unis, pairs = [], []
    for k, D in enumerate(dims):
        Eu = int(rng.integers(40, 700))   # not a multiple of the 256-entity workgroup: partial waves and lanes
        Ru = int(rng.integers(2, 9))
        ent = (torch.rand(Eu, D, generator=g) * 2 - 1).to(dev)
        rel = (torch.rand(Ru, D, generator=g) * 2 - 1).to(dev)
        nv = (torch.rand(Ru, D, generator=g) * 2 - 1).to(dev) if model == 1 else None
        remap = torch.from_numpy(np.sort(rng.choice(E, Eu, replace=False)).astype(np.int64)).to(dev)
        unis.append({"ent": ent, "rel": rel, "nv": nv, "remap": remap})
        for key in range(n_keys):
            if rng.random() < 0.7:   # the universes holding the key's anchor and relation
                pairs.append((key, k, int(rng.integers(Eu)), int(rng.integers(Ru)), key % 2))
    return unis, np.array(pairs, dtype=np.int32).reshape(-1, 5)


def _diff(a, b):
    ai, bi = a.view(torch.int32), b.view(torch.int32)
    bad = ai != bi
    if not bad.any():
        return None
    fin = torch.isfinite(a) & torch.isfinite(b)
    ulp = (ai.long() - bi.long()).abs()[bad & fin]
    return "%d of %d cells differ (%d where one is inf), ulps max %d median %d; e.g. %s vs %s" % (
        int(bad.sum()), bad.numel(), int((bad & ~fin).sum()), int(ulp.max()) if len(ulp) else -1,
        int(ulp.median()) if len(ulp) else -1, a[bad][:4].tolist(), b[bad][:4].tolist())


@pytest.mark.parametrize("p,nf", [(1, 1), (2, 0)])
@pytest.mark.parametrize("D", [20, 64, 100, 152, 200])
def test_scan_kernels_bit_identical_per_dim(D, p, nf):
    from openke import _native as n
    L = n.lib()
    E, n_keys = 2000, 11
    unis, pairs = _case([D], E, n_keys, seed=D + p)
    r1, t1 = _rows(L, n, unis, pairs, 0, p, nf, E, n_keys, 1)
    for k in (0, 2, 3):
        r0, t0 = _rows(L, n, unis, pairs, 0, p, nf, E, n_keys, k)
        d = _diff(r0, r1)
        assert d is None, "kernel %d, D %d p %d nf %d: %s" % (k, D, p, nf, d)


@pytest.mark.parametrize("p,nf", [(1, 1), (2, 1), (1, 0), (2, 0)])
def test_scan_kernels_bit_identical(p, nf):
    from openke import _native as n
    L = n.lib()
    E, n_keys = 3000, 37
    # tiers: 20 -> 32, 64, 100 -> 128, 200 (p = 1); 152 and 196 share the 200 tier's launch with 200, below it
    # (zero-padded dims); 50 and 204 (the same row shape as 200, a launch of its own): k_lp_scan_t under both
    # settings, as every dim above 128 at p = 2
    unis, pairs = _case([20, 64, 100, 152, 196, 200, 200, 50, 204], E, n_keys, seed=7 + p + 3 * nf)
    r1, t1 = _rows(L, n, unis, pairs, 0, p, nf, E, n_keys, 1)
    for k in (0, 2, 3):
        r0, t0 = _rows(L, n, unis, pairs, 0, p, nf, E, n_keys, k)
        assert torch.isfinite(r0).any()
        d = _diff(r0, r1)
        assert d is None, "kernel %d: %s" % (k, d)
        assert torch.equal(t0.view(torch.int32), t1.view(torch.int32))


def test_scan_kernel_switch_validates():
    from openke import _native as n
    L = n.lib()
    assert L.pt_get_lp_scan_kernel() == 0   # the tiled kernel is the default
    assert L.pt_set_lp_scan_kernel(4) != 0
    assert L.pt_get_lp_scan_kernel() == 0
