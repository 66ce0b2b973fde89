"""Counting-sort sampling paths of the large-neg step, batch by batch, against the oracle.

The large-neg training step (C2) reads its batch in a counting-sort layout: positives, one record per
(positive, negative) slot, and every slot's destination row inside its corrupted entity's bucket. Three
kernels produce it (capi.cpp enqueue_sample_chunk):
  * PT_PATH_FUSED    k_sample_sort: one workgroup per call, everything in LDS;
  * PT_PATH_PART     k_sample_part + k_resolve: `parts` workgroups per call, global bucket reservation,
                     the last part scans;
  * PT_PATH_TWO_PASS k_sample_csr + k_scan_counts: global atomics, separate scan.
Each is compared with the oracle's restatement of sampling()/getBatch() (Base.cpp:185-310,
Corrupt.h:9-105; the oracle is pinned to the reference's own sampler goldens in test_oracle.py):
positives and negative records bit-exact, bucket starts equal to the prefix sums of the oracle's
corrupted-entity counts, and the destinations a permutation of the slots that puts every slot inside
its own entity's bucket. (The order inside a bucket comes from atomics and may differ between paths;
the apply pass only sums a bucket.)

Shapes follow the reference's step: the k-th negative of positive b is slot b*neg + k (the reference's
(k+1)*bs + b, Base.cpp:216-232). Cases cover >= 96 calls per chunk, slot counts that are neither a
multiple of the 1024/512-thread strides nor divided by neg (bs 200, neg 13: the second lock-step slot,
the incremental (b, k) carry), neg > 1024 (db == 0), filter = 0 and bern = 0, and bs*neg >= 65536 (the
split sampler's unpacked 32-bit counts).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from conftest import KG_SMALL

pytestmark = pytest.mark.gpu

THREADS = 8


class _Ctx:
    def __init__(self, seed, dim=4, path=KG_SMALL):
        from openke import _native
        _native.require_gpu()
        self.n = _native
        self.L = _native.lib()
        self.g = ctypes.c_void_p()
        _native.check(self.L.pt_graph_load(path.encode(), ctypes.byref(self.g)))
        self.E = int(self.L.pt_graph_ent_total(self.g))
        R = int(self.L.pt_graph_rel_total(self.g))
        self.st0 = oracle.GlibcRand(seed).rand_reset(THREADS)
        self.s = ctypes.c_void_p()
        _native.check(self.L.pt_sampler_create(self.g, THREADS, self.st0.ctypes.data, ctypes.byref(self.s)))
        dev = torch.device("cuda", 0)
        self.ent = torch.zeros(self.E, dim, device=dev)
        self.rel = torch.zeros(R, dim, device=dev)
        d = _native.ModelDesc()
        d.model, d.p_norm, d.norm_flag, d.opt, d.lr, d.margin = 0, 1, 1, 0, 0.1, 1.0
        d.ent_total, d.rel_total, d.dim = self.E, R, dim
        d.ent, d.rel = self.ent.data_ptr(), self.rel.data_ptr()
        self.t = ctypes.c_void_p()
        _native.check(self.L.pt_trainer_create(ctypes.byref(d), ctypes.byref(self.t)))

    def sample(self, bs, neg, bern, filt, calls, path):
        slots = bs * neg
        pos = np.zeros((calls, bs, 3), np.int32)
        rec = np.zeros((calls, slots), np.int32)
        dst = np.zeros((calls, slots), np.int32)
        start = np.zeros((calls, self.E + 1), np.int32)
        self.n.check(self.L.pt_trainer_sample_csr(self.t, self.s, bs, neg, bern, filt, calls, path,
                                                  pos.ctypes.data, rec.ctypes.data, dst.ctypes.data,
                                                  start.ctypes.data, self.n.stream()))
        return pos, rec, dst, start

    def close(self):
        self.L.pt_trainer_free(self.t)
        self.L.pt_sampler_free(self.s)
        self.L.pt_graph_free(self.g)


def _oracle_batches(seed, bs, neg, bern, filt, calls):
    kg = oracle.KG.load(KG_SMALL)
    st = oracle.GlibcRand(seed).rand_reset(THREADS)
    out = []
    for _ in range(calls):
        h, t, r, _, side = kg.sample(st, THREADS, bs, neg, bern, filt, sides=True)
        ph, pt_, pr = h[:bs], t[:bs], r[:bs]
        nh = h[bs:].reshape(neg, bs).T   # [b][k]
        nt = t[bs:].reshape(neg, bs).T
        tail = side[bs:].reshape(neg, bs).T.astype(np.int64)   # 1: the tail was replaced (corrupt_head)
        ent = np.where(tail == 1, nt, nh)
        out.append((np.stack([ph, pr, pt_], 1), ((ent << 1) | tail).astype(np.int32).reshape(-1)))
    return out, kg.ent_total


def _check_batches(got, want, E, bs, neg):
    pos, rec, dst, start = got
    slots = bs * neg
    for c, (wpos, wrec) in enumerate(want):
        np.testing.assert_array_equal(pos[c], wpos.astype(np.int32), err_msg="call %d positives" % c)
        np.testing.assert_array_equal(rec[c], wrec, err_msg="call %d negative records" % c)
        ent = wrec >> 1
        counts = np.bincount(ent, minlength=E)
        np.testing.assert_array_equal(start[c], np.concatenate([[0], np.cumsum(counts)]).astype(np.int32),
                                      err_msg="call %d bucket starts" % c)
        d = dst[c]
        assert np.array_equal(np.sort(d), np.arange(slots)), "call %d destinations are not a permutation" % c
        assert (d >= start[c][ent]).all() and (d < start[c][ent + 1]).all(), "call %d slot outside its bucket" % c


PATHS = {"fused": 1, "part": 2, "twopass": 0}

CASES = [
    # bs, neg, bern, filter, calls, seed
    (200, 13, 1, 1, 100, 5),     # 2600 slots/call: not a multiple of the strides, neg does not divide 1024
    (200, 13, 0, 0, 100, 7),     # no filter, no bern
    (37, 1100, 1, 1, 4, 9),      # neg > 1024: db == 0 in the slot walk
    (3000, 25, 1, 1, 3, 11),     # 75,000 slots per call: the split sampler's 32-bit counts
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "bs%d-neg%d-bern%d-filter%d-calls%d" % c[:5])
@pytest.mark.parametrize("path", sorted(PATHS))
def test_sampling_path_matches_oracle(case, path):
    bs, neg, bern, filt, calls, seed = case
    want, E = _oracle_batches(seed, bs, neg, bern, filt, calls)
    ctx = _Ctx(seed)
    try:
        got = ctx.sample(bs, neg, bern, filt, calls, PATHS[path])
        _check_batches(got, want, E, bs, neg)
        # the streams advanced past exactly `calls` calls: the next call equals the oracle's next
        kg = oracle.KG.load(KG_SMALL)
        st = oracle.GlibcRand(seed).rand_reset(THREADS)
        for _ in range(calls):
            kg.sample(st, THREADS, bs, neg, bern, filt)
        nxt = ctx.sample(bs, neg, bern, filt, 1, PATHS[path])
        h, t, r, _ = kg.sample(st, THREADS, bs, neg, bern, filt)
        np.testing.assert_array_equal(nxt[0][0][:, 0], h[:bs].astype(np.int32))
        np.testing.assert_array_equal(nxt[0][0][:, 2], t[:bs].astype(np.int32))
    finally:
        ctx.close()


@pytest.mark.parametrize("parts", [2, 3, 7, 64, 200])
def test_split_sampler_any_part_count(parts):
    """k_sample_part with part counts from 2 to one positive per part (pt_trainer_set_sampling): identical
    batches."""
    bs, neg, bern, filt, calls, seed = 200, 13, 1, 1, 5, 13
    want, E = _oracle_batches(seed, bs, neg, bern, filt, calls)
    ctx = _Ctx(seed)
    ctx.n.check(ctx.L.pt_trainer_set_sampling(ctx.t, -1, parts))
    try:
        _check_batches(ctx.sample(bs, neg, bern, filt, calls, PATHS["part"]), want, E, bs, neg)
    finally:
        ctx.close()


@pytest.mark.parametrize("head", [1, 2, 7])
@pytest.mark.parametrize("case", [(200, 13, 1, 1, 20, 17), (3000, 25, 1, 1, 6, 19), (200, 13, 0, 0, 9, 23)],
                         ids=lambda c: "bs%d-neg%d-bern%d-filter%d-calls%d" % c[:5])
def test_split_sampler_two_launches(case, head):
    """A chunk sampled by two k_sample_part launches side by side (pt_trainer_set_sample_split: the first `head`
    calls on the caller's stream, the rest on the trainer's side stream, the streams advanced after both):
    the same batches as the oracle, and the streams end past exactly `calls` calls."""
    bs, neg, bern, filt, calls, seed = case
    want, E = _oracle_batches(seed, bs, neg, bern, filt, calls)
    ctx = _Ctx(seed)
    ctx.n.check(ctx.L.pt_trainer_set_sample_split(ctx.t, head))
    try:
        _check_batches(ctx.sample(bs, neg, bern, filt, calls, PATHS["part"]), want, E, bs, neg)
        kg = oracle.KG.load(KG_SMALL)
        st = oracle.GlibcRand(seed).rand_reset(THREADS)
        for _ in range(calls):
            kg.sample(st, THREADS, bs, neg, bern, filt)
        nxt = ctx.sample(bs, neg, bern, filt, 1, PATHS["part"])
        h, t, r, _ = kg.sample(st, THREADS, bs, neg, bern, filt)
        np.testing.assert_array_equal(nxt[0][0][:, 0], h[:bs].astype(np.int32))
        np.testing.assert_array_equal(nxt[0][0][:, 2], t[:bs].astype(np.int32))
    finally:
        ctx.close()


def test_split_sampling_run_equals_single_launch():
    """pt_trainer_run over a 20-step chunk (the driver's shape) with the chunk's sampling split in two launches
    (opt-in) and in one: the same per-step losses and tables, up to the float-atomic order of the step."""
    from openke import _native
    L = _native.lib()
    res = []
    for head in (0, 2):
        ctx = _Ctx(29, dim=24)
        try:
            g = torch.Generator().manual_seed(3)
            ctx.ent.copy_(((torch.rand(ctx.ent.shape, generator=g) - 0.5) * 0.2).cuda())
            ctx.rel.copy_(((torch.rand(ctx.rel.shape, generator=g) - 0.5) * 0.2).cuda())
            _native.check(L.pt_trainer_set_sample_split(ctx.t, head))
            losses = torch.zeros(20, device="cuda")
            _native.check(L.pt_trainer_run(ctx.t, ctx.s, 100, 25, 1, 1, 20, _native.ptr(losses), _native.stream()))
            torch.cuda.synchronize()
            assert L.pt_trainer_last_path(ctx.t) == PATHS["part"]
            res.append((losses.cpu(), ctx.ent.cpu(), ctx.rel.cpu()))
        finally:
            ctx.close()
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
