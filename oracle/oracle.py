"""ctypes wrapper of the CPU oracle (oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker. The product path (openke-putranse_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

i64p = ctypes.POINTER(ctypes.c_int64)
u64p = ctypes.POINTER(ctypes.c_uint64)
f32p = ctypes.POINTER(ctypes.c_float)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.okg_load.restype = ctypes.c_void_p
        L.okg_load.argtypes = [ctypes.c_char_p]
        L.okg_free.argtypes = [ctypes.c_void_p]
        for f in ("okg_ent_total", "okg_rel_total", "okg_train_total"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.okg_get_train.argtypes = [ctypes.c_void_p, i64p, i64p, i64p]
        L.okg_left_mean.restype = ctypes.c_float
        L.okg_left_mean.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.okg_right_mean.restype = ctypes.c_float
        L.okg_right_mean.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.orand_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.orand_next.restype = ctypes.c_int32
        L.orand_next.argtypes = [ctypes.c_void_p]
        L.oracle_rand_reset.argtypes = [ctypes.c_void_p, ctypes.c_int64, u64p]
        L.oracle_sampling.argtypes = [ctypes.c_void_p, u64p] + [ctypes.c_int64] * 5 + [i64p, i64p, i64p, f32p]
        L.oracle_sampling_sides.argtypes = [ctypes.c_void_p, u64p] + [ctypes.c_int64] * 5 + \
            [i64p, i64p, i64p, f32p, ctypes.c_void_p]
        L.oracle_sampling_ex.argtypes = [ctypes.c_void_p, u64p] + [ctypes.c_int64] * 7 + [i64p, i64p, i64p, f32p]
        L.oracle_universe.restype = ctypes.c_void_p
        L.oracle_universe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, i64p, i64p]
        L.oracle_train_step.restype = ctypes.c_float
        L.oracle_train_step.argtypes = ([ctypes.c_int] * 4 + [ctypes.c_float] * 2 + [ctypes.c_int64] * 3 +
                                        [f32p] * 6 + [i64p] * 3 + [ctypes.c_int64] * 2)
        L.oracle_score.argtypes = ([ctypes.c_int] * 4 + [ctypes.c_int64] + [f32p] * 3 + [i64p] * 3 +
                                   [ctypes.c_int64, f32p])
        L.oracle_sort_test.argtypes = [ctypes.c_int64, i64p, i64p, i64p]
        L.oracle_link_prediction.argtypes = ([ctypes.c_int64] + [i64p] * 3 + [ctypes.c_int64] + [i64p] * 3 +
                                             [ctypes.c_int64] + [f32p] * 2 + [i64p] * 4 + [f32p])
        L.oracle_rank_constrained.argtypes = ([ctypes.c_int64] + [i64p] * 3 + [ctypes.c_int64] + [i64p] * 3 +
                                              [ctypes.c_int64] + [f32p] * 2 + [i64p] * 6 + [i64p] * 4 + [f32p])
        L.oracle_metrics_from_ranks.argtypes = [ctypes.c_int64, i64p, i64p, f32p]
        L.oracle_grad_mass.restype = ctypes.c_float
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.oracle_grad_mass.argtypes = ([ctypes.c_int] * 3 + [ctypes.c_float] + [ctypes.c_int64] * 3 + [f32p] * 3 +
                                       [i64p] * 3 + [ctypes.c_int64] * 2 + [f32p] * 3 + [i32p] * 2)
        L.oracle_train_step_mt.restype = ctypes.c_float
        L.oracle_train_step_mt.argtypes = ([ctypes.c_int] * 4 + [ctypes.c_float] * 2 + [ctypes.c_int64] * 3 +
                                           [f32p] * 6 + [i64p] * 3 + [ctypes.c_int64] * 3)
        L.oracle_train_loop_mt.restype = ctypes.c_int64
        L.oracle_train_loop_mt.argtypes = ([ctypes.c_void_p, u64p] + [ctypes.c_int64] * 5 + [ctypes.c_int] * 4 +
                                           [ctypes.c_float] * 2 + [ctypes.c_int64] + [f32p] * 6 +
                                           [ctypes.c_int64] * 2 + [f32p])
        L.oracle_train_loop.restype = ctypes.c_int64
        L.oracle_train_loop.argtypes = ([ctypes.c_void_p, u64p] + [ctypes.c_int64] * 5 + [ctypes.c_int] * 4 +
                                        [ctypes.c_float] * 2 + [ctypes.c_int64] + [f32p] * 6 + [ctypes.c_int64])
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


class GlibcRand:
    """glibc srand()/rand() restated with private state (orand_t is 31 int32 + 2 ints)."""

    def __init__(self, seed):
        self.buf = ctypes.create_string_buffer(31 * 4 + 8)
        lib().orand_seed(self.buf, ctypes.c_uint32(seed & 0xFFFFFFFF))

    def next(self):
        return lib().orand_next(self.buf)

    def rand_reset(self, threads):
        st = np.zeros(threads, dtype=np.uint64)
        lib().oracle_rand_reset(self.buf, threads, _p(st, u64p))
        return st


class KG:
    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load(cls, path):
        if not path.endswith(os.sep):
            path += os.sep
        h = lib().okg_load(path.encode())
        if not h:
            raise FileNotFoundError(path)
        return cls(h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().okg_free(self.h)
            self.h = None

    @property
    def ent_total(self):
        return lib().okg_ent_total(self.h)

    @property
    def rel_total(self):
        return lib().okg_rel_total(self.h)

    @property
    def train_total(self):
        return lib().okg_train_total(self.h)

    def train(self):
        n = self.train_total
        h, t, r = (np.zeros(n, dtype=np.int64) for _ in range(3))
        lib().okg_get_train(self.h, _p(h, i64p), _p(t, i64p), _p(r, i64p))
        return h, t, r

    def means(self):
        R = self.rel_total
        lm = np.array([lib().okg_left_mean(self.h, i) for i in range(R)], dtype=np.float32)
        rm = np.array([lib().okg_right_mean(self.h, i) for i in range(R)], dtype=np.float32)
        return lm, rm

    def sample(self, states, threads, bs, neg, bern, filt, sides=False):
        """One sampling() call (Base.cpp:266-310). sides=True also returns int8[seq]: 1 where the tail
        was replaced (corrupt_head), 0 where the head was (positions [0, bs) stay 0)."""
        seq = bs * (1 + neg)
        h, t, r = (np.zeros(seq, dtype=np.int64) for _ in range(3))
        y = np.zeros(seq, dtype=np.float32)
        side = np.zeros(seq, dtype=np.int8)
        lib().oracle_sampling_sides(self.h, _p(states, u64p), threads, bs, neg, bern, filt, _p(h, i64p),
                                    _p(t, i64p), _p(r, i64p), _p(y, f32p), side.ctypes.data if sides else None)
        return (h, t, r, y, side) if sides else (h, t, r, y)

    def sample_ex(self, states, threads, bs, neg, neg_rel, mode, bern, filt):
        """sampling() with its mode (0 normal, -1 sampling_head, 1 sampling_tail) and neg_rel relation
        corruptions (Base.cpp:185-264); seq = bs * (1 + neg + neg_rel)."""
        seq = bs * (1 + neg + neg_rel)
        h, t, r = (np.zeros(seq, dtype=np.int64) for _ in range(3))
        y = np.zeros(seq, dtype=np.float32)
        lib().oracle_sampling_ex(self.h, _p(states, u64p), threads, bs, neg, neg_rel, mode, bern, filt,
                                 _p(h, i64p), _p(t, i64p), _p(r, i64p), _p(y, f32p))
        return h, t, r, y

    def universe(self, rng, tc, balance):
        em = np.full(max(self.ent_total, 1), -1, dtype=np.int64)
        rm = np.full(max(self.rel_total, 1), -1, dtype=np.int64)
        u = lib().oracle_universe(self.h, rng.buf, tc, ctypes.c_float(balance), _p(em, i64p), _p(rm, i64p))
        ug = KG(u)
        return ug, em[:ug.ent_total].copy(), rm[:ug.rel_total].copy()


MODELS = {"TransE": 0, "TransH": 1}
OPTS = {"sgd": 0, "adagrad": 1}


def train_step(model, p, norm_flag, opt, lr, margin, ent, rel, normv, accs, h, t, r, bs, neg):
    """In-place step on float32 C-contiguous tables; accs = (ent_acc, rel_acc, norm_acc)."""
    E, D = ent.shape
    R = rel.shape[0]
    dummy = np.zeros(1, dtype=np.float32)
    nv = normv if normv is not None else dummy
    ea, ra, na = accs
    ea = ea if ea is not None else dummy
    ra = ra if ra is not None else dummy
    na = na if na is not None else dummy
    h = np.ascontiguousarray(h, dtype=np.int64)
    t = np.ascontiguousarray(t, dtype=np.int64)
    r = np.ascontiguousarray(r, dtype=np.int64)
    return lib().oracle_train_step(MODELS[model], p, int(norm_flag), OPTS[opt], lr, margin, E, R, D,
                                   _p(ent, f32p), _p(rel, f32p), _p(nv, f32p), _p(ea, f32p), _p(ra, f32p),
                                   _p(na, f32p), _p(h, i64p), _p(t, i64p), _p(r, i64p), bs, neg)


def grad_mass(model, p, norm_flag, margin, ent, rel, normv, h, t, r, bs, neg):
    """Test infrastructure (helpers.kappa_bound): at the given tables and batch (nothing updated), per table
    {"ent", "rel", "norm"} a dict with the step's gradient "g" (summed in the reference's order), the sum of its
    contributions' magnitudes "mass", its absolute-value evaluation "abs" (the forward-error scale of any
    evaluation order), per row the contribution count "n" and the near-tie flag "tie" (oracle_grad_mass)."""
    E, D = ent.shape
    R = rel.shape[0]
    rows = E + R * (2 if model == "TransH" else 1)
    gs = np.zeros((rows, D), dtype=np.float32)
    gm = np.zeros((rows, D), dtype=np.float32)
    ga = np.zeros((rows, D), dtype=np.float32)
    cnt = np.zeros(rows, dtype=np.int32)
    tie = np.zeros(rows, dtype=np.int32)
    nv = normv if normv is not None else np.zeros(1, dtype=np.float32)
    h, t, r = (np.ascontiguousarray(x, dtype=np.int64) for x in (h, t, r))
    i32p = ctypes.POINTER(ctypes.c_int32)
    lib().oracle_grad_mass(MODELS[model], p, int(norm_flag), margin, E, R, D, _p(np.ascontiguousarray(ent), f32p),
                           _p(np.ascontiguousarray(rel), f32p), _p(np.ascontiguousarray(nv), f32p), _p(h, i64p),
                           _p(t, i64p), _p(r, i64p), bs, neg, _p(gs, f32p), _p(gm, f32p), _p(ga, f32p),
                           _p(cnt, i32p), _p(tie, i32p))
    spans = {"ent": slice(0, E), "rel": slice(E, E + R)}
    if model == "TransH":
        spans["norm"] = slice(E + R, rows)
    return {k: {"g": gs[v], "mass": gm[v], "abs": ga[v], "n": cnt[v], "tie": tie[v].astype(bool)}
            for k, v in spans.items()}


def score(model, p, norm_flag, mode, ent, rel, normv, h, t, r):
    n = max(len(h), len(t), len(r))
    h = np.ascontiguousarray(np.broadcast_to(h, (n,)), dtype=np.int64)
    t = np.ascontiguousarray(np.broadcast_to(t, (n,)), dtype=np.int64)
    r = np.ascontiguousarray(np.broadcast_to(r, (n,)), dtype=np.int64)
    out = np.zeros(n, dtype=np.float32)
    nv = normv if normv is not None else np.zeros(1, dtype=np.float32)
    lib().oracle_score(MODELS[model], p, int(norm_flag), {"normal": 0, "head_batch": 1, "tail_batch": 2}[mode],
                       ent.shape[1], _p(ent, f32p), _p(rel, f32p), _p(nv, f32p), _p(h, i64p), _p(t, i64p),
                       _p(r, i64p), n, _p(out, f32p))
    return out


def read_triples(path):
    a = np.loadtxt(path, dtype=np.int64, ndmin=2)
    return a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()


def sort_test(h, t, r):
    h, t, r = h.copy(), t.copy(), r.copy()
    lib().oracle_sort_test(len(h), _p(h, i64p), _p(t, i64p), _p(r, i64p))
    return h, t, r


def candidates(E, truth):
    """getHeadBatch/getTailBatch candidate order: [truth, 0..E-1 without truth] (Test.h:37-107)."""
    c = np.empty(E, dtype=np.int64)
    c[0] = truth
    rest = np.arange(E, dtype=np.int64)
    c[1:] = rest[rest != truth]
    return c


def link_prediction(E, all_triples, test, con_head, con_tail):
    ah, at, ar = (np.ascontiguousarray(x, dtype=np.int64) for x in all_triples)
    th, tt, tr = (np.ascontiguousarray(x, dtype=np.int64) for x in test)
    n = len(th)
    rh, fh, rt, ft = (np.zeros(n, dtype=np.int64) for _ in range(4))
    met = np.zeros(5, dtype=np.float32)
    ch = np.ascontiguousarray(con_head, dtype=np.float32)
    ct = np.ascontiguousarray(con_tail, dtype=np.float32)
    lib().oracle_link_prediction(E, _p(ah, i64p), _p(at, i64p), _p(ar, i64p), len(ah), _p(th, i64p),
                                 _p(tt, i64p), _p(tr, i64p), n, _p(ch, f32p), _p(ct, f32p), _p(rh, i64p),
                                 _p(fh, i64p), _p(rt, i64p), _p(ft, i64p), _p(met, f32p))
    return met, (rh, fh, rt, ft)


def metrics_from_ranks(frank_head, frank_tail):
    """Filtered {MRR, MR, Hits@10, Hits@3, Hits@1} of given per-query ranks (Test.h float accumulation)."""
    fh = np.ascontiguousarray(frank_head, dtype=np.int64)
    ft = np.ascontiguousarray(frank_tail, dtype=np.int64)
    met = np.zeros(5, dtype=np.float32)
    lib().oracle_metrics_from_ranks(len(fh), _p(fh, i64p), _p(ft, i64p), _p(met, f32p))
    return met


def train_step_mt(model, p, norm_flag, opt, lr, margin, ent, rel, normv, accs, h, t, r, bs, neg, workers):
    """train_step on `workers` threads (bit-identical to train_step)."""
    E, D = ent.shape
    R = rel.shape[0]
    dummy = np.zeros(1, dtype=np.float32)
    nv = normv if normv is not None else dummy
    ea, ra, na = (a if a is not None else dummy for a in accs)
    h, t, r = (np.ascontiguousarray(x, dtype=np.int64) for x in (h, t, r))
    return lib().oracle_train_step_mt(MODELS[model], p, int(norm_flag), OPTS[opt], lr, margin, E, R, D,
                                      _p(ent, f32p), _p(rel, f32p), _p(nv, f32p), _p(ea, f32p), _p(ra, f32p),
                                      _p(na, f32p), _p(h, i64p), _p(t, i64p), _p(r, i64p), bs, neg, workers)


def read_types(path, rel_total):
    """importTypeFiles (Reader.h:352-396): `type_constrain.txt` = a count, then per relation two lines
    `r n e_1 .. e_n` (heads, then tails); relationTotal records read, each list sorted in place.
    Returns (head_lef, head_rig, head_type, tail_lef, tail_rig, tail_type) with lef/rig per relation."""
    with open(path) as f:
        tok = f.read().split()
    pos = 1
    lef = [np.zeros(rel_total, dtype=np.int64) for _ in range(2)]
    rig = [np.zeros(rel_total, dtype=np.int64) for _ in range(2)]
    types = [[], []]
    for _ in range(rel_total):
        for side in range(2):
            r, n = int(tok[pos]), int(tok[pos + 1])
            pos += 2
            vals = sorted(int(x) for x in tok[pos:pos + n])
            pos += n
            lef[side][r] = len(types[side])
            types[side].extend(vals)
            rig[side][r] = len(types[side])
    ht, tt = (np.array(x if x else [0], dtype=np.int64) for x in types)
    return lef[0], rig[0], ht, lef[1], rig[1], tt


def rank_constrained(E, all_triples, test, con_head, con_tail, types):
    """Type-constrained ranks and metrics (Test.h:127-502), restated literally (see oracle.c)."""
    ah, at, ar = (np.ascontiguousarray(x, dtype=np.int64) for x in all_triples)
    th, tt, tr = (np.ascontiguousarray(x, dtype=np.int64) for x in test)
    n = len(th)
    rh, fh, rt, ft = (np.zeros(n, dtype=np.int64) for _ in range(4))
    met = np.zeros(5, dtype=np.float32)
    ch = np.ascontiguousarray(con_head, dtype=np.float32)
    ct = np.ascontiguousarray(con_tail, dtype=np.float32)
    hl, hr, hty, tl, trr, tty = (np.ascontiguousarray(x, dtype=np.int64) for x in types)
    lib().oracle_rank_constrained(E, _p(ah, i64p), _p(at, i64p), _p(ar, i64p), len(ah), _p(th, i64p),
                                  _p(tt, i64p), _p(tr, i64p), n, _p(ch, f32p), _p(ct, f32p), _p(hl, i64p),
                                  _p(hr, i64p), _p(hty, i64p), _p(tl, i64p), _p(trr, i64p), _p(tty, i64p),
                                  _p(rh, i64p), _p(fh, i64p), _p(rt, i64p), _p(ft, i64p), _p(met, f32p))
    return met, (rh, fh, rt, ft)


def train_loop(kg, states, threads, bs, neg, bern, filt, model, p, norm_flag, opt, lr, margin, tables, accs, steps,
               workers=1, losses=None):
    """`steps` sampling() calls + steps; workers > 1 runs the sampler slices and the step phases on that many
    threads (bit-identical). Returns the slots processed; losses (float32 array) receives each step's loss."""
    ent, rel, normv = tables
    ea, ra, na = accs
    dummy = np.zeros(1, dtype=np.float32)
    nv = normv if normv is not None else dummy
    ea = ea if ea is not None else dummy
    ra = ra if ra is not None else dummy
    na = na if na is not None else dummy
    lp = _p(losses, f32p) if losses is not None else None
    return lib().oracle_train_loop_mt(kg.h, _p(states, u64p), threads, bs, neg, bern, filt, MODELS[model], p,
                                      int(norm_flag), OPTS[opt], lr, margin, ent.shape[1], _p(ent, f32p),
                                      _p(rel, f32p), _p(nv, f32p), _p(ea, f32p), _p(ra, f32p), _p(na, f32p), steps,
                                      workers, lp)
