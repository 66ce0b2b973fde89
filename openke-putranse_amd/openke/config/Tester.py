# coding:utf-8
"""Link-prediction tester (mirror of openke/config/Tester.py:17-93).

run_link_prediction() returns the reference's (mrr, mr, hit10, hit3, hit1) (filtered). Scores for a
block of test queries come from one HIP launch (pt_score_rows: every entity as the missing side, row in
entity order), ranks from one more (pt_rank_rows: raw and filtered counts of testHead/testTail,
Test.h:118-359, with the known-triple filter as a per-query partner list), the metrics with the
reference's float accumulation (Test.h:398-454). Only the ranks leave the GPU."""
import ctypes

import numpy as np
import torch

from .. import _native


def device_type_lists(lib, dev):
    """The head / tail type lists of importTypeFiles (Reader.h:344-396) as device tensors
    [(lef, rig, list)] per side. The reference dereferences them unloaded when its Python asks for
    type_constrain without calling importTypeFiles (Test.h:127-130); here they are loaded on first use."""
    if lib.pt_legacy_types(0, None, None, None) < 0:
        lib.importTypeFiles()
    out = []
    for side in (0, 1):
        n = lib.pt_legacy_types(side, None, None, None)
        if n < 0:
            raise RuntimeError("type_constrain: no readable type_constrain.txt in the input folder")
        R = lib.getRelationTotal()
        lef, rig = np.zeros(R, dtype=np.int64), np.zeros(R, dtype=np.int64)
        lst = np.zeros(max(n, 1), dtype=np.int64)
        lib.pt_legacy_types(side, lef.ctypes.data, rig.ctypes.data, lst.ctypes.data)
        out.append(tuple(torch.from_numpy(x).to(dev) for x in (lef, rig, lst)))
    return out


def rank_types(lib, rows, E, d_row, d_truth, d_repl, d_rel, types, d_off, d_part, n):
    """Type-constrained raw / filtered counts on the GPU (pt_rank_types)."""
    dev = rows.device
    raw = torch.zeros(n, dtype=torch.int64, device=dev)
    filt = torch.zeros(n, dtype=torch.int64, device=dev)
    lef, rig, lst = types
    _native.check(lib.pt_rank_types(_native.ptr(rows), E, _native.ptr(d_row), _native.ptr(d_truth), _native.ptr(d_repl),
                                    _native.ptr(d_rel), _native.ptr(lef), _native.ptr(rig), _native.ptr(lst),
                                    _native.ptr(d_off), _native.ptr(d_part), n, _native.ptr(raw), _native.ptr(filt),
                                    _native.stream()))
    return raw.cpu().numpy(), filt.cpu().numpy()


class Tester(object):

    def __init__(self, model=None, data_loader=None, use_gpu=True):
        self.lib = _native.lib()
        self.model = model
        self.data_loader = data_loader
        self.use_gpu = use_gpu
        if self.model is not None:
            _native.require_gpu()
            self.model.cuda()

    def set_model(self, model):
        self.model = model

    def set_data_loader(self, data_loader):
        self.data_loader = data_loader

    def set_use_gpu(self, use_gpu):
        self.use_gpu = use_gpu
        if self.model is not None:
            self.model.cuda()

    def to_var(self, x, use_gpu):
        return torch.from_numpy(x).cuda()

    def test_one_step(self, data):
        return self.model.predict(data)

    # ---------------------------------------------------------------- batched evaluation --------
    def _query_scores(self, side, h, t, r):
        """[n][entTotal] candidate-order scores for queries (h, t, r) on the GPU (side 0 = head)."""
        kge = self.model
        dev = kge.ent_embeddings.weight.device
        E = kge.ent_embeddings.weight.shape[0]
        out = torch.empty((len(h), E), dtype=torch.float32, device=dev)
        qh, qt, qr = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (h, t, r))
        desc = kge.native_desc()
        _native.check(self.lib.pt_score_queries(ctypes.byref(desc), side, _native.ptr(qh), _native.ptr(qt),
                                                _native.ptr(qr), len(h), _native.ptr(out), _native.stream()))
        return out

    def _rank_all(self, h, t, r, E, types=None):
        """raw/filtered head and tail ranks for every test query (chunked to bound memory); with `types`
        (device_type_lists) also the type-constrained ones (ranks[4:8])."""
        n = len(h)
        known = self.lib.pt_legacy_known()
        if not known:
            raise RuntimeError("no test data imported (TestDataLoader.read() imports it)")
        kge = self.model
        dev = kge.ent_embeddings.weight.device
        desc = kge.native_desc()
        ranks = [np.zeros(n, dtype=np.int64) for _ in range(8 if types else 4)]
        chunk = max(1, min(65535, (1 << 30) // (4 * max(E, 1))))
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            m = e - s
            hh, tt, rr = (np.ascontiguousarray(x[s:e], dtype=np.int64) for x in (h, t, r))
            qh, qt, qr = (torch.from_numpy(x).to(dev) for x in (hh, tt, rr))
            rows = torch.empty((m, E), dtype=torch.float32, device=dev)
            row_of = torch.arange(m, dtype=torch.int64, device=dev)
            for side, anchor, truth in ((0, tt, qh), (1, hh, qt)):
                _native.check(self.lib.pt_score_rows(ctypes.byref(desc), side, _native.ptr(qh), _native.ptr(qt),
                                                     _native.ptr(qr), m, _native.ptr(rows), _native.stream()))
                off = np.zeros(m + 1, dtype=np.int64)
                _native.check(self.lib.pt_known_partners(known, side, m, anchor.ctypes.data, rr.ctypes.data,
                                                         off.ctypes.data, None))
                part = np.zeros(max(int(off[-1]), 1), dtype=np.int64)
                _native.check(self.lib.pt_known_partners(known, side, m, anchor.ctypes.data, rr.ctypes.data,
                                                         off.ctypes.data, part.ctypes.data))
                d_off, d_part = torch.from_numpy(off).to(dev), torch.from_numpy(part).to(dev)
                raw = torch.zeros(m, dtype=torch.int64, device=dev)
                filt = torch.zeros(m, dtype=torch.int64, device=dev)
                _native.check(self.lib.pt_rank_rows(_native.ptr(rows), E, _native.ptr(row_of), _native.ptr(truth),
                                                    None, _native.ptr(d_off), _native.ptr(d_part), m, _native.ptr(raw),
                                                    _native.ptr(filt), _native.stream()))
                ranks[2 * side][s:e] = raw.cpu().numpy()
                ranks[2 * side + 1][s:e] = filt.cpu().numpy()
                if types:
                    rc, fc = rank_types(self.lib, rows, E, row_of, truth, None, qr, types[side], d_off, d_part, m)
                    ranks[4 + 2 * side][s:e] = rc
                    ranks[5 + 2 * side][s:e] = fc
        return ranks

    def run_link_prediction(self, type_constrain=False):
        """Tester.py:70-93: filtered (mrr, mr, hit10, hit3, hit1); with type_constrain the constrained
        ones, as the reference's getters return them (Test.h:533-567)."""
        self.data_loader.set_sampling_mode('link')
        h, t, r = self.data_loader.eval_triples()
        E = self.data_loader.get_ent_tot()
        types = device_type_lists(self.lib, self.model.ent_embeddings.weight.device) if type_constrain else None
        ranks = self._rank_all(h, t, r, E, types)
        rh, fh, rt, ft = ranks[:4]
        met = np.zeros(10, dtype=np.float32)
        _native.check(self.lib.pt_lp_metrics(rh.ctypes.data, fh.ctypes.data, rt.ctypes.data, ft.ctypes.data, len(h),
                                             met.ctypes.data))
        self.last_ranks = (rh, fh, rt, ft)
        self.last_raw_metrics = tuple(float(x) for x in met[5:])
        self.last_metrics = tuple(float(x) for x in met[:5])
        if type_constrain:
            self.last_tc_ranks = tuple(ranks[4:])
            _native.check(self.lib.pt_lp_metrics(*(x.ctypes.data for x in ranks[4:]), len(h), met.ctypes.data))
        mrr, mr, hit10, hit3, hit1 = (float(x) for x in met[:5])
        print(hit10)
        return mrr, mr, hit10, hit3, hit1

    # ---------------------------------------------------------------- triple classification -----
    # Tester.py:95-191. Scores come from the model's GPU predict (one launch per batch); the threshold
    # search and accuracy are the reference's sorted sweeps, restated vectorized over the same
    # np.argsort order (identical results, ties included).
    def determine_classification_cross_table_values(self, res, threshold):
        pred = res[:, 1] < threshold
        ans = res[:, 0] == 1
        print("True Positives :{}".format(int(np.sum(pred & ans))))
        print("True Negatives :{}".format(int(np.sum(~pred & ~ans))))
        print("False Positives :{}".format(int(np.sum(pred & ~ans))))
        print("False Negatives :{}".format(int(np.sum(~pred & ans))))

    def get_best_threshlod(self, score, ans):
        res = np.concatenate([ans.reshape(-1, 1), score.reshape(-1, 1)], axis=-1)
        order = np.argsort(score)
        res = res[order]
        total_all = float(len(score))
        total_true = np.sum(ans)
        total_false = total_all - total_true
        if len(res) == 0:
            return None, 0.0
        # res_current at index i = (2 * #positives in res[:i+1] + total_false - i - 1) / total_all; the
        # loop keeps the first strict maximum above 0
        cur = np.cumsum(res[:, 0] == 1).astype(np.float64)
        idx = np.arange(len(res), dtype=np.float64)
        val = (2 * cur + total_false - idx - 1) / total_all
        best = int(np.argmax(val))
        if not val[best] > 0.0:
            return None, 0.0
        return res[best, 1], float(val[best])

    def run_triple_classification(self, threshlod=None, data_iterator=None):
        (getattr(self, "lib", None) or _native.lib()).initTest()
        score = []
        ans = []
        if data_iterator is None:
            self.data_loader.set_sampling_mode('classification')
            data_iterator = self.data_loader
        for pos_ins, neg_ins in data_iterator:
            res_pos = self.test_one_step(pos_ins)
            ans = ans + [1 for _ in range(len(res_pos))]
            score.append(res_pos)
            res_neg = self.test_one_step(neg_ins)
            ans = ans + [0 for _ in range(len(res_neg))]
            score.append(res_neg)
        score = np.concatenate(score, axis=-1)
        ans = np.array(ans)
        if threshlod is None:
            threshlod, _ = self.get_best_threshlod(score, ans)
        res = np.concatenate([ans.reshape(-1, 1), score.reshape(-1, 1)], axis=-1)
        order = np.argsort(score)
        res = res[order]
        total_all = float(len(score))
        total_true = np.sum(ans)
        total_false = total_all - total_true
        # special handling of parallel-universe scores that are all +inf (Tester.py:166-173)
        if threshlod == float("inf") and len(score[score == float("inf")]) == len(score):
            if total_true == 0:
                return 1.0, threshlod
            if total_false == 0:
                return 0.0, threshlod
            elif total_false == total_true:
                return 0.5, threshlod
        acc = 0
        if threshlod is None and len(res):
            # no threshold with a positive accuracy (e.g. a single negative score): the reference's loop fails
            # at its first comparison `score > threshlod` (Tester.py:183-184); fail the same way
            raise TypeError("'>' not supported between instances of 'numpy.float64' and 'NoneType' "
                            "(get_best_threshlod found no threshold, Tester.py:120-139)")
        above = np.nonzero(res[:, 1] > threshlod)[0] if threshlod is not None else np.zeros(0, dtype=np.int64)
        if len(above):
            index = int(above[0])
            total_current = float(np.sum(res[:index, 0] == 1))
            acc = (2 * total_current + total_false - index) / total_all
        if threshlod is not None:
            self.determine_classification_cross_table_values(res, threshlod)
        return acc, threshlod
