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

    def _rank_all(self, h, t, r, E):
        """raw/filtered head and tail ranks for every test query (chunked to bound memory)."""
        n = len(h)
        known = self.lib.pt_legacy_known()
        if not known:
            raise RuntimeError("no test data imported (TestDataLoader.read() imports it)")
        kge = self.model
        dev = kge.ent_embeddings.weight.device
        desc = kge.native_desc()
        ranks = [np.zeros(n, dtype=np.int64) for _ in range(4)]
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
        return ranks

    def run_link_prediction(self, type_constrain=False):
        if type_constrain:
            raise NotImplementedError("type-constrained ranking is outside the accelerated path")
        self.data_loader.set_sampling_mode('link')
        h, t, r = self.data_loader.eval_triples()
        E = self.data_loader.get_ent_tot()
        rh, fh, rt, ft = self._rank_all(h, t, r, E)
        met = np.zeros(10, dtype=np.float32)
        _native.check(self.lib.pt_lp_metrics(rh.ctypes.data, fh.ctypes.data, rt.ctypes.data, ft.ctypes.data, len(h),
                                             met.ctypes.data))
        self.last_ranks = (rh, fh, rt, ft)
        self.last_raw_metrics = tuple(float(x) for x in met[5:])
        mrr, mr, hit10, hit3, hit1 = (float(x) for x in met[:5])
        print(hit10)
        return mrr, mr, hit10, hit3, hit1

    def run_triple_classification(self, threshlod=None, data_iterator=None):
        raise NotImplementedError("triple classification is outside the accelerated path")
