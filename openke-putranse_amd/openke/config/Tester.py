# coding:utf-8
"""Link-prediction tester (mirror of openke/config/Tester.py:17-93).

run_link_prediction() returns the reference's (mrr, mr, hit10, hit3, hit1) (filtered). Candidate
scores for a whole block of test queries come from one HIP launch (pt_score_queries) in exactly the
candidate order of getHeadBatch/getTailBatch; ranks use the reference's rules (Test.h:118-359) on host
threads, and the metrics its float accumulation (Test.h:398-454)."""
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
        ranks = [np.zeros(n, dtype=np.int64) for _ in range(4)]
        chunk = max(1, min(65535, (256 << 20) // (4 * max(E, 1))))
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            hh, tt, rr = h[s:e].copy(), t[s:e].copy(), r[s:e].copy()
            for side in (0, 1):
                con = self._query_scores(side, hh, tt, rr).cpu().numpy()
                raw = ranks[2 * side][s:e]
                filt = ranks[2 * side + 1][s:e]
                rawb = np.zeros(e - s, dtype=np.int64)
                filtb = np.zeros(e - s, dtype=np.int64)
                _native.check(self.lib.pt_rank_queries(known, E, hh.ctypes.data, tt.ctypes.data, rr.ctypes.data,
                                                       e - s, side, con.ctypes.data, rawb.ctypes.data,
                                                       filtb.ctypes.data, 0))
                raw[:] = rawb
                filt[:] = filtb
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
